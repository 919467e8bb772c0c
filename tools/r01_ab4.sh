#!/bin/bash
# A/B: K1 at 5 blocks/CU (colour parked in acc_out, LDS 26 KB) vs 4.
export TMPDIR=/tmp
B="python bench.py --cpu-frames 0 --no-1080p --per-frame"
T="python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k fused"
tools/gpu_steps.sh \
"300:d_pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_input_half.py tests/test_gpu_sequence.py -m gpu -q -x --timeout 120 --timeout-method thread" \
"200:d_pytest_w5a:BMFR_LIB=w5a $T" \
"120:d_def1:$B" "120:d_w5a1:BMFR_LIB=w5a $B" "120:d_w5b1:BMFR_LIB=w5b $B" "120:d_w5c1:BMFR_LIB=w5c $B" \
"120:d_parklds1:BMFR_LIB=parklds $B" "120:d_def2:$B" "120:d_w5a2:BMFR_LIB=w5a $B"
