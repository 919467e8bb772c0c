#!/bin/bash
# A/B: LDS-only barriers, early phase-3 loads, pivot priority (K1).
export TMPDIR=/tmp
B="python bench.py --cpu-frames 0 --no-1080p"
tools/gpu_steps.sh \
"400:c_pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_input_half.py -m gpu -q -x --timeout 120 --timeout-method thread" \
"120:c_def1:$B" "120:c_syncbar1:BMFR_LIB=syncbar $B" "120:c_p3off1:BMFR_LIB=p3off $B" \
"120:c_prio1:BMFR_LIB=prio1 $B" "120:c_prio2:BMFR_LIB=prio2 $B" \
"120:c_def2:$B" "120:c_syncbar2:BMFR_LIB=syncbar $B"
