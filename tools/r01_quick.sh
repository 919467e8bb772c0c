#!/bin/bash
# Parity (stage + fused + tiled) then the default bench twice.
export TMPDIR=/tmp
tools/gpu_steps.sh \
"400:q_pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_host.py -m gpu -q -x --timeout 120 --timeout-method thread" \
"120:q_bench1:python bench.py --cpu-frames 0" \
"120:q_bench2:python bench.py --cpu-frames 0" "$@"
