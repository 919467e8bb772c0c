#!/bin/bash
# A/B: K2 early taps (default) vs late; K1 occupancy-5 variants.
export TMPDIR=/tmp
tools/gpu_steps.sh \
"400:ab_pytest:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py -m gpu -q -x --timeout 120 --timeout-method thread" \
"120:ab_def1:python bench.py --cpu-frames 0" \
"120:ab_k2late1:BMFR_LIB=k2late python bench.py --cpu-frames 0" \
"120:ab_a5:BMFR_LIB=a5 python bench.py --cpu-frames 0" \
"120:ab_a5b1:BMFR_LIB=a5b1 python bench.py --cpu-frames 0" \
"120:ab_def2:python bench.py --cpu-frames 0" \
"120:ab_k2late2:BMFR_LIB=k2late python bench.py --cpu-frames 0"
