#!/bin/bash
# A/B of K1 variants (same box, interleaved twice).
export TMPDIR=/tmp
tools/gpu_steps.sh \
"120:ab_sep1:python bench.py --cpu-frames 0" \
"120:ab_alias1:BMFR_LIB=alias python bench.py --cpu-frames 0" \
"120:ab_aliaspb1_1:BMFR_LIB=aliaspb1 python bench.py --cpu-frames 0" \
"120:ab_sep2:python bench.py --cpu-frames 0" \
"120:ab_alias2:BMFR_LIB=alias python bench.py --cpu-frames 0" \
"120:ab_aliaspb1_2:BMFR_LIB=aliaspb1 python bench.py --cpu-frames 0"
