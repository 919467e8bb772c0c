#!/bin/bash
# A/B of K1 variants: parity tests, bench per variant, phase stamps.
export TMPDIR=/tmp
tools/gpu_steps.sh \
"400:ab_pytest:python -m pytest tests -m gpu -q -x" \
"120:ab_bench:python bench.py --cpu-frames 0" \
"120:ab_bench_b4:BMFR_LIB=b4 python bench.py --cpu-frames 0" \
"120:ab_bench_rows:BMFR_FUSED_KERNEL=rows python bench.py --cpu-frames 0" \
"150:ab_stamps:python tools/k1_phases.py"
