#!/bin/bash
# K2 tile-shape / occupancy A/B (tools/k2_variants.py libraries): bench each.
steps=("300:k2_tests:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py tests/test_gpu_variants.py -q -x --timeout 200 --timeout-method thread")
for v in "$@"; do
    steps+=("120:k2_$v:BMFR_LIB=$v python bench.py --cpu-frames 0 --no-1080p")
done
tools/gpu_steps.sh "${steps[@]}"
