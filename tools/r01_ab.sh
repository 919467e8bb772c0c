#!/bin/bash
# A/B: XCD-aware block order vs plain order (same box, interleaved), FETCH_SIZE of both.
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 20 --warmup 3 --cpu-frames 0"
tools/gpu_steps.sh \
"400:ab_pytest:python -m pytest tests/test_gpu_parity.py tests/test_gpu_tiled.py -m gpu -q -x" \
"120:ab_xcd1:python bench.py --cpu-frames 0" \
"120:ab_noxcd1:BMFR_LIB=noxcd python bench.py --cpu-frames 0" \
"120:ab_xcd2:python bench.py --cpu-frames 0" \
"120:ab_noxcd2:BMFR_LIB=noxcd python bench.py --cpu-frames 0" \
"200:ab_fetch_xcd:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/ab_fetch_xcd_d -- $B" \
"200:ab_fetch_noxcd:cd /tmp && BMFR_LIB=noxcd rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/ab_fetch_noxcd_d -- $B"
