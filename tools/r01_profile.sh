#!/bin/bash
# Round-1 GPU evidence run: gpu tests, bench (column-split and row-split K1),
# rocprofv3 kernel stats, PMC passes.
export TMPDIR=/tmp
R=$PWD
tools/gpu_steps.sh \
"500:r01_pytest:python -m pytest tests -m gpu -q" \
"240:r01_bench:python bench.py --cpu-frames 2" \
"120:r01_bench_rows:BMFR_FUSED_KERNEL=rows python bench.py --cpu-frames 0" \
"200:r01_stats:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01_stats_d -- python3 $R/bench.py --steps 20 --warmup 3 --cpu-frames 0" \
"200:r01_fetch:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r01_fetch_d -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-frames 0" \
"200:r01_write:cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r01_write_d -- python3 $R/bench.py --steps 5 --warmup 3 --cpu-frames 0"
