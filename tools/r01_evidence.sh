#!/bin/bash
# Round-1 evidence run: GPU parity suite, default bench line, rocprofv3
# kernel stats of the same bench, FETCH_SIZE / WRITE_SIZE passes for K1 traffic.
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 20 --warmup 3 --cpu-frames 0"
tools/gpu_steps.sh \
"600:e_pytest:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
"300:e_bench:python bench.py" \
"200:e_stats:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/e_stats_d -- $B" \
"120:e_fetch:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/e_fetch_d -- $B" \
"120:e_write:cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/e_write_d -- $B"
