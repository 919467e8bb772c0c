#!/bin/bash
# Round-1 evidence: rocprofv3 kernel stats of the default bench, PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ timing) for the traffic / occupancy figures.
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 20 --warmup 3 --cpu-frames 0"
tools/gpu_steps.sh \
"200:p_stats:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p_stats_d -- $B" \
"200:p_fetch:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/p_fetch_d -- $B" \
"200:p_write:cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/p_write_d -- $B" \
"200:p_sq:cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/p_sq_d -- $B"
