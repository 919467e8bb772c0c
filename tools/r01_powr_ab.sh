#!/bin/bash
# Tone-map powr A/B: bench and K2 SQ counters with the correctly rounded powr
# (default) and the device library's (--library-powr).
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 3 --warmup 2 --cpu-frames 0 --no-1080p"
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"
tools/gpu_steps.sh \
"200:ab_cr:python bench.py --cpu-frames 0 --no-1080p" \
"200:ab_lib:python bench.py --cpu-frames 0 --no-1080p --library-powr" \
"200:sq_cr:cd /tmp && rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sqcr_d -- $B" \
"200:sq_lib:cd /tmp && rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/sqlib_d -- $B --library-powr"
