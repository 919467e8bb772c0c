#!/bin/bash
# K1/K2 diagnosis: phase stamps of the column-split K1, SQ counters (two passes).
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 3 --warmup 2 --cpu-frames 0"
tools/gpu_steps.sh \
"150:stamps_cols:python tools/k1_phases.py" \
"200:sq1:cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/sq1_d -- $B" \
"200:sq2:cd /tmp && rocprofv3 --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/sq2_d -- $B"
