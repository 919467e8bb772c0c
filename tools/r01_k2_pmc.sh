#!/bin/bash
# K2 (k_fused_taa) diagnosis: SQ stall split, memory instruction counts, HBM bytes.
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --steps 3 --warmup 2 --cpu-frames 0 --no-1080p"
tools/gpu_steps.sh \
"120:k2p1:cd /tmp && rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/k2p1 -- $B" \
"120:k2p2:cd /tmp && rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/k2p2 -- $B" \
"120:k2p3:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/k2p3 -- $B" \
"120:k2p4:cd /tmp && rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum --output-format csv -d $R/gpurun_out/k2p4 -- $B" \
"120:k2p5:cd /tmp && rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max --output-format csv -d $R/gpurun_out/k2p5 -- $B"
