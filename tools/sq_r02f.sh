# SQ / TA counter passes (one counter group per run) of K1 and K2 as separate
# launches (tools/k1_frames.py, 12 frames of 4K).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/sq_r02f
mkdir -p $O
P="python3 tools/k1_frames.py 3840 2160 12"
step() { local name=$1; shift; timeout -s KILL 150 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step pmcA rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcA -o p --output-format csv -- $P && \
step pmcB rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmcB -o p --output-format csv -- $P && \
step pmcC rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d $O/pmcC -o p --output-format csv -- $P
