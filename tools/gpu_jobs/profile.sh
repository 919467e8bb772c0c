# Profiling evidence on the GPU box (run through gpurun from the repo root):
#   bash tools/gpu_jobs/profile.sh OUT [W H [extra k1_frames/frame_times args]]
# (SKIP_STATS=1: no rocprofv3 stats pass of the default bench command;
# SKIP_SQ=1: no SQ / TA / I-cache passes; SKIP_FRAME=1: no one-launch frame
# passes -- 4K frames run as two launches, whose traffic the K1 / K2 passes give)
# rocprofv3 kernel statistics of the default bench command, then PMC passes
# (one counter group per run, each under its own time limit): SQ / TA /
# I-cache passes and HBM traffic of K1 and K2 as separate launches
# (tools/k1_frames.py: libbmfr per-kernel events split them) and HBM traffic
# of the one-launch frame kernel (tools/frame_times.py).  Output under
# gpurun_out/OUT; summarise with tools/prof_summary.py.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}
W=${2:-3840}; H=${3:-2160}; shift $(( $# < 3 ? $# : 3 )); X="$*"
mkdir -p $O
P="python3 tools/k1_frames.py $W $H 12 $X"
F="python3 tools/frame_times.py $W $H 12 $X"
step() { local name=$1; shift; timeout -s KILL 150 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
{ [ -n "$SKIP_STATS" ] || step stats rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --cpu-frames 0; } && \
{ [ -n "$SKIP_SQ" ] || { step pmcA rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcA -o p --output-format csv -- $P && \
step pmcB rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmcB -o p --output-format csv -- $P && \
step pmcC rocprofv3 --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE -d $O/pmcC -o p --output-format csv -- $P && \
step pmcD rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $O/pmcD -o p --output-format csv -- $P; }; } && \
step fetch rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- $P && \
step write rocprofv3 --pmc WRITE_SIZE -d $O/write -o p --output-format csv -- $P && \
{ [ -n "$SKIP_FRAME" ] || { step fetchF rocprofv3 --pmc FETCH_SIZE -d $O/fetchF -o p --output-format csv -- $F && \
step writeF rocprofv3 --pmc WRITE_SIZE -d $O/writeF -o p --output-format csv -- $F; }; }
