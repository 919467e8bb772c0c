#!/bin/bash
# Round-1 final evidence: full GPU suite, smoke, default bench (with CPU
# baseline), rocprofv3 kernel stats of the bench, PMC passes (traffic, SQ, TA).
export TMPDIR=/tmp
R=$PWD
B="python3 $R/bench.py --cpu-frames 0 --no-1080p"
tools/gpu_steps.sh \
"900:f_pytest:python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread" \
"300:f_smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
"400:f_bench:python bench.py" \
"200:f_stats:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/f_stats_d -- $B" \
"120:f_fetch:cd /tmp && rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/f_fetch_d -- $B" \
"120:f_write:cd /tmp && rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/f_write_d -- $B" \
"120:f_sq:cd /tmp && rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/f_sq_d -- $B" \
"120:f_sq2:cd /tmp && rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/f_sq2_d -- $B" \
"120:f_ta:cd /tmp && rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max --output-format csv -d $R/gpurun_out/f_ta_d -- $B"
