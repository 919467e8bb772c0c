set -o pipefail
mkdir -p gpurun_out/mfma
export TMPDIR=/tmp
timeout -k 10 300 python tools/mfma_experiment.py 3840 2160 4 > gpurun_out/mfma/experiment.log 2>&1; rc=$?
tail -8 gpurun_out/mfma/experiment.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mfma/trace -o run --output-format csv -- python3 tools/mfma_experiment.py 3840 2160 2 > gpurun_out/mfma/trace.log 2>&1; echo "trace rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/mfma/pmc -o pmc --output-format csv -- python3 tools/mfma_experiment.py 3840 2160 2 > gpurun_out/mfma/pmc.log 2>&1; echo "pmc rc=$?"
