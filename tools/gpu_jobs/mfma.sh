# The compact-WY MFMA fitter experiment (tools/mfma_experiment.py, DESIGN.md
# section 4) at B = 16 (BASELINE config 5's feature set) and B = 13, panel
# widths 4, 8 and 16 (one full-width panel), with its kernel trace and MFMA
# counters.  tools/libwy.so is built beforehand:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC tools/wy_fitter.hip -o tools/libwy.so
set -o pipefail
O=gpurun_out/mfma
mkdir -p $O
export TMPDIR=/tmp
for B in 16 13; do
  timeout -k 10 300 python tools/mfma_experiment.py 3840 2160 4 $B 4,8,16 > $O/experiment_b$B.log 2>&1 || exit $?
  tail -3 $O/experiment_b$B.log
done
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/mfma_experiment.py 3840 2160 2 16 4,8,16 > $O/trace.log 2>&1; echo "trace rc=$?"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o pmc --output-format csv -- python3 tools/mfma_experiment.py 3840 2160 2 16 4,8,16 > $O/pmc.log 2>&1; echo "pmc rc=$?"
