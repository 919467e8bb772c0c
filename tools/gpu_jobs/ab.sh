# usage: bash tools/gpu_jobs/ab.sh "<pytest -k expr or empty>" variant...
set -o pipefail
mkdir -p gpurun_out
K="$1"; shift
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/ab_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python tools/ab.py time "$@" > gpurun_out/ab_time.log 2>&1; rc=$?
tail -12 gpurun_out/ab_time.log; exit $rc
