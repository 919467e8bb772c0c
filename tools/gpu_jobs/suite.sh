# The GPU suite with the parity log (gpurun_out/parity.json).
set -o pipefail
mkdir -p gpurun_out
BMFR_PARITY_LOG=gpurun_out/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1; rc=$?
grep -E "passed|failed|fast_fit worst|Error" gpurun_out/suite.log | tail -12; exit $rc
