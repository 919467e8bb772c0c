# Round 3: fast_fit level 2 (fused dots and pivot norms too): its tolerance
# against the reference, then K1 A/B on the fast_fit configuration.
set -o pipefail
mkdir -p gpurun_out
BMFR_LIB=fast2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread \
  -k "fast_fit" > gpurun_out/fast2_pytest.log 2>&1; rc=$?
grep -E "passed|failed|worst|Error" gpurun_out/fast2_pytest.log | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_FAST_FIT=1 timeout -k 10 600 python tools/ab.py time base fast2 > gpurun_out/ab_fast2.log 2>&1; echo "ab rc=$?"
tail -4 gpurun_out/ab_fast2.log
