# Round 3: the fit's dots and pivot norms as fused FMAs (bit-exact by the
# exact-product argument): the whole GPU suite on the new library, then K1 A/B
# against the previous build (libbmfr_old.so), exact and fast_fit configs.
set -o pipefail
mkdir -p gpurun_out
BMFR_PARITY_LOG=gpurun_out/parity_i.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 \
  --timeout-method thread > gpurun_out/suite_i.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/suite_i.log | head -20; tail -5 gpurun_out/suite_i.log; exit 1; }
grep -E "passed" gpurun_out/suite_i.log | tail -2
timeout -k 10 600 python tools/ab.py time old base > gpurun_out/ab_i_exact.log 2>&1; echo "ab exact rc=$?"; tail -3 gpurun_out/ab_i_exact.log
AB_FAST_FIT=1 timeout -k 10 600 python tools/ab.py time old base > gpurun_out/ab_i_fast.log 2>&1; echo "ab fast rc=$?"; tail -3 gpurun_out/ab_i_fast.log
