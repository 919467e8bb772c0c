set -o pipefail
mkdir -p gpurun_out
# parity first with the flag build only (BMFR_LIB=flag), small and full sizes
BMFR_LIB=flag timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fused_frame_matches_stages or f3840x2160_h13 or sequence" > gpurun_out/flag_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/flag_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab.py time base flag > gpurun_out/ab_time.log 2>&1; rc=$?
tail -4 gpurun_out/ab_time.log; exit $rc
