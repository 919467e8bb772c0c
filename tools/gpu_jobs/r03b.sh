# Round 3: bisect the tap-sharing variants' parity (a test failure, rc 1, does
# not stop the job; any other non-zero status does), then K1/K2 A/B timing and
# the fast-fit tolerance against the reference.
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
P="python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k"
BMFR_LIB=share step share_pytest 600 $P "fused_frame_matches_stages or one_launch"; ok $? || exit 1
BMFR_LIB=sharec step sharec_pytest 600 $P "fused_frame_matches_stages or one_launch"; ok $? || exit 1
BMFR_LIB=share3 step share3b_pytest 600 $P "fused_frame_matches_stages or one_launch"; ok $? || exit 1
step ab_k1 900 python tools/ab.py time base share sharec share3 fastfit fastfit2 || exit 1
BMFR_LIB=fastfit step tol_fastfit 300 python tools/tolerance_check.py f3840x2160_h13 17 && BMFR_LIB=fastfit2 step tol_fastfit2 300 python tools/tolerance_check.py f3840x2160_h13 17
