# Round 3: GPU suite, the default bench line, then the K1 experiments:
# parity subset on share3, K1/K2 A/B timing of base / share / sharec / share3 /
# fastfit, and fastfit's TAA-output rel-L2 against the reference at 4K.
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
step r03_pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread && \
step r03_bench 300 python3 bench.py && \
BMFR_LIB=share3 step share3_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or reference_fullsize or one_launch" && \
step ab_k1 900 python tools/ab.py time base share sharec share3 fastfit && \
BMFR_LIB=fastfit step tol_fastfit 300 python tools/tolerance_check.py f3840x2160_h13 17
