# Round 3: the GPU suite (with the fast-fit and MFMA-WY tests) and the bench line.
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
BMFR_PARITY_LOG=gpurun_out/parity_r03.json step r03_pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s && \
step r03_bench 420 python3 bench.py
