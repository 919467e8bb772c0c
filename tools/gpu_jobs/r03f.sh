# Round 3: K2 threads-per-tile variants (parity through the one-launch ==
# two-launch test, then K1/K2 A/B timing), then the N > 1 bench rehearsal.
set -o pipefail
mkdir -p gpurun_out
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
P="python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k"
BMFR_LIB=k2nt768 step k2nt768_pytest 300 $P "one_launch or fast_fit_frame_apis" && \
BMFR_LIB=k2nt384 step k2nt384_pytest 300 $P "one_launch" && \
step ab_k2 600 python tools/ab.py time base k2nt384 k2nt768 && \
bash tools/gpu_jobs/r03e.sh
