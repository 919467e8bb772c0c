# Round 3, fast-fit headline: its parity test, PMC / SQ passes of the fast
# K1 and frame kernel, rocprofv3 stats of the default bench command, then
# the bench line itself.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
BMFR_PARITY_LOG=gpurun_out/parity_g.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 \
  --timeout-method thread -k "fast_fit" > gpurun_out/fast_pytest.log 2>&1 || { tail -20 gpurun_out/fast_pytest.log; exit 1; }
grep -E "passed|worst" gpurun_out/fast_pytest.log | tail -8
SKIP_STATS=1 bash tools/gpu_jobs/profile.sh r03fast 3840 2160 --fast-fit || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03fstats -o run --output-format csv -- python3 bench.py --cpu-frames 0 > gpurun_out/r03fstats.log 2>&1; echo "stats rc=$?"
timeout -k 10 420 python3 bench.py > gpurun_out/r03_bench_final.log 2>&1; echo "bench rc=$?"
grep '^{' gpurun_out/r03_bench_final.log | tail -1 | cut -c1-300
