# Round 3 closing measurements: rocprofv3 kernel stats of the default bench
# command, the bench line, the driver's command, and SQ / PMC passes of the
# fast_fit K1 and frame kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03jstats -o run --output-format csv -- python3 bench.py --cpu-frames 0 > gpurun_out/r03jstats.log 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 10 420 python3 bench.py > gpurun_out/r03j_bench.log 2>&1 || { tail -5 gpurun_out/r03j_bench.log; exit 1; }
grep '^{' gpurun_out/r03j_bench.log | tail -1 | cut -c1-200
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03j_steps20.log 2>&1 || exit 1
grep '^{' gpurun_out/r03j_steps20.log | tail -1 | cut -c1-200
SKIP_STATS=1 bash tools/gpu_jobs/profile.sh r03jfast 3840 2160 --fast-fit
