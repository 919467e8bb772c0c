# What the round-end driver runs: smoke(), then the bench with its flags.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_steps20.log 2>&1 || { tail -20 gpurun_out/bench_steps20.log; exit 1; }
grep '^{' gpurun_out/bench_steps20.log | tail -1 | cut -c1-400
