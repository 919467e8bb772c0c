set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local secs=$1 name=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -5 gpurun_out/$name.log; return $rc; }
run 900 pytest python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 400 --timeout-method thread && \
run 300 bench python bench.py --steps 20 --warmup 5 && \
run 300 gloo2 env BMFR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 10 --warmup 3 --cpu-frames 0 && \
run 300 gloo4 env BMFR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 10 --warmup 3 --cpu-frames 0
