set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local secs=$1 name=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -12 gpurun_out/$name.log; return $rc; }
run 200 frames python tools/k1_frames.py 3840 2160 100 && \
run 200 phases python tools/k1_phases.py 3840 2160 && \
run 300 gloo2 env BMFR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 10 --warmup 3 --cpu-frames 0 && \
run 300 gloo4 env BMFR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 10 --warmup 3 --cpu-frames 0
