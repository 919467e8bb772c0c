# The N > 1 bench path rehearsed on one GPU with gloo (host-staged halo
# messages): bench.py --gpus N for each N given (default 2 4), short runs.
set -o pipefail
mkdir -p gpurun_out
for n in ${@:-2 4}; do
  BMFR_DIST_BACKEND=gloo timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
    > gpurun_out/dist$n.log 2>&1 || { echo "n=$n rc=$?"; tail -20 gpurun_out/dist$n.log; exit 1; }
  echo "n=$n ok"; grep '^{' gpurun_out/dist$n.log | tail -1 | cut -c1-300
done
