#!/bin/bash
# Golden regeneration (synthetic camera changed), GPU tests incl. tiled
# parity, single-GPU bench, 2-rank tiled rehearsal on one GPU (gloo staging).
export TMPDIR=/tmp
tools/gpu_steps.sh \
"300:golden:python tests/golden/make_golden.py --out gpurun_out/golden" \
"600:t_pytest:python -m pytest tests -m gpu -q -x" \
"150:t_bench:python bench.py --cpu-frames 2" \
"300:t_rehearse2:BMFR_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2"
