# Round 3 profiles: the default bench command under rocprofv3 (kernel stats)
# with SQ / TA / I-cache / HBM passes of the 4K default, the same passes for
# BASELINE config 5 (half inputs, B = 16), and the 8K 4x2 tile cost.
set -o pipefail
mkdir -p gpurun_out
SKIP_STATS=1 bash tools/gpu_jobs/profile.sh r03prof && \
SKIP_STATS=1 bash tools/gpu_jobs/profile.sh r03cfg5 3840 2160 --third-order --input-half && \
timeout -k 10 300 python tools/tile_cost.py 1920 2160 4 2 5 > gpurun_out/r03_tile_cost.log 2>&1; echo "tile_cost rc=$?"; tail -5 gpurun_out/r03_tile_cost.log
