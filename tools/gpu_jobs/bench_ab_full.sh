# Whole bench lines (4K per-frame + sequence API + 1080p one-launch line, 100
# frames) for libbmfr variants (BMFR_LIB), two interleaved rounds; prints the
# 4K value, the sequence-API figure and the 1080p figure.
#   bash tools/gpu_jobs/bench_ab_full.sh base variant...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in "$@"; do
  lib=$v; [ "$v" = base ] && lib=""
  BMFR_LIB=$lib BMFR_ALLOW_FOREIGN_BUILD=1 timeout -k 10 300 python bench.py --steps 100 --no-8k --no-variants --cpu-frames 0 $BENCH_FLAGS > gpurun_out/fab_$v.json 2> gpurun_out/fab_$v.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/fab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], {k: v for k, v in d.items() if k.startswith('ms_per_frame_') and not isinstance(v, dict)}, {k: v.get('value') for k, v in d.items() if k.startswith('ms_per_frame_') and isinstance(v, dict)})"
done; done
