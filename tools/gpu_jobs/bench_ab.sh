# Per-frame bench lines (4K, 100 frames) for libbmfr variants (BMFR_LIB), two
# interleaved rounds.  BENCH_FLAGS: extra bench.py flags (e.g. "--third-order
# --input-half" for BASELINE config 5).
#   bash tools/gpu_jobs/bench_ab.sh base variant...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in "$@"; do
  lib=$v; [ "$v" = base ] && lib=""
  BMFR_LIB=$lib BMFR_ALLOW_FOREIGN_BUILD=1 timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --no-sequence --no-variants --cpu-frames 0 $BENCH_FLAGS > gpurun_out/sab_$v.json 2> gpurun_out/sab_$v.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/sab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['device_ms_per_frame'], d['kernel_ms'])"
done; done
