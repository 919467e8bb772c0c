# Full default bench.py lines (4K headline + 1080p + 8K + variants) for
# libbmfr variants (BMFR_LIB), interleaved.
#   bash tools/gpu_jobs/bench_full_ab.sh base variant...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=$v; [ "$v" = base ] && lib=""
  BMFR_LIB=$lib BMFR_ALLOW_FOREIGN_BUILD=1 timeout -k 10 500 python bench.py --cpu-frames 0 > gpurun_out/full_$v.json 2> gpurun_out/full_$v.err || exit $?
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/full_{v}.json").read().strip().splitlines()[-1])
keys = [k for k in d if k.startswith("ms_per_frame")]
print(v, "value", d["value"], d["kernel_ms"], {k: d[k]["value"] if isinstance(d[k], dict) else d[k] for k in keys})
PY
done
