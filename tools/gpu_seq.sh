# Per-frame vs sequence-mode bench lines at 4K (steps 100), same box; extra
# arguments: libbmfr variants (BMFR_LIB) to time in sequence mode as well.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --cpu-frames 0 > gpurun_out/seq_perframe.json 2> gpurun_out/seq_perframe.err && \
timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --cpu-frames 0 --sequence > gpurun_out/seq_seq.json 2> gpurun_out/seq_seq.err || exit $?
for v in "$@"; do
  BMFR_LIB=$v timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --cpu-frames 0 --sequence > gpurun_out/seq_seq_$v.json 2> gpurun_out/seq_seq_$v.err || exit $?
done
python - "$@" <<'PY'
import json, sys
for n in ["perframe", "seq"] + ["seq_" + v for v in sys.argv[1:]]:
    d = json.loads(open(f"gpurun_out/seq_{n}.json").read().strip().splitlines()[-1])
    print(n, d["value"], d["kernel_ms"])
PY
