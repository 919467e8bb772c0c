set -o pipefail
for r in 1 2; do for v in old base; do
  lib=$v; [ "$v" = base ] && lib=""
  for cfg in "" "--input-half --third-order"; do
    BMFR_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --no-sequence --cpu-frames 0 $cfg > gpurun_out/abh.json 2> gpurun_out/abh.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/abh.json').read().strip().splitlines()[-1]); print('$v', '$cfg', d['value'], d['kernel_ms'])"
  done
done; done
