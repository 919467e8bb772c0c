# Per-frame vs sequence-mode bench lines at 4K (steps 100), same box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --cpu-frames 0 > gpurun_out/seq_perframe.json 2> gpurun_out/seq_perframe.err && \
timeout -k 10 300 python bench.py --steps 100 --no-1080p --no-8k --cpu-frames 0 --sequence > gpurun_out/seq_seq.json 2> gpurun_out/seq_seq.err
rc=$?; tail -c 1500 gpurun_out/seq_perframe.json; echo; tail -c 1500 gpurun_out/seq_seq.json; exit $rc
