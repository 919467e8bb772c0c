set -o pipefail
mkdir -p gpurun_out/ic
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 -L > gpurun_out/ic/avail.txt 2>&1; echo "list rc=$?"
grep -E "SQC_ICACHE|SQ_IFETCH|SQ_WAIT_INST|SQC_" gpurun_out/ic/avail.txt | head -40
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d gpurun_out/ic/p1 -o p1 --output-format csv -- python3 tools/k1_frames.py 3840 2160 12 > gpurun_out/ic/p1.log 2>&1; echo "p1 rc=$?"
tail -3 gpurun_out/ic/p1.log
