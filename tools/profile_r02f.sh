# Round-2 closing evidence on the GPU box: rocprofv3 kernel statistics of the
# default bench command, the default bench line (CPU baseline included) and
# the driver's own command (--steps 20 --warmup 5).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_r02f
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step stats 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 bench.py --cpu-frames 0 && \
step bench 300 python3 bench.py && \
step bench20 300 python3 bench.py --steps 20 --warmup 5
