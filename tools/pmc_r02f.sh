# HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass) of
# K1 as its own launch (tools/k1_frames.py) and of the one-launch frame
# kernel (tools/frame_times.py), 12 frames of 4K each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_r02f
mkdir -p $O
step() { local name=$1; shift; timeout -s KILL 150 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
step fetch rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o p --output-format csv -- python3 tools/k1_frames.py 3840 2160 12 && \
step write rocprofv3 --pmc WRITE_SIZE -d $O/write -o p --output-format csv -- python3 tools/k1_frames.py 3840 2160 12 && \
step fetchF rocprofv3 --pmc FETCH_SIZE -d $O/fetchF -o p --output-format csv -- python3 tools/frame_times.py 3840 2160 12 1 && \
step writeF rocprofv3 --pmc WRITE_SIZE -d $O/writeF -o p --output-format csv -- python3 tools/frame_times.py 3840 2160 12 1
