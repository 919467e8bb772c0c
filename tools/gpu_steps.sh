#!/bin/bash
# Run a list of GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_steps.sh "<secs>:<name>:<command>" ...
# A step's output goes to gpurun_out/<name>.log.  A plain failure (exit 1,
# e.g. a failing test) lets the next step run; a crash / abort / timeout /
# kill (124, 134, 137, 139 or > 128) ends the script there.
mkdir -p gpurun_out
for step in "$@"; do
    secs="${step%%:*}"; rest="${step#*:}"
    name="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== [$name] $cmd (limit ${secs}s)"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] exit $rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ge 124 ]; then
        echo "=== stopping: step $name ended with $rc"
        exit $rc
    fi
done
exit 0
