#!/bin/bash
# Run a list of GPU steps on the gpurun box, each under its own time limit.
# Usage: tools/gpu_jobs/steps.sh "<secs>:<name>:<command>" ...
# A step's output goes to gpurun_out/<name>.log.  Any failing step ends the
# script there (a failure may be a GPU fault: nothing else runs on the GPU
# after it).
mkdir -p gpurun_out
for step in "$@"; do
    secs="${step%%:*}"; rest="${step#*:}"
    name="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== [$name] $cmd (limit ${secs}s)"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] exit $rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then
        echo "=== stopping: step $name ended with $rc"
        exit $rc
    fi
done
exit 0
