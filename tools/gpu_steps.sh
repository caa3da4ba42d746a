#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first fault-like exit status
# (timeout 124/137, abort 134, segfault 139) so nothing else touches a possibly-wedged GPU.
# usage: tools/gpu_steps.sh "<name>:<seconds>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for step in "$@"; do
    name="${step%%:*}"; rest="${step#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "=== $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== $name rc=$rc in $(( $(date +%s) - start ))s"
    tail -n 25 "gpurun_out/$name.log"
    case $rc in
        124|134|137|139) echo "!!! $name ended with fault-like status $rc; stopping"; exit $rc ;;
    esac
done
exit 0
