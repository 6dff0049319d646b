#!/bin/bash
# Run GPU steps one after another on the GPU box, each under its own time limit, each logging to
# gpurun_out/<name>.log.  A step that fails ordinarily (a test assertion: exit 1 or 2) does not stop the
# list; a step that timed out (124, 137), aborted (134) or crashed (139), or any exit > 128 (a signal),
# ends the script there -- nothing more touches the GPU after a fault or a hang.
#   bash tools/gpu_steps.sh "name:seconds:command" ["name:seconds:command" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
worst=0
for step in "$@"; do
    name="${step%%:*}"
    rest="${step#*:}"
    secs="${rest%%:*}"
    cmd="${rest#*:}"
    echo "== $name (limit ${secs}s): $cmd"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    if grep -q "+++ Timeout +++" "gpurun_out/$name.log"; then  # pytest-timeout ends a hung test with exit 1
        echo "== stopping: $name hit a test time limit"
        exit 124
    fi
    if [ "$rc" -ge 124 ]; then
        echo "== stopping: $name ended with $rc (time limit, abort, crash or signal)"
        exit "$rc"
    fi
    [ "$rc" -ne 0 ] && worst=$rc
done
exit $worst
