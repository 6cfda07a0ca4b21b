#!/bin/bash
# Run a sequence of GPU steps on the gpurun box.  Each step has its own time
# limit; a step ending in a crash / abort / timeout (exit >= 124, or killed by
# a signal) stops the session so nothing else touches a possibly-faulted GPU.
# Test failures (exit 1) do not stop later steps.
#   tools/gpu_session.sh "<name> <timeout_s> <command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name=${spec%% *}; rest=${spec#* }
    tmo=${rest%% *}; cmd=${rest#* }
    echo "=== [$name] (limit ${tmo}s) $cmd" | tee -a gpurun_out/session.log
    start=$(date +%s)
    timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
    tail -n 30 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
        echo "=== stopping: abnormal exit of [$name]" | tee -a gpurun_out/session.log
        exit $rc
    fi
done
exit 0
