#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, each pass its
# own time limit; stops at the first abnormal exit).
#   tools/pmc_session.sh <tag> "<counters pass 1>" "<counters pass 2>" ... -- [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=$1; shift
passes=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do passes+=("$1"); shift; done
[ "$1" = "--" ] && shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
i=0
for p in "${passes[@]}"; do
    i=$((i+1))
    echo "=== pass $i: $p"
    timeout -s KILL 240 rocprofv3 --pmc $p -d "$out/p$i" -o "p$i" --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
    rc=$?
    echo "=== pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
exit 0
