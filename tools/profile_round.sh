#!/bin/bash
# Kernel-trace stats and PMC traffic of the default bench on the GPU box.
#   tools/profile_round.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/...; copy the summaries into profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
run() {   # name, extra rocprofv3 args
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/$name.log" 2>&1
}
BENCH_ARGS=("$@")
run stats --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
find "$out" -name "*.csv" | sort
