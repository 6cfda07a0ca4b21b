#!/bin/bash
# One rocprofv3 --pmc pass over a short bench.py run of a config (counters of
# one pass only: <= 4 TCC, MI355X_MICROARCH.md).  Output CSV under gpurun_out/.
#   tools/pmc_pass.sh <config> <tag> <counter> [<counter> ...]
cfg=$1; tag=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/pmc_${cfg}_${tag}" -o run -- \
    python3 bench.py --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline --pmc off
