#!/bin/bash
# round-3 GPU session AH: write-combining rows / drain interval at the edge default tau 1.0 (C4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --pmc off"
bash tools/gpu_session.sh \
  "cr128 200 $B" \
  "cr64 200 $B --combine-rows 64" \
  "cr96 200 $B --combine-rows 96" \
  "cr128_f16 200 $B --combine-flush 16" \
  "cr128_f64 200 $B --combine-flush 64" \
  "cr128b 200 $B"
