#!/bin/bash
# round-3 GPU session AJ: draw kernel block size (64 / 128 / 256 threads) at C4, one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --pmc off"
bash tools/gpu_session.sh \
  "db256 200 $B" \
  "db128 200 SMORE_DRAW_BLOCK=128 $B" \
  "db64 200 SMORE_DRAW_BLOCK=64 $B" \
  "db256b 200 $B"
