#!/bin/bash
# round-3 GPU session AI: hot-row threshold for the pair-record models on C5's graph (d=128, 40 steps, window 5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "dw_c5_tau10 900 python -u tools/dw_quality.py --config c5 --dim 128 --walk-times 10 --walk-steps 40 --window 5 --settings atomic hybrid:0.3:128:0 hybrid:1.0:128:0"
