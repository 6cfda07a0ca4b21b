#!/bin/bash
# round-3 GPU session M2: c0 sweep (high end) with the source partition
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "replica_part_hi 900 python -u tools/replica_quality.py --worlds 4 8 --rules adaptive:2048+part adaptive:4096+part adaptive:16384+part sum+part mean+part"
