#!/bin/bash
# round-3 GPU session P: replica simulator at C2 scale with the source partition
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "sim_part 900 python -u tools/replica_sim.py --config c2 --ranks 1 4 8 --sync adaptive:64 adaptive:256+part adaptive:1024+part adaptive:4096+part mean+part"
