#!/bin/bash
# round-3 GPU session E: walk-model quality per mode, Go hybrid quality, adaptive exchange simulation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "walk_check 300 python -u tools/go_walk_check.py" \
  "quality_go_c2 400 python -u tools/quality.py --config c2 --semantics go --samples 268435456 --modes atomic hybrid hybrid:0.3:0 hybrid:0.1 hogwild --out gpurun_out/quality_go_c2.json" \
  "quality_cpp_c2 400 python -u tools/quality.py --config c2 --samples 268435456 --modes atomic hybrid hybrid:0.3:0 hogwild --out gpurun_out/quality_cpp_c2.json" \
  "sim_adapt 900 python -u tools/replica_sim.py --config c2 --ranks 1 2 4 8 --sync adaptive --c0 16 64 256 1024"
