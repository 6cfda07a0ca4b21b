#!/bin/bash
# round-3 GPU session Y: hot-row threshold tau at C4 (speed) and C2/C4 (held-out quality)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --pmc off"
bash tools/gpu_session.sh \
  "c4_t03 200 $B" \
  "c4_t1 200 $B --hot-tau 1.0" \
  "c4_t3 200 $B --hot-tau 3.0" \
  "c4_t10 200 $B --hot-tau 10.0" \
  "q_c2_tau 300 python -u tools/quality.py --config c2 --samples 268435456 --modes atomic hybrid:0.3 hybrid:1.0 hybrid:3.0 hybrid:10.0 --out gpurun_out/q_c2_tau.json" \
  "q_c4_tau 600 python -u tools/quality.py --config c4 --samples 1073741824 --modes atomic hybrid:0.3 hybrid:1.0 hybrid:3.0 --out gpurun_out/q_c4_tau.json"
