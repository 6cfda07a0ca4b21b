#!/bin/bash
# round-3 GPU session AD: Go LINE-2 at C4 with the per-path hot-row threshold (and W-row combining for reference)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off --semantics go"
bash tools/gpu_session.sh \
  "go_c4 300 $B" \
  "go_c4_t03 300 $B --hot-tau 0.3" \
  "q_c2_go 300 python -u tools/quality.py --config c2 --samples 268435456 --semantics go --modes atomic hybrid:0.3 hybrid:1.0 --out gpurun_out/q_c2_go_tau.json"
