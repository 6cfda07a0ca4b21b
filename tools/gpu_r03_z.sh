#!/bin/bash
# round-3 GPU session Z: hot-row threshold tau, C4 held-out quality after 2^31 samples
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "q_c4_tau 900 python -u tools/quality.py --config c4 --samples 2147483648 --modes atomic hybrid:0.3 hybrid:1.0 hybrid:3.0 --out gpurun_out/q_c4_tau31.json"
