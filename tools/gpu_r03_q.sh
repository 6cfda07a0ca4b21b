#!/bin/bash
# round-3 GPU session Q: multi-rank tests at the final defaults (partition, c0 2048)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_multi 900 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_multi.py"
