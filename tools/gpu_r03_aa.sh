#!/bin/bash
# round-3 GPU session AA: default hot-row threshold 1.0 -- full -m gpu suite, other configs, default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tests_full 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests" \
  "models 400 python -u tools/bench_models.py --configs c2 c3 c5 c5go" \
  "bench 400 python -u bench.py"
