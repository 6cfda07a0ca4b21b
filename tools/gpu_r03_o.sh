#!/bin/bash
# round-3 GPU session O: the full -m gpu suite, smoke() and the default bench at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "gputest 1100 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu tests" \
  "smoke 200 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench 400 python -u bench.py"
