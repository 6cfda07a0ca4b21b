#!/bin/bash
# round-3 GPU session R (re-entry): full -m gpu suite, smoke and default bench at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_full 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests" \
  "smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench 400 python -u bench.py"
