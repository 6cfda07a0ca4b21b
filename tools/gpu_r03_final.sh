#!/bin/bash
# round-3 final GPU check at HEAD: full -m gpu suite, smoke, default bench (live PMC), kernel-trace stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tests_full 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests" \
  "smoke 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench 400 python -u bench.py" \
  "prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
