#!/bin/bash
# round-3 GPU session H: Go walk pairs with the hybrid scatter, Go tests,
# replica exchange rules at world 2/4/8, Go C4 / C5 throughput
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_go 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_go.py tests/test_gpu_goshape.py" \
  "walk_check 300 python -u tools/go_walk_check.py" \
  "models_go 400 python -u tools/bench_models.py --configs c5go c5 --mode hybrid" \
  "bench_go 300 python -u bench.py --semantics go --steps 5 --warmup 2 --no-cpu-baseline" \
  "replica_quality 900 python -u tools/replica_quality.py"
