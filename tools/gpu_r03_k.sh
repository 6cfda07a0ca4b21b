#!/bin/bash
# round-3 GPU session K: Go walk pairs with LDS combining + record prefetch
# (rebuilt objects): tests, quality, C5 throughput, Go C4 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_go 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_go.py tests/test_gpu_goshape.py tests/test_gpu_walkmodels.py" \
  "walk_check 300 python -u tools/go_walk_check.py" \
  "models_go 400 python -u tools/bench_models.py --configs c5go c5n2v c5 --mode hybrid" \
  "bench_go 300 python -u bench.py --semantics go --steps 5 --warmup 2 --no-cpu-baseline"
