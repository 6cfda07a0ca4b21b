#!/bin/bash
# round-3 GPU session J: Go walk pairs with LDS combining + record prefetch
# (tests, quality, C5 throughput), exchange period vs quality at 8 ranks, the
# draw/update overlap at the full update grid
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_go 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_go.py tests/test_gpu_goshape.py" \
  "walk_check 300 python -u tools/go_walk_check.py" \
  "models_go 400 python -u tools/bench_models.py --configs c5go c5n2v c5 --mode hybrid" \
  "bench_dc25_full 300 SMORE_DRAW_LEAVE=0 SMORE_DRAW_CHUNK=33554432 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "bench_dc26_full 300 SMORE_DRAW_LEAVE=0 SMORE_DRAW_CHUNK=67108864 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "replica_period 900 python -u tools/replica_quality.py --worlds 8 --rules adaptive:64 mean --per 6000" \
  "replica_period2 900 python -u tools/replica_quality.py --worlds 8 --rules adaptive:64 --per 24000"
