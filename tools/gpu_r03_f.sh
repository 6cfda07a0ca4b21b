#!/bin/bash
# round-3 GPU session F: Go walk pairs on the record path (serial bit-exact
# tests, parallel quality), Go / C++ hybrid quality without W-row
# write-combining, replica exchange rules at world 2/4/8 (gloo ranks on one
# GPU), exchange pass timing at C4, Go DeepWalk throughput
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "tests_go 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_go.py tests/test_gpu_goshape.py" \
  "walk_check 300 python -u tools/go_walk_check.py" \
  "quality_go_w0 300 SMORE_SH_WROWS=0 python -u tools/quality.py --config c2 --semantics go --samples 268435456 --modes atomic hybrid --out gpurun_out/quality_go_c2_w0.json" \
  "quality_cpp_w0 300 SMORE_SH_WROWS=0 python -u tools/quality.py --config c2 --samples 268435456 --modes atomic hybrid --out gpurun_out/quality_cpp_c2_w0.json" \
  "replica_quality 900 python -u tools/replica_quality.py" \
  "exchange_passes 200 python -u tools/exchange_passes.py" \
  "bench_go_w0 300 SMORE_SH_WROWS=0 python -u bench.py --semantics go --steps 5 --warmup 2" \
  "bench_cpp_w0 300 SMORE_SH_WROWS=0 python -u bench.py --steps 5 --warmup 2" \
  "models_go 400 python -u tools/bench_models.py --configs c5go c5 --mode atomic"
