#!/bin/bash
# round-3 GPU session G: multi-rank tests, rocprof kernel stats + FETCH/WRITE
# PMC of the default C4 bench at HEAD and of C5 DeepWalk (pair_train_kernel),
# Go C5 kernel stats, the exchange passes at C4, the draw/update overlap
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
out=gpurun_out/prof_r03g
mkdir -p $out
bash tools/gpu_session.sh \
  "tests_multi 900 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_multi.py" \
  "models 300 python -u tools/bench_models.py --configs c5go c5 c3 c2" \
  "c4_stats 300 rocprofv3 --kernel-trace --stats -d $out/c4_stats -o c4_stats --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline" \
  "c4_fetch 240 rocprofv3 --pmc FETCH_SIZE -d $out/c4_fetch -o c4_fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "c4_write 240 rocprofv3 --pmc WRITE_SIZE -d $out/c4_write -o c4_write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline" \
  "c5_stats 300 rocprofv3 --kernel-trace --stats -d $out/c5_stats -o c5_stats --output-format csv -- python3 tools/bench_models.py --configs c5 c5go --steps 2" \
  "c5_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $out/c5_fetch -o c5_fetch --output-format csv -- python3 tools/bench_models.py --configs c5 --steps 2" \
  "c5_write 300 rocprofv3 --pmc WRITE_SIZE -d $out/c5_write -o c5_write --output-format csv -- python3 tools/bench_models.py --configs c5 --steps 2" \
  "ex_stats 200 rocprofv3 --kernel-trace --stats -d $out/ex_stats -o ex_stats --output-format csv -- python3 tools/exchange_passes.py" \
  "bench_dc25 300 SMORE_DRAW_CHUNK=33554432 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
  "bench_dc26 300 SMORE_DRAW_CHUNK=67108864 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
