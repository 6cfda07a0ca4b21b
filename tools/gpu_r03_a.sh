#!/bin/bash
# round-3 GPU session A: probes, C4 tests, Go hogwild test, bench, draw-pattern PMC calibration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
P="timeout -s KILL 60 rocprofv3"
bash tools/gpu_session.sh \
  "probe_rand 240 ./tools/probe_r3 rand" \
  "probe_rows 300 ./tools/probe_r3 rows" \
  "pmc_rand_nt8 90 $P --pmc FETCH_SIZE -d gpurun_out/pmc_rand/nt8 -o nt8 --output-format csv -- ./tools/probe_r3 rand1 80000000 8" \
  "pmc_rand_ct16 90 $P --pmc FETCH_SIZE -d gpurun_out/pmc_rand/ct16 -o ct16 --output-format csv -- ./tools/probe_r3 rand1 6400000000 16" \
  "pmc_rand_vt32 90 $P --pmc FETCH_SIZE -d gpurun_out/pmc_rand/vt32 -o vt32 --output-format csv -- ./tools/probe_r3 rand1 320000000 32" \
  "pmc_rand_big8 90 $P --pmc FETCH_SIZE -d gpurun_out/pmc_rand/big8 -o big8 --output-format csv -- ./tools/probe_r3 rand1 6400000000 8" \
  "tests_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_go.py -k \"c4 or hogwild_matches\"" \
  "bench 400 python -u bench.py" \
  "tests_shim 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_goshape.py" \
  "tests_multi 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_multi.py -k n_ranks"
