#!/bin/bash
# round-3 GPU session C: waves=3 default build -- GPU suite, bench, replica-exchange simulations, rocprof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "gputest 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k \"not n_ranks\"" \
  "bench 400 python -u bench.py" \
  "bench_go 300 python -u bench.py --no-cpu-baseline --semantics go" \
  "sim_c2 600 python -u tools/replica_sim.py --config c2 --ranks 1 2 4 8 --sync sum --sub 8 --hot 16384 65536" \
  "sim_c4 600 python -u tools/replica_sim.py --config c4 --ranks 1 4 --sync sum --sub 8 --hot 65536 262144 --total 2147483648" \
  "quality_c4 600 python -u tools/quality.py --config c4 --samples 2000000000 --modes atomic hybrid hybrid:0.1 hybrid:1.0 --out gpurun_out/quality_c4_r03.json" \
  "prof 600 bash tools/profile_round.sh r03c"
