#!/bin/bash
# round-3 GPU session D: W-row write-combining, Go packed draws, mean exchange default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "gputest 1100 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread" \
  "bench 400 python -u bench.py" \
  "bench_go 300 python -u bench.py --no-cpu-baseline --semantics go" \
  "models 600 python -u tools/bench_models.py --configs c2 c3 c5 c5go" \
  "sim_mean 600 python -u tools/replica_sim.py --config c2 --ranks 1 2 4 8 --sync mean" \
  "prof 600 bash tools/profile_round.sh r03d"
