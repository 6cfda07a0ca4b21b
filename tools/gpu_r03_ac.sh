#!/bin/bash
# round-3 GPU session AC: final kernel-trace stats of the default bench at HEAD (and the env a profiled run sees)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "prof_final 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline" \
  "envcheck 100 rocprofv3 --kernel-trace -d gpurun_out/envchk -o run -- python3 -c 'import os; print(sorted(k for k in os.environ if \"ROC\" in k or \"HSA\" in k))'"
