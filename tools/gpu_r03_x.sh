#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
export TMPDIR=/tmp
B="python3 bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --pmc off"
bash tools/gpu_session.sh \
  "c2_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2prof -o run -- $B" \
  "c2_t01 200 $B --hot-tau 0.1" \
  "c2_t1 200 $B --hot-tau 1.0" \
  "c2_t3 200 $B --hot-tau 3.0" \
  "c2_cr256 200 $B --combine-rows 256" \
  "c2_cr0 200 $B --combine-rows 0" \
  "c2_hog 200 $B --mode hogwild" \
  "c2_atomic 200 $B --mode atomic"
