#!/bin/bash
# round-3 GPU session AF: BPR row prefetch A/B at C3 (same box), BPR GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "c3_pf 300 python -u tools/bench_models.py --configs c3 --steps 5" \
  "c3_nopf 300 SMORE_LIB=tmp_nopf/libsmore_hip.so python -u tools/bench_models.py --configs c3 --steps 5" \
  "c3_pf2 300 python -u tools/bench_models.py --configs c3 --steps 5" \
  "bpr_tests 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k 'bpr or BPR or c3' tests"
