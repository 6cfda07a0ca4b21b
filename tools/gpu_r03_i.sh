#!/bin/bash
# round-3 GPU session I: Go C5 walk models with the hybrid scatter, the full
# -m gpu suite and smoke() at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash tools/gpu_session.sh \
  "models_go 400 python -u tools/bench_models.py --configs c5go c5n2v --mode hybrid" \
  "gputest 1000 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu tests" \
  "smoke 200 python -u -c 'import __graft_entry__ as g; g.smoke()'"
