set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pairs_tests.log 2>&1; echo pairs_rc=$?
grep -E "PASS|FAIL|per call|Error" gpurun_out/pairs_tests.log | tail -20
bash tools/gpu/r05_walkdbg2.sh
