set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_blocks.py -v -s --timeout 600 --timeout-method thread > gpurun_out/multi_tests.log 2>&1; rc=$?; echo multi_rc=$rc
grep -E "PASS|FAIL|group [0-9]|Error|assert" gpurun_out/multi_tests.log | tail -40
exit $rc
