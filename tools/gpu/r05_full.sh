set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/full_gpu.log 2>&1; rc=$?; echo gpu_rc=$rc
grep -cE "PASSED" gpurun_out/full_gpu.log
grep -E "FAILED|Error|passed|failed" gpurun_out/full_gpu.log | tail -15
exit $rc
