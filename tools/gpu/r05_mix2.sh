set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_goshape.py -v -s --timeout 300 --timeout-method thread -k "rows or pairs" > gpurun_out/pairs_rows.log 2>&1; rc=$?; echo pairs_rc=$rc
grep -E "PASS|FAIL|per call|Error" gpurun_out/pairs_rows.log | tail -12
[ $rc -le 1 ] || exit $rc
bash tools/gpu/r05_walkdbg3.sh
