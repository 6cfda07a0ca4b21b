set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for sp in 0 1; do
  SMORE_SPLIT=$sp timeout -k 10 600 python -u tools/bench_models.py --configs c3 c2 c4 > gpurun_out/split_$sp.jsonl 2> gpurun_out/split_$sp.err || { tail -20 gpurun_out/split_$sp.err; exit 1; }
  sed "s/^/split=$sp /" gpurun_out/split_$sp.jsonl | cut -c1-400
done
SMORE_SPLIT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 600 --timeout-method thread -k "full_grid_hybrid_matches_atomic" > gpurun_out/split_tests.log 2>&1; rc=$?; echo tests_rc=$rc
grep -E "PASS|FAIL|Error|assert|rel|loss" gpurun_out/split_tests.log | tail -20
