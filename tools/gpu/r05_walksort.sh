set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -v --timeout 600 --timeout-method thread -k "walk" > gpurun_out/walksort_tests.log 2>&1; rc=$?; echo rc=$rc
grep -E "PASS|FAIL|Error" gpurun_out/walksort_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 4 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bwsort.jsonl 2> gpurun_out/bwsort.err || { tail -20 gpurun_out/bwsort.err; exit 1; }
python tools/block_sim.py gpurun_out/bwsort.jsonl
python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d.get('part')==0 or d['nparts']==1: print(d['nparts'], d['epoch_ms'], d.get('prepare_ms'), [c[2] for c in d.get('cells',[])])" gpurun_out/bwsort.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py -v -s --timeout 600 --timeout-method thread -k "c5" > gpurun_out/walksort_c5.log 2>&1; rc=$?; echo rc=$rc
grep -E "PASS|FAIL|group [0-9]" gpurun_out/walksort_c5.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -v --timeout 600 --timeout-method thread > gpurun_out/bench_tests.log 2>&1; rc=$?; echo bench_rc=$rc
grep -E "PASS|FAIL" gpurun_out/bench_tests.log | tail -4
exit $rc
