set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 4 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bws.jsonl 2> gpurun_out/bws.err || { tail -20 gpurun_out/bws.err; exit 1; }
python tools/block_sim.py gpurun_out/bws.jsonl
python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d.get('part')==0 or d['nparts']==1: print(d['nparts'], d['epoch_ms'], d.get('prepare_ms'), [c[2] for c in d.get('cells',[])])" gpurun_out/bws.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_blocks.py -v -s --timeout 600 --timeout-method thread -k "c5 or walk" > gpurun_out/walkslice_tests.log 2>&1; rc=$?; echo tests_rc=$rc
grep -E "PASS|FAIL|group [0-9]|blocks" gpurun_out/walkslice_tests.log | tail -20
exit $rc
