set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -v --timeout 600 --timeout-method thread > gpurun_out/setup_tests.log 2>&1; rc=$?; echo rc=$rc
grep -E "PASS|FAIL" gpurun_out/setup_tests.log | tail -14
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 4 8 --parts 0 > gpurun_out/bset.jsonl 2> gpurun_out/bset.err || { tail -20 gpurun_out/bset.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bset.jsonl'):
    d=json.loads(l); print(d['nparts'], d.get('setup_s'), d['epoch_ms'])"
