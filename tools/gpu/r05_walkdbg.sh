set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -v -s --timeout 300 --timeout-method thread -k "walks_parallel" > gpurun_out/walkdbg.log 2>&1; echo rc=$?
grep -E "DeepWalk|PASS|FAIL|Error" gpurun_out/walkdbg.log | head -20
for m in atomic hybrid; do
timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 2 --totals 2 --mode $m > gpurun_out/bq_dw_$m.jsonl 2> gpurun_out/bq_dw_$m.err || { tail -20 gpurun_out/bq_dw_$m.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bq_dw_$m.jsonl'):
    d=json.loads(l); print('$m', d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])"
done
