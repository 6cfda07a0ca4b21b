set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "--combine-rows 0" "--hot-tau 0" "--combine-rows 64 --hot-tau 1000"; do
timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 2 --totals 4 --mode hybrid $a > gpurun_out/bq_dw_dbg.jsonl 2> gpurun_out/bq_dw_dbg.err || { tail -20 gpurun_out/bq_dw_dbg.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bq_dw_dbg.jsonl'):
    d=json.loads(l); print('$a', d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])"
done
