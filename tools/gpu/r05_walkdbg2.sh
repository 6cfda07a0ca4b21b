set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in atomic hybrid; do
timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 1 2 --totals 10 --mode $m --diag > gpurun_out/bq_dw10_$m.jsonl 2> gpurun_out/bq_dw10_$m.err || { tail -20 gpurun_out/bq_dw10_$m.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bq_dw10_$m.jsonl'):
    d=json.loads(l); print('$m', d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'], d.get('diag_W',{}).get('top_norm'), d.get('diag_W',{}).get('top_rate_rank'), d.get('diag_C',{}).get('top_norm'), d.get('diag_C',{}).get('top_rate_rank'))"
done
