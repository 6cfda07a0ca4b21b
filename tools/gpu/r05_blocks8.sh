set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "--combine-rows 0" "--combine-rows 32" "--mode atomic"; do
timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 4 --reps 1 $a > gpurun_out/br8.jsonl 2> gpurun_out/br8.err || { tail -30 gpurun_out/br8.err; exit 1; }
echo "$a"; cut -c1-900 gpurun_out/br8.jsonl
done
timeout -k 10 900 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 1 2 4 8 --totals 10 > gpurun_out/bq_dw.jsonl 2> gpurun_out/bq_dw.err || { tail -20 gpurun_out/bq_dw.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bq_dw.jsonl'):
    d=json.loads(l); print(d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])"
