set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for a in "--mode hybrid" "--mode hybrid --combine-rows 0" "--mode hybrid --hot-tau 1000" "--mode hybrid --combine-rows 0 --hot-tau 1000" "--mode hogwild"; do
i=$((i+1))
timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 2 --totals 10 $a > gpurun_out/wd4_$i.jsonl 2> gpurun_out/wd4_$i.err || { tail -20 gpurun_out/wd4_$i.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/wd4_$i.jsonl'):
    d=json.loads(l); print('$a', d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])"
done
