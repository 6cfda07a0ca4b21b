set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/replica_study.py --model line2 --config c4 --schedule replicas --totals 34 --ranks 8 > gpurun_out/c4q_rep.jsonl 2> gpurun_out/c4q_rep.err || { tail -20 gpurun_out/c4q_rep.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c4q_rep.jsonl'): d=json.loads(l); print('replicas', d['ranks'], d['loss'], d['auc'], d['wall_s'], d.get('samples_per_exchange'))"
