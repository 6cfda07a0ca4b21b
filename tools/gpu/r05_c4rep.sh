set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/replica_study.py --model line2 --config c4 --schedule blocks --totals 34 --per-row 0 --ranks 2 4 > gpurun_out/c4q_b24.jsonl 2> gpurun_out/c4q_b24.err || { tail -20 gpurun_out/c4q_b24.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c4q_b24.jsonl'): d=json.loads(l); print('blocks', d['ranks'], d['loss'], d['auc'], d['wall_s'], d.get('samples_per_exchange'))"
