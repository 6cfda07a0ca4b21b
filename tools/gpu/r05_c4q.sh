set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u tools/replica_study.py --model line2 --config c4 --schedule blocks --totals 34 --per-row 0 --ranks 1 8 > gpurun_out/c4q_t03.jsonl 2> gpurun_out/c4q_t03.err || { tail -20 gpurun_out/c4q_t03.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c4q_t03.jsonl'): d=json.loads(l); print('c4 tau-default', d['ranks'], d['loss'], d['auc'], d['wall_s'])"
