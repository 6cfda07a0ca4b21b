set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --ranks 1 2 4 8 --hot-tau 0.4 > gpurun_out/bq_t04.jsonl 2> gpurun_out/bq_t04.err || { tail -20 gpurun_out/bq_t04.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bq_t04.jsonl'): d=json.loads(l); print('tau0.4', d['ranks'], d['loss'], d['auc'])"
timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 --hot-tau 0.4 > gpurun_out/bb_t04.jsonl 2> gpurun_out/bb_t04.err || { tail -20 gpurun_out/bb_t04.err; exit 1; }
python tools/block_sim.py gpurun_out/bb_t04.jsonl | sed "s/^/tau0.4 /" | cut -c1-300
