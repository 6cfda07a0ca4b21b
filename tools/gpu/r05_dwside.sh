set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 env SMORE_SH_DEBUG=1 SMORE_CELL_SIDE=c python -u tools/block_rate.py --model deepwalk --config c5 --nparts 8 --parts 0 1 2 3 4 5 6 7 --skip-one > gpurun_out/bdws.jsonl 2> gpurun_out/bdws.err || { tail -20 gpurun_out/bdws.err; exit 1; }
grep "\[cell\] part 5/8" gpurun_out/bdws.err | head -4
python -c "
import json
for l in open('gpurun_out/bdws.jsonl'):
    d=json.loads(l); print(d['part'], round(sum(c[2] for c in d['cells']),1), d['prepare_ms'])"
timeout -k 10 600 env SMORE_CELL_SIDE=c python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 4 8 --totals 10 > gpurun_out/qdws.jsonl 2> gpurun_out/qdws.err || { tail -20 gpurun_out/qdws.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/qdws.jsonl'): d=json.loads(l); print('side c', d['ranks'], d['loss'], d['auc'])"
