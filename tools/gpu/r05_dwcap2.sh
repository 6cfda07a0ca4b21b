set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1024 768; do
timeout -k 10 600 env SMORE_CELL_RATE=$r python -u tools/block_rate.py --model deepwalk --config c5 --nparts 4 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bdw_$r.jsonl 2> gpurun_out/bdw_$r.err || { tail -20 gpurun_out/bdw_$r.err; exit 1; }
python tools/block_sim.py gpurun_out/bdw_$r.jsonl | sed "s/^/cap$r /" | cut -c1-260
timeout -k 10 600 env SMORE_CELL_RATE=$r python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 4 8 --totals 10 > gpurun_out/qdw_$r.jsonl 2> gpurun_out/qdw_$r.err || { tail -20 gpurun_out/qdw_$r.err; exit 1; }
python -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print('cap', sys.argv[2], d['ranks'], d['loss'], d['auc'])" gpurun_out/qdw_$r.jsonl $r
done
