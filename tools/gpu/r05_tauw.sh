set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for tw in 1.0 3.0; do
timeout -k 10 600 env SMORE_CELL_TAU_W=$tw python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --ranks 8 > gpurun_out/tw_$tw.jsonl 2> gpurun_out/tw_$tw.err || { tail -20 gpurun_out/tw_$tw.err; exit 1; }
python -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print('tauw', sys.argv[2], d['ranks'], d['loss'], d['auc'])" gpurun_out/tw_$tw.jsonl $tw
timeout -k 10 600 env SMORE_CELL_TAU_W=$tw python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/btw_$tw.jsonl 2> gpurun_out/btw_$tw.err || { tail -20 gpurun_out/btw_$tw.err; exit 1; }
python tools/block_sim.py gpurun_out/btw_$tw.jsonl | sed "s/^/tauw$tw /"
done
