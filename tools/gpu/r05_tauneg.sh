set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for tn in 1.0 3.0; do
timeout -k 10 600 env SMORE_CELL_TAU_NEG=$tn python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --ranks 4 8 > gpurun_out/tn_$tn.jsonl 2> gpurun_out/tn_$tn.err || { tail -20 gpurun_out/tn_$tn.err; exit 1; }
python -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print('tauneg', sys.argv[2], d['ranks'], d['loss'], d['auc'])" gpurun_out/tn_$tn.jsonl $tn
timeout -k 10 600 env SMORE_CELL_TAU_NEG=$tn python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/btn_$tn.jsonl 2> gpurun_out/btn_$tn.err || { tail -20 gpurun_out/btn_$tn.err; exit 1; }
python tools/block_sim.py gpurun_out/btn_$tn.jsonl | sed "s/^/tauneg$tn /" | cut -c1-300
done
