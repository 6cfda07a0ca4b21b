set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
for b in 12288 9216; do
  timeout -k 10 600 env SMORE_SH_BUDGET=$b python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --ranks 8 > gpurun_out/bq_$b.jsonl 2> gpurun_out/bq_$b.err || { tail -20 gpurun_out/bq_$b.err; exit 1; }
  show gpurun_out/bq_$b.jsonl budget$b
  timeout -k 10 600 env SMORE_SH_BUDGET=$b python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bb_$b.jsonl 2> gpurun_out/bb_$b.err || { tail -20 gpurun_out/bb_$b.err; exit 1; }
  python tools/block_sim.py gpurun_out/bb_$b.jsonl | sed "s/^/budget$b /"
done
