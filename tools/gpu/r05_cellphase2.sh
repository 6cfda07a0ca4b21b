set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in hogwild atomic comb0; do
  if [ $m = comb0 ]; then A="--combine-rows 0"; else A="--mode $m"; fi
  timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 $A > gpurun_out/bp_$m.jsonl 2> gpurun_out/bp_$m.err || { tail -20 gpurun_out/bp_$m.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d['nparts']==1: print(sys.argv[2], 'one', d['epoch_ms'], d['draw_update_ms'])
    else: print(sys.argv[2], [c[4] for c in d['cells']])" gpurun_out/bp_$m.jsonl $m
done
