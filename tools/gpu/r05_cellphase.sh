set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for t in default 1.0; do
  if [ $t = default ]; then A=""; else A="--hot-tau $t"; fi
  timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 $A > gpurun_out/bp_$t.jsonl 2> gpurun_out/bp_$t.err || { tail -20 gpurun_out/bp_$t.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d['nparts']==1: print(sys.argv[2], 'one', d['epoch_ms'], d['draw_update_ms'])
    else: print(sys.argv[2], [c[2:] for c in d['cells']])" gpurun_out/bp_$t.jsonl $t
done
