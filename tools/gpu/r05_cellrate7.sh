set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/cr7_$tag.jsonl 2> gpurun_out/cr7_$tag.err || { tail -20 gpurun_out/cr7_$tag.err; exit 1; }
  show gpurun_out/cr7_$tag.jsonl $tag
}
br() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/br7_$tag.jsonl 2> gpurun_out/br7_$tag.err || { tail -20 gpurun_out/br7_$tag.err; exit 1; }
  python tools/block_sim.py gpurun_out/br7_$tag.jsonl | sed "s/^/$tag /"
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d.get('part')==0: print(d['nparts'], [c[2] for c in d['cells']])" gpurun_out/br7_$tag.jsonl
}
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --hot-tau 0.3"
BR="python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 --hot-tau 0.3"
run b24k SMORE_CELL_RATE=0 SMORE_SH_BUDGET=24576 $LN --ranks 8
br b24k SMORE_CELL_RATE=0 SMORE_SH_BUDGET=24576 $BR
