set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/cr6_$tag.jsonl 2> gpurun_out/cr6_$tag.err || { tail -20 gpurun_out/cr6_$tag.err; exit 1; }
  show gpurun_out/cr6_$tag.jsonl $tag
}
br() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/br6_$tag.jsonl 2> gpurun_out/br6_$tag.err || { tail -20 gpurun_out/br6_$tag.err; exit 1; }
  python tools/block_sim.py gpurun_out/br6_$tag.jsonl | sed "s/^/$tag /"
}
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0"
BR="python -u tools/block_rate.py --model line2 --config c4 --nparts 4 8 --parts 0 1 2 3 4 5 6 7"
run tau05_nocap SMORE_CELL_RATE=0 $LN --ranks 8 --hot-tau 0.5
run tau03_nocap_n24 SMORE_CELL_RATE=0 $LN --ranks 1 2 4 --hot-tau 0.3
br tau03_nocap SMORE_CELL_RATE=0 $BR --hot-tau 0.3
br tau05_nocap SMORE_CELL_RATE=0 $BR --hot-tau 0.5
