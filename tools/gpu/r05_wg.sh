set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/wg_$tag.jsonl 2> gpurun_out/wg_$tag.err || { tail -20 gpurun_out/wg_$tag.err; exit 1; }
  show gpurun_out/wg_$tag.jsonl $tag
}
br() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/brwg_$tag.jsonl 2> gpurun_out/brwg_$tag.err || { tail -20 gpurun_out/brwg_$tag.err; exit 1; }
  head -1 gpurun_out/brwg_$tag.jsonl
  python tools/block_sim.py gpurun_out/brwg_$tag.jsonl | sed "s/^/$tag /"
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d.get('part')==0: print(d['nparts'], [c[2] for c in d['cells']])" gpurun_out/brwg_$tag.jsonl
}
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --hot-tau 0.3"
BR="python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 --hot-tau 0.3"
br wg512 SMORE_CELL_RATE=0 SMORE_EDGE_WG=512 $BR
run wg512 SMORE_CELL_RATE=0 SMORE_EDGE_WG=512 $LN --ranks 1 8
timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 2 --parts 0 > gpurun_out/brwg_one256.jsonl 2>&1 && head -1 gpurun_out/brwg_one256.jsonl
SMORE_EDGE_WG=512 timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 2 --parts 0 > gpurun_out/brwg_one512.jsonl 2>&1 && head -1 gpurun_out/brwg_one512.jsonl
