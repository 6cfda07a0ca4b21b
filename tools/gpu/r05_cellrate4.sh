set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/cr4_$tag.jsonl 2> gpurun_out/cr4_$tag.err || { tail -20 gpurun_out/cr4_$tag.err; exit 1; }
  show gpurun_out/cr4_$tag.jsonl $tag
}
br() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/br4_$tag.jsonl 2> gpurun_out/br4_$tag.err || { tail -20 gpurun_out/br4_$tag.err; exit 1; }
  python tools/block_sim.py gpurun_out/br4_$tag.jsonl | sed "s/^/$tag /"
}
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 8 --totals 31 --per-row 0"
BR="python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7"
run ln_c512 SMORE_CELL_SIDE=c SMORE_CELL_RATE=512 $LN
run ln_w512 SMORE_CELL_SIDE=w SMORE_CELL_RATE=512 $LN
run ln_768 SMORE_CELL_RATE=768 $LN
run ln_1024 SMORE_CELL_RATE=1024 $LN
br c4_c512 SMORE_SH_DEBUG=1 SMORE_CELL_SIDE=c SMORE_CELL_RATE=512 $BR
grep "\[cell\] part 0/8" gpurun_out/br4_c4_c512.err | head -16
br c4_768 SMORE_CELL_RATE=768 $BR
