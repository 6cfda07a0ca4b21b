set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/cr5_$tag.jsonl 2> gpurun_out/cr5_$tag.err || { tail -20 gpurun_out/cr5_$tag.err; exit 1; }
  show gpurun_out/cr5_$tag.jsonl $tag
}
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 8 --totals 31 --per-row 0"
run atomic_nocap SMORE_CELL_RATE=0 $LN --mode atomic
run atomic_cap512 SMORE_CELL_RATE=512 $LN --mode atomic
run tau03_nocap SMORE_CELL_RATE=0 $LN --hot-tau 0.3
run comb0_nocap SMORE_CELL_RATE=0 $LN --combine-rows 0
run tau03_comb0_nocap SMORE_CELL_RATE=0 $LN --combine-rows 0 --hot-tau 0.3
