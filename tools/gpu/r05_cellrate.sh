set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {  # tag env... -- args
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/cr_$tag.jsonl 2> gpurun_out/cr_$tag.err || { tail -20 gpurun_out/cr_$tag.err; exit 1; }
  show gpurun_out/cr_$tag.jsonl $tag
}
DW="python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 8 --totals 10"
LN="python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 8 --totals 31 --per-row 0"
for r in 1024 512 256; do run dw_r$r SMORE_CELL_RATE=$r $DW; done
for b in 2048 1024; do run ln_b$b SMORE_SH_BUDGET=$b $LN; done
for r in 512 256; do run ln_r$r SMORE_CELL_RATE=$r $LN; done
