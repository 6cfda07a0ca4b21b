set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/c4q_$tag.jsonl 2> gpurun_out/c4q_$tag.err || { tail -20 gpurun_out/c4q_$tag.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]): d=json.loads(l); print(sys.argv[2], d['ranks'], d['loss'], d['auc'], d['wall_s'])" gpurun_out/c4q_$tag.jsonl $tag
}
Q="python -u tools/replica_study.py --model line2 --config c4 --schedule blocks --totals 34 --per-row 0 --ranks 8"
run atomic SMORE_CELL_RATE=0 $Q --mode atomic
run b6144 SMORE_SH_BUDGET=6144 $Q
run tau02 SMORE_CELL_RATE=0 $Q --hot-tau 0.2
