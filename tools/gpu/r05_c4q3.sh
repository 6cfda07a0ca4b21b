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
run b4096 SMORE_SH_BUDGET=4096 $Q
run b3072 SMORE_SH_BUDGET=3072 $Q
timeout -k 10 600 env SMORE_SH_BUDGET=4096 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bb_4096.jsonl 2> gpurun_out/bb_4096.err || { tail -20 gpurun_out/bb_4096.err; exit 1; }
python tools/block_sim.py gpurun_out/bb_4096.jsonl | sed "s/^/b4096 /" | cut -c1-300
