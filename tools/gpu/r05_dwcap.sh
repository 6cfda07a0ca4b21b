set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
run() {
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/dc_$tag.jsonl 2> gpurun_out/dc_$tag.err || { tail -20 gpurun_out/dc_$tag.err; exit 1; }
  show gpurun_out/dc_$tag.jsonl $tag
}
DW="python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 8 --totals 10"
run atomic_nocap SMORE_CELL_RATE=0 $DW --mode atomic
run comb0_nocap SMORE_CELL_RATE=0 $DW --combine-rows 0
run comb0_cap1024 SMORE_CELL_RATE=1024 $DW --combine-rows 0
timeout -k 10 600 env SMORE_CELL_RATE=0 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 8 --parts 0 1 2 3 4 5 6 7 --combine-rows 0 > gpurun_out/bdc.jsonl 2> gpurun_out/bdc.err || { tail -20 gpurun_out/bdc.err; exit 1; }
python tools/block_sim.py gpurun_out/bdc.jsonl | sed "s/^/comb0_nocap /"
