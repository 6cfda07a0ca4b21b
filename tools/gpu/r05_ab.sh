set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ab() {
  tag=$1; dir=$2
  (cd $dir && timeout -k 10 300 python -u bench.py --steps 10 --pmc off --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/ab_$tag.json 2> $GRAFT_REPO_ROOT/gpurun_out/ab_$tag.err) || { tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['roofline']['kernel']; print(sys.argv[2], d['value'], k['ms_per_launch'], k['exposed_draw_ms_per_step'])" gpurun_out/ab_$tag.json $tag
}
ab new1 .
ab old1 ab_old
ab new2 .
ab old2 ab_old
