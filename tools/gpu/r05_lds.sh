set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
b() {
  tag=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --steps 10 --pmc off --no-cpu-baseline $EXTRA > gpurun_out/lds_$tag.json 2> gpurun_out/lds_$tag.err || { tail -5 gpurun_out/lds_$tag.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['roofline']['kernel']; print(sys.argv[2], d['value'], k['ms_per_launch'], k['exposed_draw_ms_per_step'])" gpurun_out/lds_$tag.json $tag
}
EXTRA="" b base SMORE_SH_LDS=8192
EXTRA="--combine-rows 160" b r160 SMORE_SH_LDS=10240
EXTRA="" b base2 SMORE_SH_LDS=8192
timeout -k 10 600 env SMORE_SH_LDS=10240 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 --combine-rows 160 > gpurun_out/bl_160.jsonl 2> gpurun_out/bl_160.err || { tail -20 gpurun_out/bl_160.err; exit 1; }
python tools/block_sim.py gpurun_out/bl_160.jsonl | sed "s/^/rows160 /"
timeout -k 10 600 python -u tools/bench_models.py --configs c2 > gpurun_out/lds_c2_base.jsonl 2>/dev/null && cut -c1-300 gpurun_out/lds_c2_base.jsonl
