set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
br() {  # tag env... -- args
  tag=$1; shift
  timeout -k 10 600 env "$@" > gpurun_out/br3_$tag.jsonl 2> gpurun_out/br3_$tag.err || { tail -20 gpurun_out/br3_$tag.err; exit 1; }
  python tools/block_sim.py gpurun_out/br3_$tag.jsonl | sed "s/^/$tag /"
}
BR="python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7"
br c4_coarse SMORE_TABLE_MEM=coarse python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0
python -c "
import json
for l in open('gpurun_out/br3_c4_coarse.jsonl'):
    d=json.loads(l); print('coarse', d.get('part'), d.get('cells'))"
br c4_cap512 SMORE_CELL_RATE=512 $BR
br c4_cap1024 SMORE_CELL_RATE=1024 $BR
br c4_cap0 SMORE_CELL_RATE=0 $BR
br c5_dw SMORE_CELL_RATE=512 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 8 --parts 0 1 2 3 4 5 6 7
