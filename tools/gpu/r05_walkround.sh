set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 4 8 --parts 0 1 2 3 4 5 6 7 --walks 1048576 > gpurun_out/bw20.jsonl 2> gpurun_out/bw20.err || { tail -20 gpurun_out/bw20.err; exit 1; }
python tools/block_sim.py gpurun_out/bw20.jsonl
python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    if d.get('part')==0 or d['nparts']==1: print(d['nparts'], d['epoch_ms'], d.get('prepare_ms'), [c[2] for c in d.get('cells',[])])" gpurun_out/bw20.jsonl
