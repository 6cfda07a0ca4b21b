set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
true; rc=0
true
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --config c2 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --pmc off > gpurun_out/bench_n2_c2.json 2> gpurun_out/bench_n2_c2.err || { tail -20 gpurun_out/bench_n2_c2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/bench_n2_c2.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['roofline']['kernel']))"
