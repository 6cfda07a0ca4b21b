set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rehearsal
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --pmc off > gpurun_out/rehearsal/bench_n4_gloo.json 2> gpurun_out/rehearsal/bench_n4_gloo.err || { tail -30 gpurun_out/rehearsal/bench_n4_gloo.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/rehearsal/bench_n4_gloo.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['parallelism'], json.dumps(d['setup']))"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline --pmc off > gpurun_out/rehearsal/bench_n1.json 2> gpurun_out/rehearsal/bench_n1.err || { tail -20 gpurun_out/rehearsal/bench_n1.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/rehearsal/bench_n1.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['setup']))"
