set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rehearsal
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --config c2 --steps 2 --warmup 1 --dist-backend gloo --no-cpu-baseline --pmc off > gpurun_out/rehearsal/bench_n8_c2_gloo.json 2> gpurun_out/rehearsal/bench_n8_c2_gloo.err || { tail -30 gpurun_out/rehearsal/bench_n8_c2_gloo.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/rehearsal/bench_n8_c2_gloo.json').read().strip().splitlines()[-1]); print(d['value'], d['config']['parallelism'], d['ms_per_step'], json.dumps(d['setup'])[:600])"
