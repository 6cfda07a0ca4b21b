set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rehearsal
true
true
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --no-cpu-baseline --pmc off > gpurun_out/rehearsal/bench_n4_gloo.json 2> gpurun_out/rehearsal/bench_n4_gloo.err || { tail -30 gpurun_out/rehearsal/bench_n4_gloo.err; exit 1; }
cat gpurun_out/rehearsal/bench_n4_gloo.json
