# round-2 GPU check: the -m gpu suite, a 2-rank gloo rehearsal of the N>1 bench
# path on one GPU, then the default bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/gputest.log | tail -3
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_gloo2.log 2>&1
echo "gloo2 rc=$?"
tail -1 gpurun_out/bench_gloo2.log | cut -c1-300
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
