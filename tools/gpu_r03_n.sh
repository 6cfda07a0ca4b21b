#!/bin/bash
# round-3 GPU session N: source partition (library + dist.py + bench) -- the
# multi-rank tests, the partition draw test, bench.py's N > 1 path rehearsed
# with gloo ranks on the one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export MASTER_ADDR=127.0.0.1
bash tools/gpu_session.sh \
  "tests_multi 900 python -u -m pytest -v -s --timeout 900 --timeout-method thread -m gpu tests/test_gpu_multi.py" \
  "bench_n2_c4_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo" \
  "bench_n4_c2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --config c2"
