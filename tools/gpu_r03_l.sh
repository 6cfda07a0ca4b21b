#!/bin/bash
# round-3 GPU session L: bench.py's N > 1 path rehearsed with gloo ranks
# sharing the one GPU (the driver's SCALE run uses RCCL on 8 GPUs), new
# exchange tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export MASTER_ADDR=127.0.0.1
bash tools/gpu_session.sh \
  "tests_ex 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multi.py -k world1 tests/test_gpu_configs.py -k exchange" \
  "bench_n2_c4_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo" \
  "bench_n4_c2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --config c2"
