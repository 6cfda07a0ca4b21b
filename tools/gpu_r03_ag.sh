#!/bin/bash
# round-3 GPU session AG: bench.py's N>1 path at HEAD rehearsed with gloo ranks sharing the GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "bench_n2_c4_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --dist-backend gloo" \
  "bench_n4_c2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 3 --warmup 1 --dist-backend gloo --config c2"
