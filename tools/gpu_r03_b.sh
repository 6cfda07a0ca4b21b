#!/bin/bash
# round-3 GPU session B: the float4 row layout -- full GPU suite, bench variants, replica-exchange simulation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
steps=("gputest 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k \"not n_ranks\""
       "bench_uc 300 python -u bench.py --no-cpu-baseline"
       "bench_coarse 300 SMORE_TABLE_MEM=coarse python -u bench.py --no-cpu-baseline")
[ -f var/w3/libsmore_hip.so ] && steps+=("bench_w3 300 SMORE_LIB=var/w3/libsmore_hip.so python -u bench.py --no-cpu-baseline"
                                          "bench_w3_coarse 300 SMORE_TABLE_MEM=coarse SMORE_LIB=var/w3/libsmore_hip.so python -u bench.py --no-cpu-baseline")
steps+=("replica_sim 600 python -u tools/replica_sim.py --config c2 --ranks 1 2 4 8 --sync sum mean")
bash tools/gpu_session.sh "${steps[@]}"
