set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C="TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d gpurun_out/cpmc_cells -o run -- python3 tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 --reps 1 --skip-one > gpurun_out/cpmc_cells.log 2>&1 || { tail -20 gpurun_out/cpmc_cells.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d gpurun_out/cpmc_one -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pmc off > gpurun_out/cpmc_one.log 2>&1 || { tail -20 gpurun_out/cpmc_one.log; exit 1; }
find gpurun_out/cpmc_cells gpurun_out/cpmc_one -name "*counter_collection.csv" | head
