set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/final/gputest_full.txt 2>&1; rc=$?; echo gpu_rc=$rc
tail -1 gpurun_out/final/gputest_full.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench_c4.json 2> gpurun_out/final/bench_c4.err || { tail -20 gpurun_out/final/bench_c4.err; exit 1; }
tail -1 gpurun_out/final/bench_c4.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o c4 --output-format csv -- python3 bench.py --steps 10 --pmc off --no-cpu-baseline > gpurun_out/final/c4_prof.log 2>&1 || { tail -20 gpurun_out/final/c4_prof.log; exit 1; }
head -3 gpurun_out/final/prof/c4_kernel_stats.csv
timeout -k 10 900 python -u tools/block_rate.py --model line2 --config c4 --nparts 2 4 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/final/cells_c4.jsonl 2> gpurun_out/final/cells_c4.err || { tail -20 gpurun_out/final/cells_c4.err; exit 1; }
python tools/block_sim.py gpurun_out/final/cells_c4.jsonl
