set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/head
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head/smoke.log 2>&1 || { tail -20 gpurun_out/head/smoke.log; exit 1; }
tail -2 gpurun_out/head/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/head/bench_c4.json 2> gpurun_out/head/bench_c4.err || { tail -20 gpurun_out/head/bench_c4.err; exit 1; }
tail -1 gpurun_out/head/bench_c4.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/head/prof -o c4 --output-format csv -- python3 bench.py --steps 10 --pmc off --no-cpu-baseline > gpurun_out/head/c4_prof.log 2>&1 || { tail -20 gpurun_out/head/c4_prof.log; exit 1; }
find gpurun_out/head/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/head/prof_c3 -o c3 --output-format csv -- python3 tools/bench_models.py --configs c3 c2 > gpurun_out/head/c3c2_prof.log 2>&1 || { tail -20 gpurun_out/head/c3c2_prof.log; exit 1; }
grep "^{" gpurun_out/head/c3c2_prof.log | cut -c1-300
