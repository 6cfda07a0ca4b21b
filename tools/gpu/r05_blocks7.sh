set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -x -q --timeout 300 --timeout-method thread -k "not quality" > gpurun_out/blocks_tests.log 2>&1 || { echo TESTFAIL; tail -50 gpurun_out/blocks_tests.log; exit 1; }
tail -2 gpurun_out/blocks_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --pmc off --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('C4', d['value'], d['roofline']['kernel']['ms_per_launch'])"
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --pmc off --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -20 gpurun_out/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2.json')); print('C2', d['value'], d['roofline']['kernel']['ms_per_launch'])"
timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 4 > gpurun_out/block_rate_c4_lvl.jsonl 2> gpurun_out/block_rate_c4_lvl.err || { tail -30 gpurun_out/block_rate_c4_lvl.err; exit 1; }
cat gpurun_out/block_rate_c4_lvl.jsonl
