set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -x -v --timeout 300 --timeout-method thread -k "not quality" > gpurun_out/blocks_tests.log 2>&1 || { echo TESTFAIL; tail -50 gpurun_out/blocks_tests.log; exit 1; }
tail -5 gpurun_out/blocks_tests.log
timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 2 4 8 --parts 0 > gpurun_out/block_rate_c4.jsonl 2> gpurun_out/block_rate_c4.err || { tail -30 gpurun_out/block_rate_c4.err; exit 1; }
cat gpurun_out/block_rate_c4.jsonl
