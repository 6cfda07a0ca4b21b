set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/block_rate.py --model line2 --config c4 --nparts 2 4 8 --parts 0 3 > gpurun_out/block_rate_c4.jsonl 2> gpurun_out/block_rate_c4.err || { tail -30 gpurun_out/block_rate_c4.err; exit 1; }
cat gpurun_out/block_rate_c4.jsonl
timeout -k 10 400 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 2 4 8 --parts 0 > gpurun_out/block_rate_c5.jsonl 2> gpurun_out/block_rate_c5.err || { tail -30 gpurun_out/block_rate_c5.err; exit 1; }
cat gpurun_out/block_rate_c5.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_blocks.py -x -v -s --timeout 500 --timeout-method thread -k "quality" > gpurun_out/blocks_quality.log 2>&1 || { echo QFAIL; grep -E "C2|assert|Error" gpurun_out/blocks_quality.log | tail -20; exit 1; }
grep -E "C2|passed|failed" gpurun_out/blocks_quality.log
