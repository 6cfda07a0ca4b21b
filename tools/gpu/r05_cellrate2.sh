set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_blocks.py -v -s --timeout 600 --timeout-method thread > gpurun_out/blocks_tests2.log 2>&1; rc=$?; echo blocks_rc=$rc
grep -E "PASS|FAIL|blocks [0-9]|Error|assert" gpurun_out/blocks_tests2.log | tail -30
[ $rc -le 1 ] || exit $rc
for rate in default 0; do
  if [ $rate = default ]; then E=""; else E="SMORE_CELL_RATE=$rate"; fi
  timeout -k 10 600 env $E python -u tools/block_rate.py --model line2 --config c4 --nparts 4 8 --parts 0 3 > gpurun_out/br_c4_$rate.jsonl 2> gpurun_out/br_c4_$rate.err || { tail -20 gpurun_out/br_c4_$rate.err; exit 1; }
  python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], {k:v for k,v in d.items() if k not in ('cells',)})" gpurun_out/br_c4_$rate.jsonl $rate
done
timeout -k 10 600 python -u tools/block_rate.py --model deepwalk --config c5 --nparts 4 8 --parts 0 > gpurun_out/br_c5.jsonl 2> gpurun_out/br_c5.err || { tail -20 gpurun_out/br_c5.err; exit 1; }
python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print('c5', {k:v for k,v in d.items() if k not in ('cells',)})" gpurun_out/br_c5.jsonl
