set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -v -s --timeout 600 --timeout-method thread -k "c2_line_group_defaults" > gpurun_out/c2def.log 2>&1; rc=$?; echo rc=$rc
grep -E "group [0-9]|PASS|FAIL" gpurun_out/c2def.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 4 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bb_def.jsonl 2> gpurun_out/bb_def.err || { tail -20 gpurun_out/bb_def.err; exit 1; }
python tools/block_sim.py gpurun_out/bb_def.jsonl | sed "s/^/default /"
timeout -k 10 600 env SMORE_SH_BUDGET=16384 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --totals 31 --per-row 0 --ranks 8 > gpurun_out/bq_16384.jsonl 2> gpurun_out/bq_16384.err || { tail -20 gpurun_out/bq_16384.err; exit 1; }
cat gpurun_out/bq_16384.jsonl | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('b16384', d['ranks'], d['loss'], d['auc'])"
timeout -k 10 600 env SMORE_SH_BUDGET=16384 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 > gpurun_out/bb_16384.jsonl 2> gpurun_out/bb_16384.err || { tail -20 gpurun_out/bb_16384.err; exit 1; }
python tools/block_sim.py gpurun_out/bb_16384.jsonl | sed "s/^/b16384 /"
