set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in "--mode atomic --periods 1 4" "--mode hybrid --hot-tau 0.3 --periods 1" "--mode hybrid --hot-tau 0.1 --periods 1"; do
timeout -k 10 600 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 8 --totals 31 --per-row 13.42 $a >> gpurun_out/bq5.jsonl 2>> gpurun_out/bq5.err || { tail -20 gpurun_out/bq5.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/bq5.jsonl'):
    d=json.loads(l); print(d['ranks'], d['mode'], d['hot_tau'], d['period'], d['loss'], d['wall_s'])"
for t in 0.3 0.1; do
timeout -k 10 300 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 --hot-tau $t > gpurun_out/block_rate_c4_tau$t.jsonl 2> gpurun_out/block_rate_c4_tau$t.err || { tail -30 gpurun_out/block_rate_c4_tau$t.err; exit 1; }
cut -c1-300 gpurun_out/block_rate_c4_tau$t.jsonl
done
