set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SMORE_SH_DEBUG=1 timeout -k 10 300 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 1 2 --totals 1 > gpurun_out/wd5_dbg.jsonl 2> gpurun_out/wd5_dbg.err || { tail -20 gpurun_out/wd5_dbg.err; exit 1; }
grep "\[sh\]" gpurun_out/wd5_dbg.err | sort | uniq -c | head -30
i=0
for st in 4096 512; do
i=$((i+1))
SMORE_SH_STALE=$st timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 2 --totals 10 > gpurun_out/wd5_$i.jsonl 2> gpurun_out/wd5_$i.err || { tail -20 gpurun_out/wd5_$i.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/wd5_$i.jsonl'):
    d=json.loads(l); print('stale $st', d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])"
done
