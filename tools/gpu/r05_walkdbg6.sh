set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
show() { python -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['ranks'], d['schedule'], d['loss'], d['auc'], d['wall_s'])" "$@"; }
timeout -k 10 600 python -u tools/replica_study.py --model deepwalk --config c5 --schedule blocks --ranks 1 2 4 8 --totals 10 > gpurun_out/wd6_dw.jsonl 2> gpurun_out/wd6_dw.err || { tail -20 gpurun_out/wd6_dw.err; exit 1; }
show gpurun_out/wd6_dw.jsonl dw
SMORE_SH_DEBUG=1 timeout -k 10 600 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 1 8 --totals 31 --per-row 0 > gpurun_out/wd6_l0.jsonl 2> gpurun_out/wd6_l0.err || { tail -20 gpurun_out/wd6_l0.err; exit 1; }
show gpurun_out/wd6_l0.jsonl line-default
grep "\[sh\]" gpurun_out/wd6_l0.err | sort | uniq -c | sort -rn | head -24
i=0
for st in 8192 2048; do
i=$((i+1))
SMORE_SH_STALE=$st timeout -k 10 600 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 8 --totals 31 --per-row 0 > gpurun_out/wd6_l$i.jsonl 2> gpurun_out/wd6_l$i.err || { tail -20 gpurun_out/wd6_l$i.err; exit 1; }
show gpurun_out/wd6_l$i.jsonl line-stale$st
done
