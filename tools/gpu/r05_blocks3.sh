set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 1 8 --totals 31 --mode atomic > gpurun_out/bq_atomic.jsonl 2> gpurun_out/bq_atomic.err || { tail -20 gpurun_out/bq_atomic.err; exit 1; }
cat gpurun_out/bq_atomic.jsonl
timeout -k 10 500 python -u tools/replica_study.py --model line2 --config c2 --schedule blocks --ranks 1 8 --totals 31 --mode hybrid --per-row 13.42 --periods 0.25 4 > gpurun_out/bq_epoch.jsonl 2> gpurun_out/bq_epoch.err || { tail -20 gpurun_out/bq_epoch.err; exit 1; }
cat gpurun_out/bq_epoch.jsonl
mkdir -p gpurun_out/kt8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt8 -o run --output-format csv -- python tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 --reps 1 > gpurun_out/kt8/rate.jsonl 2> gpurun_out/kt8/rate.err || { tail -20 gpurun_out/kt8/rate.err; exit 1; }
cat gpurun_out/kt8/rate.jsonl
find gpurun_out/kt8 -name "*kernel_stats.csv" | head -3
