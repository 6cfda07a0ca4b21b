set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bpr_quality.py --log2-total 28 --variants atomic hybrid hogwild hybrid@4 hybrid@16 > gpurun_out/bpr_q.jsonl 2> gpurun_out/bpr_q.err || { tail -20 gpurun_out/bpr_q.err; exit 1; }
cut -c1-250 gpurun_out/bpr_q.jsonl
timeout -k 10 600 python -u tools/bench_models.py --configs c3 --mode hogwild > gpurun_out/bpr_hog.jsonl 2> gpurun_out/bpr_hog.err || { tail -20 gpurun_out/bpr_hog.err; exit 1; }
cut -c1-400 gpurun_out/bpr_hog.jsonl
