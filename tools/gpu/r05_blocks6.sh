set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/block_rate.py --model line2 --config c4 --nparts 8 --parts 0 1 2 3 4 5 6 7 --reps 1 > gpurun_out/block_cells_c4_n8.jsonl 2> gpurun_out/block_cells_c4_n8.err || { tail -30 gpurun_out/block_cells_c4_n8.err; exit 1; }
cut -c1-250 gpurun_out/block_cells_c4_n8.jsonl
