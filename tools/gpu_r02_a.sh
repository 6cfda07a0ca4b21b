# round-2 GPU check: the -m gpu suite, then a short bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed" gpurun_out/gputest.log | tail -3
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_models.py --configs c2 c3 c5 > gpurun_out/models.log 2>&1
