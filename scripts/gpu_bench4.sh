set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_part.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 8 --warmup 5 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?
echo "exit $rc"
tail -2 gpurun_out/pytest_part.log
grep -E "cold suite|warmup|step|modes|graphs:|not captured" gpurun_out/bench_sf100.log | cut -c1-400 | sort | uniq -c | sort -rn | head -30
exit $rc
