set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_speculation_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graphs.log 2>&1 && \
timeout -k 10 240 python -u bench.py --sf 1 --steps 5 --warmup 1 --per-query > gpurun_out/bench_sf1.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?
echo "exit $rc"
tail -4 gpurun_out/pytest_graphs.log
tail -1 gpurun_out/bench_sf1.log | cut -c1-300
tail -1 gpurun_out/bench_sf100.log | cut -c1-300
exit $rc
