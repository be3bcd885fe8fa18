set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --per-query > gpurun_out/bench_sf100.log 2>&1
echo "exit $?"
tail -3 gpurun_out/pytest_gpu.log
tail -2 gpurun_out/bench_sf100.log | cut -c1-400
