#!/bin/bash
# One GPU session: tests, then short benches. Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:randomly > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
for sf in ${BENCH_SFS:-1 10}; do
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --sf $sf --steps 2 --warmup 1 --per-query > gpurun_out/bench_sf$sf.log 2>&1
  rc=$?; echo "bench sf=$sf rc=$rc"; tail -30 gpurun_out/bench_sf$sf.log
  [ $rc -eq 0 ] || exit $rc
done
