#!/bin/bash
# Iteration loop on the GPU box: kernel/query tests, SF100 bench, EXPLAIN ANALYZE.
# Stops at the first failure (each GPU step has its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:randomly > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --sf ${SF:-100} --steps 2 --warmup 1 --per-query > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -26 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$EXPLAIN" ]; then
  timeout -k 10 500 python scripts/explain_queries.py --sf ${SF:-100} --queries $EXPLAIN > gpurun_out/explain.log 2>&1
  rc=$?; echo "explain rc=$rc"; grep -E "^=====|^total" gpurun_out/explain.log; exit $rc
fi
