#!/bin/bash
# One GPU session: new-kernel tests first, then the GPU suite, the SF100
# Parquet bench and a rocprofv3 kernel-stats pass over the warm steps.
# Each step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
if [ -n "$FIRST" ]; then
  timeout -k 10 400 $T $FIRST > gpurun_out/first.log 2>&1; rc=$?; echo "first rc=$rc"; tail -15 gpurun_out/first.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOSUITE" ]; then
  timeout -k 10 700 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py --sf ${SF:-100} --steps ${STEPS:-5} --warmup ${WARM:-1} --per-query > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; grep -E "cold suite|Q[0-9]" gpurun_out/bench.log | tr '\n' ' '; echo; tail -1 gpurun_out/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  R="$(pwd)"
  IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- \
    python3 "$R/bench.py" --sf ${SF:-100} --steps 2 --warmup 1 > gpurun_out/prof.log 2>&1; rc=$?
  echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  TR=$(find gpurun_out/prof -name "*kernel_trace.csv" | sort | tail -n 1)
  python3 scripts/kernel_summary.py "$TR" --steps 2 --top 45 > gpurun_out/kernel_summary.txt 2>&1
  cp gpurun_out/prof/*/*/*kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null; head -48 gpurun_out/kernel_summary.txt
fi
if [ -n "$HOSTPROF" ]; then
  timeout -k 10 300 python scripts/host_profile.py --sf ${HOSTPROF} --top 60 > gpurun_out/host_profile.txt 2>&1; rc=$?
  echo "hostprof rc=$rc"; head -5 gpurun_out/host_profile.txt; [ $rc -eq 0 ] || exit $rc
fi
