#!/bin/bash
# rocprofv3 kernel statistics for a subset of TPC-H queries at a given SF.
# usage: QUERIES=1,6 SF=100 bash scripts/prof_queries.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_q" -o run -- \
  python3 "$R/bench.py" --sf ${SF:-100} --steps ${STEPS:-2} --warmup 1 --queries ${QUERIES:-1,6} > gpurun_out/prof_q.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_q.log
f=$(find gpurun_out/prof_q -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python3 scripts/kernel_summary.py "$f" --steps ${STEPS:-2} --top ${TOP:-30} | tee gpurun_out/prof_q_summary.txt
exit $rc
