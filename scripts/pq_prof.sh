#!/bin/bash
# rocprofv3 kernel stats of a cold GPU Parquet scan (SF${SF:-10} TPC-H tables).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$R/gpurun_out/pqprof" -o run -- \
  python3 "$R/scripts/parquet_scan_bench.py" --sf ${SF:-10} --no-host --queries 1 > gpurun_out/pqprof.log 2>&1
rc=$?; echo "pqprof rc=$rc"; grep -E "^\[scan\]|\[write\]" gpurun_out/pqprof.log | cut -c1-400
head -25 gpurun_out/pqprof/*/*/run_kernel_stats.csv 2>/dev/null || find gpurun_out/pqprof -name "*stats*"
exit $rc
