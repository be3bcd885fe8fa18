#!/bin/bash
# SF100 headline bench + rocprofv3 kernel stats (SF10). Stops at first failure.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 ${SF100_TIMEOUT:-900} python bench.py --sf ${SF:-100} --steps 2 --warmup 1 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?; echo "bench sf100 rc=$rc"; tail -32 gpurun_out/bench_sf100.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_sf10" -o run -- \
  python3 "$R/bench.py" --sf 10 --steps 1 --warmup 1 > gpurun_out/prof_sf10.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 gpurun_out/prof_sf10.log
find gpurun_out/prof_sf10 -name "*stats*" | head
