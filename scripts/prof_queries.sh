#!/bin/bash
# rocprofv3 kernel statistics for a subset of TPC-H queries at a given SF.
# usage: QUERIES=1,6 SF=100 bash scripts/prof_queries.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_q" -o run -- \
  python3 "$R/bench.py" --sf ${SF:-100} --steps 1 --warmup 1 --queries ${QUERIES:-1,6} > gpurun_out/prof_q.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_q.log
f=$(find gpurun_out/prof_q -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d}  {float(r["AverageNs"])/1e3:10.1f} us  {r["Name"][:110]}')
PY
exit $rc
