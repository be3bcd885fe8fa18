#!/bin/bash
# rocprofv3 kernel summary of the timed steps of selected queries (QS) at SF100
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp IGLOO_PROF_GAP=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_q" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 5 --queries "${QS:-9}" > gpurun_out/prof_q.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
T=$(find gpurun_out/prof_q -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$T" --steps 3 --top 25 > gpurun_out/prof_q_summary.txt
rm -f "$T"
cat gpurun_out/prof_q_summary.txt | cut -c1-200
