#!/bin/bash
# rocprofv3 kernel trace of the warm SF100 suite with query graphs; summaries
# of the timed steps only (IGLOO_PROF_GAP idle gap before them).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp IGLOO_PROF_GAP=1
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_graphs" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 5 > gpurun_out/prof_graphs.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_graphs.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
T=$(find gpurun_out/prof_graphs -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$T" --steps 3 --top 40 > gpurun_out/r2_graphs_kernel_summary.txt
python3 scripts/aten_share.py "$T" --steps 3 > gpurun_out/r2_graphs_aten_share.txt
head -3 gpurun_out/r2_graphs_kernel_summary.txt; head -3 gpurun_out/r2_graphs_aten_share.txt
rm -f "$T"
