#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
for q in 3 5 7 8 9 12 14 19; do
  QUERIES=$q SF=100 TOP=8 STEPS=1 bash scripts/prof_queries.sh > gpurun_out/pq_$q.log 2>&1 || exit 1
  echo "== Q$q"; head -10 gpurun_out/prof_q_summary.txt
done
