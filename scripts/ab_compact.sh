#!/bin/bash
# A/B of the fused scan compaction (IGLOO_COMPACT=1, default) against mask ->
# indices -> gather (IGLOO_COMPACT=0) on the warm graphed SF100 suite, tables
# in HBM, same box back to back.   bash scripts/ab_compact.sh -> gpurun_out/ab_compact.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/ab_compact.txt
for v in 1 0 1 0; do
  IGLOO_COMPACT=$v timeout -k 10 400 python3 bench.py --source hbm --sf ${SF:-100} --steps ${STEPS:-10} --warmup 3 \
    --eager-steps 0 --vary-params 0 > gpurun_out/ab_compact_$v.log 2>&1 || exit $?
  echo "IGLOO_COMPACT=$v $(tail -1 gpurun_out/ab_compact_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')" >> gpurun_out/ab_compact.txt
done
cat gpurun_out/ab_compact.txt
