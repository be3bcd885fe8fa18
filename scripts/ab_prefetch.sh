#!/bin/bash
# Morsel prefetch A/B under a 1 GB device cap (SF10, all 22 queries, GPU reference)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for p in 0 1; do
  IGLOO_MORSEL_PREFETCH=$p timeout -k 10 500 python -u scripts/budget_check.py --sf ${SF:-10} --cap-gb 1 --budget-gb 0.25 \
    --ref gpu > gpurun_out/ab_prefetch$p.log 2>&1
  rc=$?; echo "prefetch=$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep "^Q" gpurun_out/ab_prefetch$p.log | awk '{s+=$3} END {print "sum s", s}'
done
