#!/bin/bash
# Same-box A/B of one or more switches (off = the OFF environment, on = the
# defaults). Box-to-box spread is several percent, so only same-box pairs are
# compared. Default command: the HBM SF100 suite with graphs.
#   OFF="IGLOO_DENSE_JOIN=0" bash scripts/ab_env.sh
#   OFF="IGLOO_MORSEL_PREFETCH=0" CMD="python -u scripts/budget_check.py --sf 10 --cap-gb 1 --budget-gb 0.25 --ref gpu" \
#     bash scripts/ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
CMD="${CMD:-python -u bench.py --source hbm --steps 10 --warmup 3 --eager-steps 0 --vary-params 0 --per-query}"
for mode in off on; do
  if [ $mode = off ]; then e="$OFF"; else e=""; fi
  env $e timeout -k 10 500 $CMD > gpurun_out/ab_env_$mode.log 2>&1
  rc=$?; echo "$mode ($e) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ab_env_$mode.log | cut -c1-120
  grep "\] Q[0-9]\|^Q[0-9]*:" gpurun_out/ab_env_$mode.log | awk '{printf "%s=%s ", $1 == "[bench]" ? $2 : $1, $1 == "[bench]" ? $3 : $3}'; echo
done
