#!/bin/bash
# Same-box A/B of one switch on the HBM SF100 suite (graphs):
#   OFF="IGLOO_X=0 IGLOO_Y=1" bash scripts/ab_env.sh     (on = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for mode in off on; do
  if [ $mode = off ]; then e="$OFF"; else e=""; fi
  env $e timeout -k 10 500 python -u bench.py --source hbm --steps 10 --warmup 3 --eager-steps 0 --vary-params 0 \
    --per-query ${QARGS} > gpurun_out/ab_env_$mode.log 2>&1
  rc=$?; echo "$mode ($e) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ab_env_$mode.log | cut -c1-120
  grep "\] Q[0-9]" gpurun_out/ab_env_$mode.log | awk '{printf "%s=%s ", $2, $3}'; echo
done
