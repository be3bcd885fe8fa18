#!/bin/bash
# Same-box A/B of this session's query-path changes (HBM tables, SF100, graphs):
# off = fused HAVING, mid-size secondary-index joins and masked eager COUNT
# disabled through their switches; on = defaults. Box-to-box spread is
# several percent, so only same-box pairs are compared.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for mode in off on; do
  if [ $mode = off ]; then
    export IGLOO_SORTED_HAVING=0 IGLOO_PERM_INDEX_SORT_FRAC=20 IGLOO_EAGER_COUNT_MASKED=0
  else
    unset IGLOO_SORTED_HAVING IGLOO_PERM_INDEX_SORT_FRAC IGLOO_EAGER_COUNT_MASKED
  fi
  timeout -k 10 500 python -u bench.py --source hbm --steps 10 --warmup 3 --eager-steps 0 --vary-params 0 \
    --per-query > gpurun_out/ab_session_$mode.log 2>&1
  rc=$?; echo "$mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/ab_session_$mode.log | cut -c1-120
done
