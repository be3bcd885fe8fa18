#!/bin/bash
# A/B of env-switchable code paths on ONE box: SF100 suite per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for cfg in "${@:-IGLOO_NONE=1}"; do
  env $cfg timeout -k 10 300 python bench.py --sf ${SF:-100} --steps 3 --warmup 1 --per-query > gpurun_out/ab.log 2>&1 || exit 1
  echo "$cfg $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -E "${QRE:-Q0[4579]|Q12|Q21}" gpurun_out/ab.log | awk '{print $2":"$3}' | tr '\n' ' ')"
done
