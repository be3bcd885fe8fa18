#!/bin/bash
# Bounded-memory SPMD on the GPU: the world-1 RCCL path (IGLOO_FORCE_SPMD=1)
# over TPC-H SF10 in HBM, uncapped and under a 1 GB device budget
# (IGLOO_DEVICE_BUDGET_GB: morsel pipelines, streamed scans, grace joins);
# every query's result digest must agree.
#   bash scripts/spmd_budget_check.sh -> gpurun_out/spmd_budget.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
common="--source hbm --sf ${SF:-10} --steps 1 --warmup 0 --eager-steps 0 --vary-params 0 --per-query"
IGLOO_FORCE_SPMD=1 timeout -k 10 ${T:-400} python3 bench.py $common --digests-out gpurun_out/dig_free.json \
  > gpurun_out/spmd_free.log 2>&1 || exit $?
IGLOO_FORCE_SPMD=1 IGLOO_DEVICE_BUDGET_GB=${GB:-1} timeout -k 10 ${T:-400} python3 bench.py $common \
  --digests-out gpurun_out/dig_capped.json > gpurun_out/spmd_capped.log 2>&1 || exit $?
python3 - <<'PY' | tee gpurun_out/spmd_budget.txt
import json
a = json.load(open("gpurun_out/dig_free.json")); b = json.load(open("gpurun_out/dig_capped.json"))
bad = [q for q in a if a[q] != b.get(q)]
print(f"queries={len(a)} digest mismatches={bad}")
for tag, f in (("uncapped", "gpurun_out/spmd_free.log"), ("capped", "gpurun_out/spmd_capped.log")):
    for line in open(f):
        if "cold per query" in line or "cold suite" in line:
            print(tag, line.strip()[:400])
PY
