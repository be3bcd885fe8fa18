#!/bin/bash
# One rocprofv3 counter pass over selected TPC-H queries (kernel-trace only, no
# runtime/sys trace). usage: QUERIES=1 PMC="SQ_WAVES SQ_INSTS_VALU ..." bash scripts/pmc_query.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -s KILL 300 rocprofv3 --pmc ${PMC} --output-format csv -d "$R/gpurun_out/pmc" -o run -- \
  python3 "$R/bench.py" --sf ${SF:-100} --steps 1 --warmup 1 --queries ${QUERIES:-1} > gpurun_out/pmc.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
