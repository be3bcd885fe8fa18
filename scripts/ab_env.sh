#!/bin/bash
# A/B of an on/off environment switch on the warm graphed SF100 suite, tables
# in HBM, same box back to back (VALS, default 1 0 1 0):
#   VAR=IGLOO_DEBUG VALS="like_nodword none like_nodword none" QS=13 bash scripts/ab_env.sh
#   -> gpurun_out/ab_$VAR.txt (IGLOO_DEBUG tokens: like_nodword, having_general, ff_mfma, ...;
#   an unknown token such as "none" is the default path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
VAR=${VAR:?set VAR}
OUT=gpurun_out/ab_$VAR.txt
: > $OUT
for v in ${VALS:-1 0 1 0}; do
  env $VAR=$v timeout -k 10 400 python3 bench.py --source hbm --sf ${SF:-100} --queries ${QS:-1-22} --steps ${STEPS:-10} \
    --warmup 3 --eager-steps 0 --vary-params 0 --per-query > gpurun_out/ab_${VAR}_$v.log 2>&1 || exit $?
  echo "$VAR=$v $(tail -1 gpurun_out/ab_${VAR}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $OUT
  echo "  $(grep -o 'Q[0-9][0-9] *[0-9.]* ms' gpurun_out/ab_${VAR}_$v.log | awk '{printf "%s=%s ", $1, $2}')" >> $OUT
done
cat $OUT
