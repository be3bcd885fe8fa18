#!/bin/bash
# A/B of an on/off environment switch on the ad-hoc (fresh substitution
# parameters) SF100 suite, tables in HBM, same box back to back:
#   VAR=IGLOO_TEMPLATE_REPLAY bash scripts/ab_adhoc.sh -> gpurun_out/ab_adhoc_$VAR.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
VAR=${VAR:?set VAR}
OUT=gpurun_out/ab_adhoc_$VAR.txt
: > $OUT
for v in ${VALS:-1 0 1 0}; do
  env $VAR=$v timeout -k 10 400 python3 bench.py --source hbm --sf ${SF:-100} --steps 2 --warmup 3 --eager-steps 0 \
    --vary-params ${STREAMS:-3} > gpurun_out/abad_${VAR}_$v.log 2>&1 || exit $?
  echo "$VAR=$v $(grep 'ad-hoc (fresh' gpurun_out/abad_${VAR}_$v.log | cut -c1-260)" >> $OUT
done
cat $OUT
