#!/bin/bash
# MFMA vs VALU hash / compare A/B (csrc/kernels/mfma_probe.hip): timings,
# then one rocprofv3 counter pass per counter group over the same script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/mfma_hash_ab.py > gpurun_out/mfma_hash_ab_times.json 2> gpurun_out/mfma_hash_ab.err || exit $?
for pmc in "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pmc | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --stats -d gpurun_out/mfma_pmc_$tag -o run \
    -- python3 scripts/mfma_hash_ab.py --reps 3 > gpurun_out/mfma_pmc_$tag.log 2>&1 || exit $?
done
echo done
