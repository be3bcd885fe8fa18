#!/bin/bash
# rocprofv3 counter passes (each with kernel-trace only; no runtime/sys trace)
# over the warm TPC-H suite on tables generated in HBM, then a per-kernel
# roofline table (scripts/pmc_summary.py). One pass per counter set (the
# hardware cannot split counters over passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R="$(pwd)"
rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
i=0
while read -r SET; do
  [ -z "$SET" ] && continue
  i=$((i+1))
  IGLOO_PROF_GAP=1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run -- \
    python3 "$R/bench.py" --source hbm --sf ${SF:-100} --steps 1 --warmup 1 --queries ${QUERIES:-1-22} \
    > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($SET) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<SETS
${PMC_SETS:-FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES
WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_MFMA}
SETS
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; head -40 gpurun_out/pmc/summary.txt
