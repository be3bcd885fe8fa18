#!/bin/bash
# Roofline of the warm graphed SF100 suite: three rocprofv3 passes, each with
# --kernel-trace and one counter group that fits the hardware limits (at most
# 4 TCC counters per pass: FETCH_SIZE needs 3 and WRITE_SIZE 2, so they take
# a pass each), merged per kernel by scripts/pmc_summary.py (bytes over the
# summed kernel time, % of 8 TB/s; VALU / LDS / MFMA instructions per wave).
#   SF=100 QS=1-22 [TAG=x] bash scripts/roofline.sh  -> gpurun_out/roofline[_x].txt
# (environment switches pass through, e.g. IGLOO_JIT=off IGLOO_DEBUG=ff_mfma TAG=mfma)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
SUF=${TAG:+_$TAG}
OUT="$R/gpurun_out/roofline$SUF"
rm -rf "$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  echo "pass $i: $grp"
  IGLOO_PROF_GAP=1 timeout -s KILL ${PASS_TIMEOUT:-420} rocprofv3 --kernel-trace --pmc $grp --output-format csv \
    -d "$OUT/p$i" -o run -- python3 "$R/bench.py" --source hbm --sf ${SF:-100} --queries ${QS:-1-22} --steps 1 \
    --warmup ${WARMUP:-3} --eager-steps 0 --vary-params 0 > "$R/gpurun_out/roofline${SUF}_p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 "$R/scripts/pmc_summary.py" "$OUT" --top ${TOP:-20} > "$R/gpurun_out/roofline$SUF.txt"
cat "$R/gpurun_out/roofline$SUF.txt"
rm -rf "$OUT"
