#!/bin/bash
# MFMA A/B on the TPC-H scan aggregations (Q1: 4 groups x 8 aggregates, Q6:
# one global SUM) at SF100, tables in HBM:
#   A  the generated scan_agg kernel (exec/fused_jit.py; the default)
#   B  the one-hot MFMA kernel (csrc/kernels/fused.hip ff_mfma_agg_kernel,
#      v_mfma_i32_16x16x64_i8 over one-hot group ids x value byte limbs)
#   C  the interpreted LDS-slot kernel B replaces
# Per arm: a rocprofv3 kernel trace of the timed steps (scripts/ff_ab.sh) and
# one counter pass (SQ_INSTS_MFMA, SQ_INSTS_VALU, SQ_INSTS_LDS, SQ_WAVES,
# --kernel-trace only) summarised per kernel (scripts/pmc_summary.py).
# usage: bash scripts/mfma_ab.sh   -> gpurun_out/mfma_ab.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
OUT="$R/gpurun_out/mfma_ab.txt"
: > "$OUT"
QS=${QS:-1,6} bash scripts/ff_ab.sh "IGLOO_JIT=sync" "IGLOO_JIT=off IGLOO_DEBUG=ff_mfma" "IGLOO_JIT=off" \
  >> "$OUT" 2>&1 || exit 1
i=0
for cfg in "IGLOO_JIT=sync" "IGLOO_JIT=off IGLOO_DEBUG=ff_mfma" "IGLOO_JIT=off"; do
  i=$((i+1))
  rm -rf "$R/gpurun_out/mfmapmc$i"
  env IGLOO_PROF_GAP=1 $cfg timeout -s KILL 300 rocprofv3 --kernel-trace \
    --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv \
    -d "$R/gpurun_out/mfmapmc$i/p1" -o run -- python3 "$R/bench.py" --sf ${SF:-100} --source hbm \
    --queries ${QS:-1,6} --steps 1 --warmup 2 --eager-steps 0 --vary-params 0 \
    > "$R/gpurun_out/mfmapmc$i.log" 2>&1 || exit 1
  echo "== counters: $cfg" >> "$OUT"
  python3 scripts/pmc_summary.py "$R/gpurun_out/mfmapmc$i" --top 8 >> "$OUT" 2>&1
  rm -rf "$R/gpurun_out/mfmapmc$i"
done
rm -rf "$R"/gpurun_out/ffab[0-9]*/
cat "$OUT" | head -80
