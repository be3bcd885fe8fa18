#!/bin/bash
# Kernel-level A/B of env-switchable scan paths (e.g. IGLOO_JIT=off vs sync,
# IGLOO_DEBUG=ff_mfma) on the SF100 scan queries: rocprofv3 kernel trace of
# the timed steps per configuration, summarised by scripts/kernel_summary.py.
# usage: bash scripts/ff_ab.sh "IGLOO_JIT=off" "IGLOO_JIT=sync"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
i=0
for cfg in "${@:-IGLOO_NONE=1}"; do
  i=$((i+1))
  rm -rf "$R/gpurun_out/ffab$i"
  env IGLOO_PROF_GAP=1 $cfg timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d "$R/gpurun_out/ffab$i" -o run -- python3 "$R/bench.py" --sf ${SF:-100} --source ${SRC:-hbm} \
    --queries ${QS:-1,6,12,14,19} --steps 5 --warmup ${WARM:-1} --per-query > "$R/gpurun_out/ffab$i.log" 2>&1 || exit 1
  TR=$(find "$R/gpurun_out/ffab$i" -name "*kernel_trace.csv" | sort | tail -n 1)
  echo "== $cfg $(grep -E '^\[bench\] Q' "$R/gpurun_out/ffab$i.log" | awk '{print $2":"$3}' | tr '\n' ' ')"
  python3 scripts/kernel_summary.py "$TR" --steps 5 --top ${TOP:-12} | tee "$R/gpurun_out/ffab$i.txt"
done
