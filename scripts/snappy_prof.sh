#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp; R="$(pwd)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/snp" -o run -- \
  python3 "$R/scripts/snappy_bench.py" --sf ${SF:-10} --reps 2 > gpurun_out/snp.log 2>&1
rc=$?; echo "rc=$rc"; grep rep gpurun_out/snp.log | cut -c1-200
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/snp/**/*kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {r['Calls']:>5} {r['Name'][:80]}")
PY
exit $rc
