#!/bin/bash
# One rocprofv3 counter pass (--kernel-trace + --pmc only) over the warm
# graphed suite of the queries in QS at SF (tables in HBM); per-kernel counter
# table for kernels matching KF.   QS="13" KF=like_seg PMC="SQ_WAVES ..." bash scripts/pmc_one.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
PMC="${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS}"
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d "$R/gpurun_out/pmc1" -o run -- \
  python3 "$R/bench.py" --source hbm --sf ${SF:-100} --queries ${QS:-13} --steps 1 --warmup 3 --eager-steps 0 \
  --vary-params 0 > gpurun_out/pmc1.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pmc1 -name "*counter_collection.csv" | head -1)
python3 - "$f" "${KF:-.}" "$PMC" > gpurun_out/pmc1_summary.txt <<'PY'
import csv, re, sys, collections
f, kf, names = sys.argv[1], sys.argv[2], sys.argv[3].split()
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r.get("Kernel_Name", "")
    if not re.search(kf, k):
        continue
    k = k.replace("(anonymous namespace)::", "")
    key = k.split("(")[0].replace("void ", "")[-100:]
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[(key, r["Counter_Name"])] += 1
print("kernel | " + " ".join(names))
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:20]:
    print(k, f"calls={calls[(k, names[0])]}", "|", " ".join(f"{d.get(n, 0):.4g}" for n in names))
PY
cat gpurun_out/pmc1_summary.txt | head -30
rm -rf gpurun_out/pmc1
