#!/bin/bash
# rocprofv3 marker + kernel trace of a few warm SF10 queries with roctx ranges
# per query / operator / phase (IGLOO_DEBUG=roctx); summarised per range name.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
rm -rf "$R/gpurun_out/roctx"
IGLOO_DEBUG=roctx IGLOO_PROF_GAP=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv \
  -d "$R/gpurun_out/roctx" -o run -- python3 "$R/bench.py" --sf ${SF:-10} --source hbm --queries ${QS:-3,5,9} \
  --steps 1 --warmup 2 > "$R/gpurun_out/roctx.log" 2>&1 || exit 1
NQ=$(python3 -c "import sys; sys.path.insert(0, '$R'); from bench import parse_queries; print(len(parse_queries('${QS:-3,5,9}')))")
python3 - "$R/gpurun_out/roctx" "$NQ" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = (glob.glob(sys.argv[1] + "/**/*marker_api_trace.csv", recursive=True) or [None])[0]
if f is None:
    print("no marker trace"); sys.exit(0)
rows = list(csv.DictReader(open(f)))
print("columns:", list(rows[0].keys()) if rows else [])
agg = defaultdict(lambda: [0.0, 0])
for r in rows:
    name = r.get("Message") or r.get("Function") or "?"
    try:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    except (KeyError, ValueError):
        continue
    agg[name][0] += d
    agg[name][1] += 1
for k, (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"{ms:10.3f} ms {n:6d}  {k}")
# per query of the timed step: wall (roctx "query" range) vs kernel busy inside it
kt = (glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True) or [None])[0]
qs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
            if (r.get("Function") or r.get("Message")) == "query")
nq = int(sys.argv[2])
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(kt))) if kt else []
print("\nper query (timed step): wall ms, kernel-busy ms, idle ms")
tw = tb = 0.0
for i, (a, b) in enumerate(qs[-nq:]):
    busy, cur = 0, a
    for s0, e0 in ks:
        if e0 <= a or s0 >= b:
            continue
        s1, e1 = max(s0, cur), min(e0, b)
        if e1 > s1:
            busy += e1 - s1
            cur = e1
    tw += (b - a) / 1e6
    tb += busy / 1e6
    print(f"  q{i + 1:2d} {(b - a) / 1e6:8.2f} {busy / 1e6:8.2f} {(b - a - busy) / 1e6:8.2f}")
print(f"  total {tw:8.2f} {tb:8.2f} {tw - tb:8.2f}")
PY
