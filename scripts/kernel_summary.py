"""Per-kernel time of the timed steps from a rocprofv3 kernel trace.

bench.py (with IGLOO_PROF_GAP=1) idles for 1 s between warmup and the timed
steps; everything before the last gap > 0.5 s (data generation, warmup) is
dropped, the rest is grouped by kernel name and divided by --steps.

usage: python scripts/kernel_summary.py <run_kernel_trace.csv> [--steps N] [--top 30]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gap-ms", type=float, default=500.0)
    ap.add_argument("--dispatches", default=None, metavar="REGEX",
                    help="also list every dispatch of the matching kernels in the timed steps (us, grid)")
    a = ap.parse_args()
    grid = {}
    rows = []
    for r in csv.DictReader(open(a.trace)):
        t = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
        rows.append(t)
        grid[t] = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
    rows.sort(key=lambda x: x[0])
    cut = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > a.gap_ms * 1e6:
            cut = i
    rows = rows[cut:]
    tot, cnt = defaultdict(int), defaultdict(int)
    for s, e, n in rows:
        tot[short(n)] += e - s
        cnt[short(n)] += 1
    busy = sum(tot.values())
    span = rows[-1][1] - rows[0][0] if rows else 0
    print(f"kernels={len(rows)} busy={busy / 1e6 / a.steps:.2f} ms/step span={span / 1e6 / a.steps:.2f} ms/step "
          f"(busy/span={busy / max(span, 1):.2f})")
    print(f"{'ms/step':>9} {'calls':>6} {'us/call':>9}  kernel")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{t / 1e6 / a.steps:9.3f} {cnt[n] // a.steps:6d} {t / 1e3 / cnt[n]:9.1f}  {n}")
    # idle time between consecutive kernels, by gap size: short gaps are the
    # per-dispatch cost inside a graph / launch stream, long ones host work
    gaps = [rows[i][0] - rows[i - 1][1] for i in range(1, len(rows))]
    edges = [(0, 2e3), (2e3, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e6), (1e6, 1e12)]
    print("idle between kernels (ms/step by gap size):", "  ".join(
        f"{lo / 1e3:g}-{hi / 1e3:g}us: {sum(g for g in gaps if lo <= g < hi) / 1e6 / a.steps:.2f} "
        f"({sum(1 for g in gaps if lo <= g < hi) // a.steps})" for lo, hi in edges))
    # which kernel pairs the mid-size gaps (5-100 us: inside a query) sit
    # between: a graph's non-kernel nodes (memset / memcpy) or a host
    # readback between launches show up here
    pairs = defaultdict(lambda: [0, 0])
    for i in range(1, len(rows)):
        g = rows[i][0] - rows[i - 1][1]
        if 5e3 <= g < 1e5:
            k = (short(rows[i - 1][2])[:48], short(rows[i][2])[:48])
            pairs[k][0] += g
            pairs[k][1] += 1
    if pairs:
        print("\nlargest 5-100 us gaps by kernel pair (ms/step, count/step): before -> after")
        for (x, y), (g, c) in sorted(pairs.items(), key=lambda kv: -kv[1][0])[:25]:
            print(f"{g / 1e6 / a.steps:7.3f} {c / a.steps:6.1f}  {x} -> {y}")
    if a.dispatches:
        print(f"\ndispatches matching {a.dispatches!r} (all timed steps, in order): us  grid  kernel")
        for r in rows:
            if re.search(a.dispatches, r[2]):
                print(f"{(r[1] - r[0]) / 1e3:9.1f} {grid[r]:>10}  {short(r[2])[:70]}")


if __name__ == "__main__":
    main()
