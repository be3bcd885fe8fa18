"""Per-kernel counter / roofline table from scripts/pmc_passes.sh output.

For every pass directory: counter_collection.csv (per dispatch counters) is
joined with kernel_trace.csv (dispatch durations) on the dispatch id; per
kernel name the counters are summed over dispatches. FETCH_SIZE / WRITE_SIZE
(KB) over the summed kernel time give achieved HBM-side bandwidth, reported
against the ~8 TB/s MI355X peak.

usage: python scripts/pmc_summary.py gpurun_out/pmc [--top 15]
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict

PEAK_GBS = 8000.0


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:60]


def load_pass(d, gap_ns=500e6):
    """Counters of the dispatches after the last idle gap > 0.5 s (bench.py
    with IGLOO_PROF_GAP=1 idles 1 s before the timed steps)."""
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        return {}, {}
    dur, start = {}, {}
    for r in csv.DictReader(open(kt[0])) if kt else []:
        dur[r.get("Dispatch_Id")] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        start[r.get("Dispatch_Id")] = int(r["Start_Timestamp"])
    cut = 0
    ts = sorted(start.values())
    for a, b in zip(ts, ts[1:]):
        if b - a > gap_ns:
            cut = b
    keep = {k for k, v in start.items() if v >= cut}
    per = defaultdict(lambda: defaultdict(float))
    seen = set()
    time_ns = defaultdict(float)
    for r in csv.DictReader(open(cc[0])):
        if keep and r.get("Dispatch_Id") not in keep:
            continue
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        did = r.get("Dispatch_Id")
        if did not in seen:
            seen.add(did)
            time_ns[k] += dur.get(did, 0)
    return per, time_ns


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--raw", action="store_true", help="also dump every counter (per wave where it is a count)")
    ap.add_argument("--exclude", default=r"textgen|datagen|gen_|_gen\b|rand", help="kernel-name regex to drop (data generation)")
    a = ap.parse_args()
    counters = defaultdict(dict)
    times = defaultdict(float)
    for d in sorted(glob.glob(os.path.join(a.root, "p*"))):
        if not os.path.isdir(d):
            continue
        per, tns = load_pass(d)
        for k, cs in per.items():
            counters[k].update(cs)
            times[k] = max(times[k], tns.get(k, 0))
    rx = re.compile(a.exclude) if a.exclude else None
    rows = sorted(((k, t) for k, t in times.items() if not (rx and rx.search(k))), key=lambda kv: -kv[1])[:a.top]
    print(f"{'kernel':60s} {'ms':>8s} {'fetch GB':>9s} {'write GB':>9s} {'GB/s':>8s} {'%peak':>6s} "
          f"{'VALU/wave':>10s} {'LDS/wave':>9s} {'LDSconf':>8s} {'MFMA':>6s}")
    for k, t in rows:
        c = counters[k]
        ms = t / 1e6
        fetch = c.get("FETCH_SIZE", 0) / 1e6   # KB -> GB
        write = c.get("WRITE_SIZE", 0) / 1e6
        gbs = (fetch + write) / (ms / 1e3) if ms else 0
        waves = max(c.get("SQ_WAVES", 1), 1)
        print(f"{k:60s} {ms:8.2f} {fetch:9.3f} {write:9.3f} {gbs:8.0f} {100 * gbs / PEAK_GBS:6.1f} "
              f"{c.get('SQ_INSTS_VALU', 0) / waves:10.0f} {c.get('SQ_INSTS_LDS', 0) / waves:9.0f} "
              f"{c.get('SQ_LDS_BANK_CONFLICT', 0):8.0f} {c.get('SQ_INSTS_MFMA', 0):6.0f}")
    if a.raw:
        for k, t in rows:
            c = counters[k]
            waves = max(c.get("SQ_WAVES", 1), 1)
            print(f"\n{k} ({t / 1e6:.2f} ms, {waves:.0f} waves)")
            for name in sorted(c):
                v = c[name]
                extra = f"  ({v / waves:.1f}/wave)" if name.startswith("SQ_INSTS") or name.startswith("SQ_WAIT") else ""
                print(f"    {name:32s} {v:16.0f}{extra}")


if __name__ == "__main__":
    main()
