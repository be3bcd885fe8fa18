"""Per-query GPU work of the single-rank path vs the SPMD path (world of one,
every collective real), for rocprofv3 kernel traces:

    rocprofv3 --kernel-trace --output-format csv -d out -o run -- \
        python3 scripts/spmd_overhead.py --sf 10 --queries 1,6,10,22
    python3 scripts/spmd_overhead.py --parse out/.../run_kernel_trace.csv --queries 1,6,10,22

Run mode: both engines read the same HBM tables; every query is warmed up
until it replays as a graph, then -- after a 1 s idle gap -- each (mode,
query) runs ``--reps`` times with 30 ms idle gaps, so the trace splits into
one segment per execution. Parse mode prints, per query and mode, the kernel
count, GPU busy time and the kernels the SPMD path adds.
"""
from __future__ import annotations

import argparse
import collections
import csv
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _qs(s):
    out = []
    for part in s.split(","):
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


def run(a):
    os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + os.getpid() % 200))
    import torch
    import igloo_amd as ig
    import igloo_amd.catalog as C
    from igloo_amd.models.tpch import datagen, queries as Q
    from igloo_amd.parallel.comm import Communicator
    dev = "cuda:0"
    comm = Communicator.init(backend="nccl", device=dev, force_spmd=True, timeout_s=300)
    spmd = ig.QueryEngine(device=dev, comm=comm)
    single = ig.QueryEngine(device=dev)
    for n, t in datagen.generate(a.sf, dev, 0, 1, spmd=True).items():
        spmd.register_table(n, t)
        single.register_table(n, C.MemoryTable(t.columns, t.num_rows(), cluster_key=t.cluster_key))
    qs = _qs(a.queries)
    engines = [("single", single), ("spmd", spmd)]
    from igloo_amd.ops import jit as _jit
    for rnd in range(2):
        for _, e in engines:
            for q in qs:
                for _ in range(6):
                    e.sql(Q.QUERIES[q])
        _jit.wait_all(timeout=300)     # generated kernels in place: the second round captures graphs
    torch.cuda.synchronize()
    time.sleep(1.0)
    ms = collections.defaultdict(list)
    windows = []
    for name, e in engines:
        for q in qs:
            for _ in range(a.reps):
                t0 = time.perf_counter()
                w0 = time.monotonic_ns()
                e.sql(Q.QUERIES[q])
                torch.cuda.synchronize()
                windows.append([name, q, w0, time.monotonic_ns(), e.last_metrics.get("speculation")])
                ms[(name, q)].append((time.perf_counter() - t0) * 1e3)
                time.sleep(0.03)
    import json
    with open(a.windows, "w") as f:
        json.dump(windows, f)
    for q in qs:
        s, p = min(ms[("single", q)]), min(ms[("spmd", q)])
        print(f"Q{q:02d} wall single {s:7.2f} ms  spmd {p:7.2f} ms  (+{p - s:.2f})  "
              f"spmd collectives {spmd.last_metrics.get('collectives') if q == qs[-1] else ''}", flush=True)
    spmd.close()
    comm.shutdown()


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"<.*", "", n)
    return n[:70]


def parse(a):
    rows = []
    with open(a.parse) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if a.windows and os.path.exists(a.windows):
        import bisect
        import json
        wins = json.load(open(a.windows))
        starts = [r[0] for r in rows]
        table = {}
        for name, q, w0, w1, mode in wins:
            seg = rows[bisect.bisect_left(starts, w0):bisect.bisect_right(starts, w1)]
            if seg and (name, q) not in table or seg and sum(e - b for b, e, _ in seg) < \
                    sum(e - b for b, e, _ in table[(name, q)]):
                table[(name, q)] = seg
        if len(table) == 2 * len(_qs(a.queries)):
            return _report(a, table)
        print(f"host windows matched {len(table)} executions: falling back to idle-gap splitting")
    # drop the warmup: everything before the last idle gap > 0.5 s
    cut = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > 5e8:
            cut = i
    rows = rows[cut:]
    segs, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - cur[-1][1] > 1.5e7:
            segs.append(cur)
            cur = []
        cur.append(r)
    segs.append(cur)
    qs = _qs(a.queries)
    want = 2 * len(qs) * a.reps
    print(f"{len(segs)} segments (expected {want})")
    if len(segs) != want:
        return
    k = 0
    table = {}
    for mode in ("single", "spmd"):
        for q in qs:
            reps = segs[k:k + a.reps]
            k += a.reps
            best = min(reps, key=lambda s: sum(e - b for b, e, _ in s))
            table[(mode, q)] = best
    _report(a, table)


def _report(a, table):
    qs = _qs(a.queries)
    tot = collections.Counter()
    for q in qs:
        s, p = table[("single", q)], table[("spmd", q)]
        bs = sum(e - b for b, e, _ in s) / 1e6
        bp = sum(e - b for b, e, _ in p) / 1e6
        span_s = (s[-1][1] - s[0][0]) / 1e6
        span_p = (p[-1][1] - p[0][0]) / 1e6
        print(f"Q{q:02d}: single {len(s):4d} kernels busy {bs:7.3f} ms span {span_s:7.3f} | "
              f"spmd {len(p):4d} kernels busy {bp:7.3f} ms span {span_p:7.3f} | +{len(p) - len(s)} kernels "
              f"+{bp - bs:.3f} ms busy")
        cs = collections.Counter(short(n) for _, _, n in s)
        cp = collections.Counter(short(n) for _, _, n in p)
        tp = collections.defaultdict(float)
        for b, e, n in p:
            tp[short(n)] += (e - b) / 1e6
        extra = sorted(((cp[n] - cs.get(n, 0), n) for n in cp if cp[n] > cs.get(n, 0)), reverse=True)[:a.top]
        for d, n in extra:
            print(f"      +{d:3d} x {n:70s} ({tp[n]:.3f} ms in spmd)")
        if a.seq:
            # the long kernels of both executions in launch order, side by side
            ls = [(short(n), (e - b) / 1e3) for b, e, n in s if e - b >= a.seq * 1e3]
            lp = [(short(n), (e - b) / 1e3) for b, e, n in p if e - b >= a.seq * 1e3]
            print(f"      kernels >= {a.seq:.0f} us (single | spmd):")
            for i in range(max(len(ls), len(lp))):
                x = f"{ls[i][0][:44]:44s} {ls[i][1]:7.1f}" if i < len(ls) else " " * 52
                y = f"{lp[i][0][:44]:44s} {lp[i][1]:7.1f}" if i < len(lp) else ""
                print(f"        {x} | {y}")
        tot["single_busy"] += bs
        tot["spmd_busy"] += bp
        tot["single_span"] += span_s
        tot["spmd_span"] += span_p
    print("suite: " + ", ".join(f"{k} {v:.2f} ms" for k, v in tot.items()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--queries", default="1,6,10,13,22")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--parse", default=None)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--seq", type=float, default=0.0, help="also list kernels longer than this many us, in order")
    ap.add_argument("--windows", default="gpurun_out/spmd_overhead_windows.json",
                    help="host monotonic-clock window of every timed execution (written by the run)")
    a = ap.parse_args()
    if a.parse:
        parse(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
