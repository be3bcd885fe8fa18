"""Where ad-hoc TPC-H statements (fresh substitution parameters every time:
no plan, readback or graph reuse) spend their time: per query wall time vs
device time (engine last_metrics: one event pair per query), then one stream
under cProfile.

usage: python scripts/adhoc_profile.py [--sf 100] [--streams 2] [--out gpurun_out/adhoc_profile.txt]
Tables are generated in HBM (bench.py --source hbm)."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100.0)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/adhoc_profile.txt")
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, params, queries
    from igloo_amd.ops import jit
    qs = list(range(1, 23))
    e = ig.QueryEngine(device="cuda:0")
    for name, t in datagen.generate(a.sf, "cuda:0").items():
        e.register_table(name, t)
    for _ in range(2):
        for q in qs:
            e.sql(queries.QUERIES[q])
    jit.wait_all(timeout=120)
    rows = {q: [0.0, 0.0, 0, 0.0] for q in qs}    # wall ms, dev span ms, host steps, plan ms
    per_stream = {q: [] for q in qs}                # (wall ms, readbacks) per stream
    t_streams = []
    for k in range(a.streams):
        st = params.stream(qs, 2000 + k, a.sf)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for q in qs:
            e.sql(st[q])
            m = e.last_metrics
            r = rows[q]
            r[0] += m["elapsed_ms"]
            r[1] += m.get("device_span_ms", 0.0)
            r[2] += m.get("host_steps", 0)
            per_stream[q].append((m["elapsed_ms"], m.get("readbacks", 0)))
        torch.cuda.synchronize()
        t_streams.append(time.perf_counter() - t0)
    # planning alone (parse + bind + optimize) of a fresh stream
    from igloo_amd.sql import parse
    st = params.stream(qs, 2999, a.sf)
    for q in qs:
        t0 = time.perf_counter()
        e._plan_query(parse(st[q])[0])
        rows[q][3] = (time.perf_counter() - t0) * 1e3
    s = io.StringIO()
    n = a.streams
    s.write(f"SF{a.sf:g} ad-hoc streams: {[round(t, 4) for t in t_streams]} s per suite\n")
    s.write(f"{'query':>6} {'wall ms':>9} {'dev span ms':>10} {'host ms':>9} {'plan ms':>8} {'host steps':>10}\n")
    tot = [0.0, 0.0, 0.0]
    for q in qs:
        w, d, h, p = rows[q][0] / n, rows[q][1] / n, rows[q][2] / n, rows[q][3]
        tot[0] += w
        tot[1] += d
        tot[2] += p
        s.write(f"{'Q%d' % q:>6} {w:9.2f} {d:10.2f} {w - d:9.2f} {p:8.2f} {h:10.1f}\n")
    s.write(f"{'total':>6} {tot[0]:9.2f} {tot[1]:10.2f} {tot[0] - tot[1]:9.2f} {tot[2]:8.2f}\n\n")
    s.write("per stream (wall ms / blocking readbacks):\n")
    for q in qs:
        s.write(f"{'Q%d' % q:>6} " + "  ".join(f"{w:8.2f}/{rb:3d}" for w, rb in per_stream[q]) + "\n")
    s.write("\n")
    pr = cProfile.Profile()
    st = params.stream(qs, 3000, a.sf)
    pr.enable()
    for q in qs:
        e.sql(st[q])
    torch.cuda.synchronize()
    pr.disable()
    ps = pstats.Stats(pr, stream=s)
    ps.sort_stats("tottime").print_stats(40)
    ps.sort_stats("cumulative").print_stats(60)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(s.getvalue())
    print(s.getvalue()[:4000])


if __name__ == "__main__":
    main()
