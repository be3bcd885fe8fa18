"""Host-side profile of the eager (graphs off) warm TPC-H suite: where the
Python operator driver spends its time per query.

usage: python scripts/eager_profile.py [--sf 1] [--runs 3] [--out gpurun_out/eager_profile.txt]
Runs the 22 queries ``--runs`` times with query graphs disabled (replayed
readbacks stay on, as in bench.py's warm_eager_s), then once more under
cProfile, and writes the suite time plus the top functions by own time and by
cumulative time."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["IGLOO_GRAPHS"] = "0"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/eager_profile.txt")
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, a.sf)
    qs = [queries.QUERIES[q] for q in range(1, 23)]
    times = []
    for _ in range(a.runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for sql in qs:
            e.sql(sql)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    per_q = {}
    for i, sql in enumerate(qs, 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.sql(sql)
        torch.cuda.synchronize()
        per_q[i] = (time.perf_counter() - t0) * 1e3
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    for sql in qs:
        e.sql(sql)
    torch.cuda.synchronize()
    pr.disable()
    prof_s = time.perf_counter() - t0
    s = io.StringIO()
    s.write(f"SF{a.sf} eager warm suite (graphs off, replayed readbacks on): runs {[round(t, 4) for t in times]} s; "
            f"profiled run {prof_s:.4f} s\n")
    s.write("per query ms: " + ", ".join(f"Q{q} {v:.1f}" for q, v in per_q.items()) + "\n\n")
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(s.getvalue())
    print(s.getvalue()[:600])


if __name__ == "__main__":
    main()
