"""cProfile of the warm TPC-H suite (host-side overhead: Python, syncs, launches).

usage: python scripts/host_profile.py --sf 100 [--queries 1-22] [--top 40]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igloo_amd as ig  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, a.sf)
    from igloo_amd.ops import jit
    for _ in range(5):      # JIT compiles settle, recordings confirmed, graphs captured
        for q in qs:
            e.sql(queries.QUERIES[q])
        jit.wait_all(120)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for q in qs:
        e.sql(queries.QUERIES[q])
    torch.cuda.synchronize()
    pr.disable()
    print(f"suite {time.perf_counter() - t0:.3f}s (profiled)")
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_callers(r"method 'item'|method 'cpu'|method 'tolist'")
    print(s.getvalue())
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue())


if __name__ == "__main__":
    main()
