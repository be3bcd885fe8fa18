"""EXPLAIN ANALYZE of the first and second fresh-parameter statement of a
TPC-H query after the validation statement warmed up (what does the first
ad-hoc statement of a template pay once?).

    python scripts/first_fresh.py --sf 100 --queries 18
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--queries", default="18")
    a = ap.parse_args()
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, params, queries as Q
    from igloo_amd.ops import jit
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, a.sf)
    qs = [int(x) for x in a.queries.split(",")]
    for q in qs:
        for _ in range(3):
            e.sql(Q.QUERIES[q])
    jit.wait_all(timeout=120)
    for q in qs:
        for seed in (1000, 1001):
            sql = params.stream([q], seed, a.sf)[q]
            print(f"===== Q{q} seed {seed}\n" + e.explain(sql, analyze=True), flush=True)


if __name__ == "__main__":
    main()
