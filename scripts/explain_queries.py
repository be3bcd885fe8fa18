"""EXPLAIN ANALYZE selected TPC-H queries on one device (operator times, join order).

usage: python scripts/explain_queries.py --sf 100 --queries 10,18 [--device cuda:0]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igloo_amd as ig  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--queries", default="10,18")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--lean", action="store_true")
    ap.add_argument("--parquet", default=None, help="write + register the bench's Parquet dataset here")
    a = ap.parse_args()
    e = ig.QueryEngine(device=a.device)
    t0 = time.time()
    if a.parquet:
        from igloo_amd.models.tpch import parquet_gen
        parquet_gen.write_dataset(a.sf, a.parquet, device=a.device, rank=0, world=1, lean=a.lean)
        torch.cuda.empty_cache()
        parquet_gen.register_dataset(e, a.parquet, a.sf, 0, 1, lean=a.lean)
    else:
        datagen.register(e, a.sf, lean=a.lean)
    print(f"datagen sf={a.sf} {time.time() - t0:.1f}s", flush=True)
    for q in [int(x) for x in a.queries.split(",")]:
        e.query(queries.QUERIES[q])  # warm
        if a.device.startswith("cuda"):
            torch.cuda.synchronize()
        t = time.perf_counter()
        e.query(queries.QUERIES[q])
        if a.device.startswith("cuda"):
            torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3
        print(f"===== Q{q:02d} wall {wall:.2f} ms")
        print(e.explain(queries.QUERIES[q], analyze=True), flush=True)


if __name__ == "__main__":
    main()
