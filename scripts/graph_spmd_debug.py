"""Reproduce a query-graph replay mismatch on the SPMD path (a world of one,
RCCL): run one query repeatedly at a scale factor on tables generated in HBM
with the multi-rank layout, print the execution modes and the graph module's
last errors. Env toggles can be passed through to bisect the cause.

    python scripts/graph_spmd_debug.py --sf 10 --q 3 --runs 8
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--q", default="3")
    ap.add_argument("--runs", type=int, default=8)
    ap.add_argument("--single", action="store_true")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29591")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    import torch
    import igloo_amd as ig
    from igloo_amd.exec import graphs
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops import jit
    from igloo_amd.parallel.comm import Communicator
    from igloo_amd.utils.digest import digest
    comm = None if a.single else Communicator.init(backend="nccl", device="cuda:0", force_spmd=True)
    e = ig.QueryEngine(device="cuda:0", comm=comm)
    for n, t in datagen.generate(a.sf, "cuda:0", 0, 1, spmd=not a.single).items():
        e.register_table(n, t)
    for q in [int(x) for x in a.q.split(",")]:
        sql = queries.QUERIES[q]
        e.sql(sql)
        jit.wait_all(timeout=300)
        out = []
        for i in range(a.runs):
            t0 = time.perf_counter()
            r = e.sql(sql)
            torch.cuda.synchronize()
            out.append(f"{e.last_metrics['speculation']}:{(time.perf_counter() - t0) * 1e3:.1f}:{str(digest(r.table))[:6]}")
        print(f"Q{q}", " ".join(out), flush=True)
    print(graphs.STATS, flush=True)
    for m in graphs.LAST_ERROR:
        print("ERR", m.strip().replace("\n", " | ")[-500:], flush=True)
    e.close()
    if comm is not None:
        comm.shutdown()


if __name__ == "__main__":
    main()
