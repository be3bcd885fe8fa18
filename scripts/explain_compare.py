"""EXPLAIN ANALYZE of the same queries on a single-rank engine and on the SPMD
path (world of one, every collective real), side by side: where does the
SPMD path spend its extra time?

    python scripts/explain_compare.py --sf 10 --queries 10,21 --device cuda:0
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--queries", default="10")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args()
    os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29900 + os.getpid() % 90))
    import igloo_amd as ig
    import igloo_amd.catalog as C
    from igloo_amd.models.tpch import datagen, queries as Q
    from igloo_amd.parallel.comm import Communicator
    comm = Communicator.init(backend="nccl" if a.device != "cpu" else "gloo", device=a.device, force_spmd=True)
    spmd = ig.QueryEngine(device=a.device, comm=comm)
    single = ig.QueryEngine(device=a.device)
    for n, t in datagen.generate(a.sf, a.device, 0, 1, spmd=True).items():
        spmd.register_table(n, t)
        single.register_table(n, C.MemoryTable(t.columns, t.num_rows(), cluster_key=t.cluster_key))
    for q in [int(x) for x in a.queries.split(",")]:
        for name, e in (("single", single), ("spmd", spmd)):
            for _ in range(3):
                e.sql(Q.QUERIES[q])
            print(f"===== Q{q} {name}\n" + e.explain(Q.QUERIES[q], analyze=True), flush=True)
    spmd.close()
    comm.shutdown()


if __name__ == "__main__":
    main()
