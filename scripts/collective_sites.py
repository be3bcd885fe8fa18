"""Where a query's collectives come from: runs TPC-H on a forced world of one
(the SPMD code path: every exchange and collective runs, gloo on the CPU or
RCCL on a GPU) and prints, per query, each collective with the engine frames
that issued it.

    python scripts/collective_sites.py --sf 0.01 --queries 10,15,17 [--low]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=0.01)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--low", action="store_true", help="small data takes the large-data paths")
    ap.add_argument("--all-partitioned", action="store_true", help="every table hash-partitioned")
    a = ap.parse_args()
    os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("PORT", "29611"))
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries as Q
    from igloo_amd.parallel import comm as C
    if a.low:
        from igloo_amd.exec import joins as O
        from igloo_amd.ops import hashing as H
        from igloo_amd.parallel import slicing as SL
        O.SORTED_JOIN_MIN_ROWS = 1000
        H.SORTED_CHECK_ROWS = 1000
        SL.SLICE_MIN_ROWS = 1000
        SL.SLICE_MIXED_MIN_ROWS = 1000
    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    sites = []
    names = [n for n in vars(C.Communicator) if not n.startswith("_") and n not in ("init", "abort", "shutdown")]
    for n in names:
        fn = getattr(C.Communicator, n)
        if not callable(fn):
            continue

        def wrap(f, name):
            def w(self, *args, **kw):
                if getattr(self, "_depth", 0) == 0:
                    fr = [f"{os.path.basename(x.filename)}:{x.lineno}:{x.name}" for x in traceback.extract_stack()[:-1]
                          if "igloo_amd" in x.filename and "comm.py" not in x.filename]
                    sites.append((name, " <- ".join(reversed(fr[-4:]))))
                self._depth = getattr(self, "_depth", 0) + 1
                try:
                    return f(self, *args, **kw)
                finally:
                    self._depth -= 1
            return w
        setattr(C.Communicator, n, wrap(fn, n))
    comm = C.Communicator.init(backend="gloo" if a.device == "cpu" else "nccl", device=a.device, force_spmd=True)
    e = ig.QueryEngine(device=a.device, comm=comm)
    for name, t in datagen.generate(a.sf, a.device, 0, 1, replicate_dims=not a.all_partitioned, spmd=True).items():
        e.register_table(name, t)
    total = collections.Counter()
    for q in qs:
        for rep in range(2):
            del sites[:]
            e.sql(Q.QUERIES[q])
        print(f"Q{q}: {e.last_metrics.get('collectives')} collectives")
        for name, where in sites:
            print(f"    {name:22s} {where}")
            total[where.split(' <- ')[0]] += 1
    print("\nby innermost site:")
    for k, v in total.most_common():
        print(f"  {v:4d}  {k}")
    e.close()
    comm.shutdown()


if __name__ == "__main__":
    main()
