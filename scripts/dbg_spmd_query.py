"""Debug: one TPC-H query on N SPMD ranks sharing cuda:0 (gloo), partitioned
layout, low thresholds, under a list of env / threshold variants; prints the
row count and the rows that differ from sqlite for each variant."""
import json
import os
import sys
import tempfile

import torch.multiprocessing as mp

DEV = os.environ.get("DBG_DEVICE", "cuda:0")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _worker(rank, world, port, out, q, env, thr, replicate):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.environ.update(env)
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen
    from igloo_amd.models.tpch import queries as Q
    from igloo_amd.models.tpch.oracle import normalize
    from igloo_amd.parallel.comm import Communicator
    from igloo_amd.exec import joins as O
    from igloo_amd.ops import hashing as H
    from igloo_amd.parallel import exchange as X
    from igloo_amd.parallel import slicing as SL
    low = dict(X_SMALL_AGG_GATHER=0, X_SMALL_GATHER_STR_BYTES=16, X_PIPELINE_MIN_BYTES=0, X_PIPELINE_CHUNK_BYTES=2048,
               O_SORTED_JOIN_MIN_ROWS=1000, H_SORTED_CHECK_ROWS=1000, H_BLOOM_MIN_RATIO=2, SL_SLICE_MIN_ROWS=1000,
               SL_SLICE_MIXED_MIN_ROWS=1000)
    mods = {"X": X, "O": O, "H": H, "SL": SL}
    for k, v in low.items():
        if k in thr:
            continue   # this low threshold left at its default
        m, name = k.split("_", 1)
        setattr(mods[m], name, v)
    for item in filter(None, os.environ.get("DBG_SET", "").split(",")):
        path, val = item.split("=")
        mod, attr = path.rsplit(".", 1)
        import importlib
        setattr(importlib.import_module(mod), attr, type(getattr(importlib.import_module(mod), attr))(int(val)))
    if os.environ.get("DBG_TRUE_UNIQUE"):
        # key_unique() from the data itself (lets the unique-pairs path run on CPU)
        import torch
        H.key_unique = lambda k: k.dim() == 1 and torch.unique(k).numel() == k.numel()
    comm = Communicator.init(backend="gloo", device=DEV, timeout_s=120)
    e = ig.QueryEngine(device=DEV, comm=comm)
    for name, t in datagen.generate(0.01, DEV, rank, world, replicate_dims=replicate).items():
        e.register_table(name, t)
    rows = [[normalize(v) for v in r.values()] for r in e.sql(Q.QUERIES[q]).table.to_pylist()]
    if os.environ.get("DBG_WARM"):
        if comm.trace is not None:
            comm.trace.clear()
        e.sql(Q.QUERIES[q])
        if rank == 0:
            print("[warm] exchanges", e.last_metrics.get("exchanges"), "collectives", e.last_metrics.get("collectives"))
            for t in (comm.trace or []):
                print("   ", t)
    if rank == 0:
        json.dump(rows, open(out, "w"))
    comm.shutdown()


def main():
    import socket
    q = int(sys.argv[1])
    world = int(sys.argv[2])
    replicate = sys.argv[3] == "1"
    variants = json.loads(sys.argv[4])   # [[name, {env}, [thresholds kept at default]], ...]
    from igloo_amd.models.tpch import datagen, oracle
    import igloo_amd as ig
    e = ig.QueryEngine(device="cpu")
    tabs = datagen.register(e, 0.01)
    con = oracle.load_sqlite(datagen.to_arrow(tabs))
    exp = oracle.run_sqlite(con, q)
    for name, env, thr in variants:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "r.json")
            mp.start_processes(_worker, args=(world, port, out, q, env, thr, replicate), nprocs=world, join=True,
                               start_method="spawn")
            got = json.load(open(out))
        diff = oracle.rows_match([tuple(r) for r in got], exp)
        print(f"[{name}] rows={len(got)} diff={str(diff)[:600]}", flush=True)
        if diff:
            gs = {tuple(map(str, r)) for r in got}
            es = {tuple(map(str, r)) for r in exp}
            print(f"[{name}] missing {sorted(es - gs)[:5]} extra {sorted(gs - es)[:5]}", flush=True)


if __name__ == "__main__":
    main()
