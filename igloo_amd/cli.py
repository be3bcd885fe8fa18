"""``igloo`` command-line interface.

Parity: reference crates/igloo/src/main.rs — clap flags ``--sql/-s``,
``--config/-c``, ``--distributed`` (:9-20); with no arguments it runs
``SELECT 42 as answer, 'Hello Igloo' as message`` (:40-46); local queries see
an in-memory ``users(id Int32, name Utf8)`` table (Alice..Eve, :64-77); output
is pretty-printed (:92) and ``hello()`` is always printed (:49).
``--distributed`` (a local fallback in the reference, :97-100) sends the query
to the coordinator's Flight endpoint and falls back to local execution only
when no coordinator answers. Extra: ``--device``, ``--data-dir`` (auto-registers
*.parquet / *.csv), ``--tpch SF`` (synthetic TPC-H tables), ``--explain``.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import List, Optional

import pyarrow as pa

SAMPLE_SQL = "SELECT 42 as answer, 'Hello Igloo' as message"


def _users() -> pa.Table:
    return pa.table({"id": pa.array([1, 2, 3, 4, 5], pa.int32()),
                     "name": pa.array(["Alice", "Bob", "Charlie", "Diana", "Eve"], pa.string())})


def build_engine(device=None, data_dir: Optional[str] = None, tpch_sf: Optional[float] = None, cfg=None):
    import igloo_amd as ig
    e = ig.QueryEngine(device=device)
    e.register_table("users", _users())
    if data_dir and os.path.isdir(data_dir):
        for f in sorted(os.listdir(data_dir)):
            p = os.path.join(data_dir, f)
            name, ext = os.path.splitext(f)
            try:
                if ext == ".parquet":
                    e.register_parquet(name, p)
                elif ext == ".csv":
                    e.register_csv(name, p)
            except ig.IglooError as ex:
                print(f"skipping {p}: {ex}", file=sys.stderr)
    if tpch_sf:
        from .models.tpch import datagen
        datagen.register(e, tpch_sf)
    if cfg is not None:
        from .utils.config import register_config_tables
        register_config_tables(e, cfg)
    return e


def run_local(sql: str, device=None, data_dir=None, tpch_sf=None, explain=False, cfg=None) -> int:
    from .engine import print_batches
    e = build_engine(device, data_dir, tpch_sf, cfg)
    t0 = time.perf_counter()
    if explain:
        print(e.explain(sql, analyze=True))
        return 0
    res = e.sql(sql)
    print("Query Results:")
    print_batches(res)
    print(f"{res.num_rows} row(s) in {(time.perf_counter() - t0) * 1e3:.1f} ms on {e.device}")
    return 0


def run_distributed(sql: str, coordinator: str, **kw) -> int:
    from .engine import print_batches
    try:
        from .service.client import IglooClient
        with IglooClient(coordinator, timeout=5.0) as c:
            t = c.query(sql)
        print("Query Results (distributed):")
        print_batches(t)
        return 0
    except Exception as ex:  # noqa: BLE001 - any connection problem falls back (reference behaviour)
        print(f"Coordinator {coordinator} unavailable ({type(ex).__name__}: {ex}); falling back to local execution.")
        return run_local(sql, **kw)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="igloo", description="igloo MI355X SQL query engine")
    ap.add_argument("-c", "--config", help="configuration file (json/yaml/toml)")
    ap.add_argument("-s", "--sql", help="SQL query to execute")
    ap.add_argument("--distributed", action="store_true", help="run on the coordinator / GPU workers")
    ap.add_argument("--coordinator", default="grpc://127.0.0.1:50051")
    ap.add_argument("--device", default=None, help="cuda[:N] or cpu (default: GPU when present)")
    ap.add_argument("--data-dir", default="data", help="auto-register *.parquet / *.csv in this directory")
    ap.add_argument("--tpch", type=float, default=None, help="register synthetic TPC-H tables at this scale factor")
    ap.add_argument("--explain", action="store_true", help="print EXPLAIN ANALYZE instead of rows")
    a = ap.parse_args(argv)
    import igloo_amd as ig
    print("Igloo Query Engine CLI (MI355X)")
    cfg = None
    kw = dict(device=a.device, data_dir=a.data_dir, tpch_sf=a.tpch, explain=a.explain)
    try:
        if a.config:
            from .utils.config import load_config
            cfg = load_config(a.config, {"device": a.device})
            print(f"Config file specified: {a.config}")
            kw["cfg"] = cfg
        if a.sql:
            if a.distributed:
                print(f"Executing distributed query: {a.sql}")
                rc = run_distributed(a.sql, a.coordinator, **kw)
            else:
                print(f"Executing local query: {a.sql}")
                rc = run_local(a.sql, **kw)
        elif cfg is None:
            print("No config file specified. Starting in default mode or showing help.")
            print(f"Running sample query: {SAMPLE_SQL}")
            rc = run_local(SAMPLE_SQL, **kw)
        else:
            rc = 0
    except ig.IglooError as ex:
        print(f"error: {type(ex).__name__}: {ex}", file=sys.stderr)
        rc = 1
    print(ig.hello())
    return rc


if __name__ == "__main__":
    sys.exit(main())
