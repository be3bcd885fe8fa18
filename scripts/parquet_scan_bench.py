"""Cold Parquet scan + query benchmark (BASELINE.md "cold" rows).

TPC-H tables are generated on the GPU, written to Parquet files on local disk
(pyarrow writer, one file per table), and then read back through the engine:

* per table: native pread + H2D + GPU page decode of every column (cold: a
  fresh ParquetTable, nothing resident) vs the host decoder (pyarrow) + H2D;
* the 22-query suite over the Parquet tables: first run (cold: includes the
  scans of every column a query touches) and second run (warm: columns
  resident in HBM).

usage: python scripts/parquet_scan_bench.py --sf 10 [--compression snappy|none] [--dir /tmp/igloo_pq]
"""
import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pyarrow.parquet as pq  # noqa: E402
import torch  # noqa: E402

import igloo_amd as ig  # noqa: E402
from igloo_amd.connectors import parquet as P  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402


def log(*a):
    print(*a, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--compression", default="snappy")
    ap.add_argument("--dir", default="/tmp/igloo_pq")
    ap.add_argument("--row-group", type=int, default=1 << 21)
    ap.add_argument("--no-host", action="store_true", help="skip the host-decoder comparison")
    ap.add_argument("--queries", default="1-22")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out_dir = os.path.join(a.dir, f"sf{a.sf:g}_{a.compression}")
    shutil.rmtree(out_dir, ignore_errors=True)
    os.makedirs(out_dir)
    t0 = time.perf_counter()
    tabs = datagen.generate(a.sf, dev)
    torch.cuda.synchronize()
    log(f"[gen] sf={a.sf} {time.perf_counter() - t0:.1f}s")
    paths = {}
    t0 = time.perf_counter()
    for name, t in tabs.items():
        at = datagen.to_arrow({name: t})[name]
        p = os.path.join(out_dir, f"{name}.parquet")
        pq.write_table(at, p, row_group_size=a.row_group, compression=a.compression)
        paths[name] = p
        del at
    del tabs
    torch.cuda.empty_cache()
    log(f"[write] {time.perf_counter() - t0:.1f}s  {sum(os.path.getsize(p) for p in paths.values()) / 1e9:.2f} GB")

    res = {"sf": a.sf, "compression": a.compression, "tables": {}}
    e0 = ig.QueryEngine(device=dev)
    for name, p in paths.items():
        row = {"file_bytes": os.path.getsize(p)}
        for mode in (["gpu"] if a.no_host else ["gpu", "host"]):
            P.GPU_DECODE = mode == "gpu"
            src = P.ParquetTable(p)
            cols = [f.name for f in src.schema()]
            ctx = e0.make_context()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            b = src.scan(cols, ctx)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t1
            row[f"{mode}_s"] = round(dt, 4)
            row["rows"] = b.num_rows
            if mode == "gpu":
                row["gpu_stats"] = {k: (round(v, 4) if isinstance(v, float) else v)
                                    for k, v in src.last_gpu_stats.items()}
            del b, src
        P.GPU_DECODE = True
        row["gpu_rows_per_s"] = round(row["rows"] / row["gpu_s"], 1)
        row["gpu_file_GBps"] = round(row["file_bytes"] / row["gpu_s"] / 1e9, 2)
        res["tables"][name] = row
        log(f"[scan] {name:9s} {json.dumps(row)}")

    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    e = ig.QueryEngine(device=dev)
    for name, p in paths.items():
        e.register_parquet(name, p)
    for run in ("cold", "warm"):
        per = {}
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for q in qs:
            tq = time.perf_counter()
            e.sql(queries.QUERIES[q])
            torch.cuda.synchronize()
            per[q] = round((time.perf_counter() - tq) * 1e3, 2)
        total = time.perf_counter() - t1
        res[f"suite_{run}_s"] = round(total, 4)
        res[f"suite_{run}_ms"] = per
        log(f"[suite] {run}: {total:.3f}s  {per}")
    scanned = sum(res["tables"][t]["rows"] for t in res["tables"])
    res["all_tables_gpu_scan_s"] = round(sum(r["gpu_s"] for r in res["tables"].values()), 4)
    res["all_tables_rows_per_s"] = round(scanned / res["all_tables_gpu_scan_s"], 1)
    print(json.dumps(res), flush=True)
    shutil.rmtree(out_dir, ignore_errors=True)


if __name__ == "__main__":
    main()
