"""TPC-H Parquet datasets: generate on the device, write files in parallel.

The north-star benchmark reads "synthetic TPC-H-shaped Parquet data"
(BASELINE.json). The reference reads Parquet through ParquetScanExec /
DataFusion ListingTable (reference crates/engine/src/operators/
parquet_scan.rs:40-85, crates/engine/tests/integration_test.rs:46-56) but
ships no data (its data/sample.parquet is a text placeholder), so this module
produces the dataset:

* tables come from ``datagen`` (device-side generator, spec distributions);
* each table is split into files of ``rows_per_file`` rows (row groups of
  ``row_group`` rows inside), written by a thread pool (pyarrow's encoder
  releases the GIL, so files encode concurrently on all host cores);
* layout ``<root>/<table>/part-NNNNN.parquet``; a multi-rank dataset holds one
  such tree per rank (``<root>/r<rank>of<world>/...``), each rank writing its
  own hash partition (the same partition function as the exchanges), so the
  per-rank directories are co-partitioned like a bucketed table layout;
* low-cardinality strings are written as Arrow dictionaries (Parquet
  dictionary pages; the GPU reader turns them back into dictionary columns),
  decimals as INT64 (``store_decimal_as_integer``), dates as INT32;
* ``_manifest.json`` is written last: its presence marks a complete dataset,
  so a rerun with the same parameters reuses the files.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import shutil
import time
from typing import Dict, List, Optional

import pyarrow as pa
import pyarrow.parquet as pq
import torch

from ...columnar import Column
from . import datagen
from . import schema as S

#: per-table partitioning column of the multi-rank layout (None = replicated)
PARTITION_KEY = {"region": None, "nation": None, "supplier": "s_suppkey", "customer": "c_custkey",
                 "part": "p_partkey", "partsupp": "ps_partkey", "orders": "o_orderkey", "lineitem": "l_orderkey"}
FORMAT_VERSION = 2


def column_slice(c: Column, a: int, b: int) -> Column:
    """Rows [a, b) of a device column (views; string bytes re-based)."""
    valid = None if c.valid is None else c.valid[a:b]
    if c.offsets is not None:
        off = c.offsets[a:b + 1]
        lo, hi = (int(x) for x in off[[0, -1]].tolist())
        return Column(c.dtype, c.data[lo:hi], valid, offsets=off - lo)
    return Column(c.dtype, c.data[a:b], valid, dictionary=c.dictionary)


def column_to_arrow(c: Column) -> pa.Array:
    """Arrow array for the writer: dictionary columns stay dictionary-encoded."""
    if c.dictionary is not None:
        codes = pa.array(c.data.cpu().numpy(), pa.int32(),
                         mask=None if c.valid is None else ~c.valid.cpu().numpy())
        return pa.DictionaryArray.from_arrays(codes, c.dictionary.to_arrow().cast(pa.string()))
    arr = c.to_arrow()
    if pa.types.is_large_string(arr.type):
        arr = arr.cast(pa.string())
    return arr


def _write_chunk(path: str, cols: Dict[str, Column], a: int, b: int, row_group: int, compression: str) -> int:
    arrays = {k: column_to_arrow(column_slice(c, a, b)) for k, c in cols.items()}
    t = pa.table(arrays)
    dict_cols = [k for k, c in cols.items() if c.dictionary is not None]
    pq.write_table(t, path, row_group_size=row_group, compression=compression,
                   use_dictionary=dict_cols or False, store_decimal_as_integer=True,
                   write_statistics=True)
    return os.path.getsize(path)


def dataset_dir(root: str, sf: float, rank: int = 0, world: int = 1, lean: bool = False) -> str:
    tag = f"sf{sf:g}{'_lean' if lean else ''}"
    return os.path.join(root, tag, f"r{rank}of{world}")


def write_dataset(sf: float, root: str, device="cuda", rank: int = 0, world: int = 1, lean: bool = False,
                  rows_per_file: int = 8 << 20, row_group: int = 1 << 20, compression: str = "snappy",
                  threads: Optional[int] = None, log=None) -> dict:
    """Generate this rank's TPC-H partition and write it as Parquet under
    ``dataset_dir(root, ...)``; returns the manifest (reused when complete)."""
    out = dataset_dir(root, sf, rank, world, lean)
    man_path = os.path.join(out, "_manifest.json")
    want = {"format": FORMAT_VERSION, "sf": sf, "rank": rank, "world": world, "lean": lean,
            "rows_per_file": rows_per_file, "row_group": row_group, "compression": compression}
    if os.path.exists(man_path):
        with open(man_path) as f:
            man = json.load(f)
        if all(man.get(k) == v for k, v in want.items()):
            man["reused"] = True
            return man
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(out)
    threads = threads or min(16, os.cpu_count() or 4)
    t0 = time.perf_counter()
    tabs = datagen.generate(sf, device, rank, world, lean=lean)
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    t1 = time.perf_counter()
    jobs = []
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        for name in S.TABLES:
            t = tabs[name]
            os.makedirs(os.path.join(out, name))
            n = t.num_rows()
            step = max(rows_per_file, 1)
            for i, a in enumerate(range(0, max(n, 1), step)):
                b = min(n, a + step)
                p = os.path.join(out, name, f"part-{i:05d}.parquet")
                jobs.append(ex.submit(_write_chunk, p, t.columns, a, b, row_group, compression))
        nbytes = sum(j.result() for j in jobs)
    write_s = time.perf_counter() - t1
    man = dict(want, rows={k: v.num_rows() for k, v in tabs.items()}, bytes=nbytes, files=len(jobs),
               gen_s=round(gen_s, 3), write_s=round(write_s, 3), reused=False)
    del tabs
    with open(man_path + ".tmp", "w") as f:
        json.dump(man, f)
    os.replace(man_path + ".tmp", man_path)
    if log:
        log(f"[parquet] wrote {len(jobs)} files, {nbytes / 1e9:.2f} GB in {write_s:.1f}s (gen {gen_s:.1f}s) -> {out}")
    return man


def register_dataset(engine, root: str, sf: float, rank: int = 0, world: int = 1, lean: bool = False,
                     tables: Optional[List[str]] = None, **kw) -> Dict[str, object]:
    """Register every table of a written dataset (this rank's partition)."""
    out = dataset_dir(root, sf, rank, world, lean)
    srcs = {}
    for name in tables or S.TABLES:
        key = PARTITION_KEY[name]
        srcs[name] = engine.register_parquet(
            name, os.path.join(out, name), local=True, replicated=(key is None and world > 1),
            partitioned_by=key if world > 1 else None, **kw)
    return srcs
