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

#: multi-rank layout (models/tpch/datagen.py): fact tables partitioned by
#: order key in per-rank directories, dimension tables written once to a shared
#: directory that every rank reads whole (replicated); None = replicated
PARTITION_KEY = {t: (datagen.PARTITION_KEY[t] if t in datagen.PARTITIONED else None) for t in datagen.PARTITION_KEY}
FORMAT_VERSION = 3


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
    """This rank's partition of the fact tables."""
    tag = f"sf{sf:g}{'_lean' if lean else ''}"
    return os.path.join(root, tag, f"r{rank}of{world}")


def shared_dir(root: str, sf: float, lean: bool = False) -> str:
    """The replicated dimension tables (identical for every world size, so the
    1/2/4/8-GPU runs of one node write them once)."""
    tag = f"sf{sf:g}{'_lean' if lean else ''}"
    return os.path.join(root, tag, "shared")


def _table_dir(root, sf, name, rank, world, lean) -> str:
    if PARTITION_KEY[name] is None:
        return os.path.join(shared_dir(root, sf, lean), name)
    return os.path.join(dataset_dir(root, sf, rank, world, lean), name)


def _write_tables(out: str, want: dict, tables, gen, rows_per_file: int, row_group: int, compression: str,
                  threads: int) -> dict:
    man_path = os.path.join(out, "_manifest.json")
    if os.path.exists(man_path):
        with open(man_path) as f:
            man = json.load(f)
        if all(man.get(k) == v for k, v in want.items()):
            man["reused"] = True
            return man
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(out)
    t0 = time.perf_counter()
    tabs = gen()
    if any(c.data.is_cuda for t in tabs.values() for c in t.columns.values()):
        torch.cuda.synchronize()
    gen_s = time.perf_counter() - t0
    t1 = time.perf_counter()
    jobs = []
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        for name in tables:
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
    return man


def write_dataset(sf: float, root: str, device="cuda", rank: int = 0, world: int = 1, lean: bool = False,
                  rows_per_file: int = 8 << 20, row_group: int = 1 << 20, compression: str = "snappy",
                  threads: Optional[int] = None, log=None, wait_s: float = 3600.0) -> dict:
    """Generate and write this rank's partition of the fact tables and (rank 0)
    the shared dimension tables; other ranks wait for the shared manifest.
    Returns the combined manifest (complete datasets are reused)."""
    threads = threads or min(16, os.cpu_count() or 4)
    base = {"sf": sf, "lean": lean, "rows_per_file": rows_per_file, "row_group": row_group,
            "compression": compression}
    facts = [t for t in S.TABLES if PARTITION_KEY[t] is not None]
    dims = [t for t in S.TABLES if PARTITION_KEY[t] is None]
    m1 = _write_tables(dataset_dir(root, sf, rank, world, lean),
                       dict(base, format=FORMAT_VERSION, rank=rank, world=world), facts,
                       lambda: datagen.generate(sf, device, rank, world, lean=lean, tables=facts),
                       rows_per_file, row_group, compression, threads)
    sd = shared_dir(root, sf, lean)
    want2 = dict(base, format=FORMAT_VERSION, shared=True)
    if rank == 0:
        m2 = _write_tables(sd, want2, dims, lambda: datagen.generate(sf, device, 0, 1, lean=lean, tables=dims),
                           rows_per_file, row_group, compression, threads)
    else:
        t0 = time.perf_counter()
        mp_ = os.path.join(sd, "_manifest.json")
        while True:
            if os.path.exists(mp_):
                with open(mp_) as f:
                    m2 = json.load(f)
                if all(m2.get(k) == v for k, v in want2.items()):
                    m2["reused"] = True
                    break
            if time.perf_counter() - t0 > wait_s:
                raise TimeoutError(f"shared dimension tables not written to {sd}")
            time.sleep(0.5)
    man = {"format": FORMAT_VERSION, "sf": sf, "rank": rank, "world": world, "lean": lean,
           "rows": dict(m1["rows"], **m2["rows"]), "bytes": m1["bytes"] + (m2["bytes"] if rank == 0 else 0),
           "files": m1["files"] + (m2["files"] if rank == 0 else 0),
           "gen_s": round(m1["gen_s"] + (m2["gen_s"] if rank == 0 and not m2["reused"] else 0), 3),
           "write_s": round(m1["write_s"] + (m2["write_s"] if rank == 0 and not m2["reused"] else 0), 3),
           "reused": m1["reused"] and m2["reused"], "compression": compression}
    if log:
        log(f"[parquet] {man['files']} files, {man['bytes'] / 1e9:.2f} GB written in {man['write_s']:.1f}s "
            f"(gen {man['gen_s']:.1f}s, reused {man['reused']}) -> {dataset_dir(root, sf, rank, world, lean)} + {sd}")
    return man


def register_dataset(engine, root: str, sf: float, rank: int = 0, world: int = 1, lean: bool = False,
                     tables: Optional[List[str]] = None, spmd: Optional[bool] = None, **kw) -> Dict[str, object]:
    """Register every table of a written dataset (this rank's partition of
    the fact tables, the shared dimension tables whole). ``spmd`` (default
    world > 1) tags them with the multi-rank layout."""
    spmd = world > 1 if spmd is None else spmd
    srcs = {}
    for name in tables or S.TABLES:
        key = PARTITION_KEY[name]
        srcs[name] = engine.register_parquet(
            name, _table_dir(root, sf, name, rank, world, lean), local=True, replicated=(key is None and spmd),
            partitioned_by=key if spmd else None, cluster_key=datagen.CLUSTER_KEY[name], **kw)
    return srcs
