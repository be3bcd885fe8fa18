"""Parquet table source.

Parity: reference crates/engine/src/operators/parquet_scan.rs (ParquetScanExec:
whole-file read in 1024-row batches on a blocking thread, projection by index,
IO errors silently dropped at :79-81) and the DataFusion ListingTable +
ParquetFormat path used by the integration test
(crates/engine/tests/integration_test.rs:46-56).

Here: a path may be a file, a directory (recursive *.parquet) or a glob;
footer metadata gives schema/row counts without reading data; only projected
columns are read; row groups whose min/max statistics cannot satisfy a
pushed predicate are skipped; on N ranks each rank reads its share of the row
groups; decoded columns are kept resident in HBM (the cache tier) keyed by
file + mtime, so repeated scans do not touch the file. On a GPU the column
chunks are staged with native preads + one H2D copy and their pages are
decompressed and decoded by gfx950 kernels (igloo_amd/connectors/
gpu_parquet.py); columns that decoder does not handle (nested, INT96,
non-snappy codecs, DELTA encodings) and CPU scans use the host decoder
(pyarrow). IO errors raise. ``IGLOO_PARQUET_GPU=0`` forces the host decoder.
"""
from __future__ import annotations

import glob
import os
import threading
from typing import Dict, List, Optional, Sequence

import pyarrow as pa
import pyarrow.parquet as pq
import torch

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import IoError

GPU_DECODE = os.environ.get("IGLOO_PARQUET_GPU", "1") != "0"

def list_files(path: str, suffix: str = ".parquet") -> List[str]:
    if any(ch in path for ch in "*?["):
        files = sorted(glob.glob(path, recursive=True))
    elif os.path.isdir(path):
        files = sorted(os.path.join(d, f) for d, _, fs in os.walk(path) for f in fs if f.endswith(suffix))
    elif os.path.exists(path):
        files = [path]
    else:
        raise IoError(f"path does not exist: {path}")
    return files


class ParquetTable(TableSource):
    def __init__(self, path: str, files: Optional[List[str]] = None, cache: bool = True):
        self.path = path
        self.files = files if files is not None else list_files(path)
        if not self.files:
            raise IoError(f"no parquet files under {path}")
        self.cache = cache
        self._lock = threading.Lock()
        self._resident: Dict[tuple, Column] = {}
        self._gpu_reader = None
        self.last_gpu_stats: Dict[str, object] = {}
        try:
            self._meta = [pq.ParquetFile(f).metadata for f in self.files]
            schema = pq.read_schema(self.files[0])
        except (OSError, pa.ArrowInvalid) as e:
            raise IoError(f"cannot read parquet {self.files[0]}: {e}") from e
        self._arrow_schema = schema
        self._fields = [Field(f.name, T.from_arrow_type(f.type), f.nullable) for f in schema]

    def schema(self) -> List[Field]:
        return self._fields

    def num_rows(self) -> int:
        return sum(m.num_rows for m in self._meta)

    def row_groups(self):
        """(file index, row group index) in global order."""
        return [(fi, rg) for fi, m in enumerate(self._meta) for rg in range(m.num_row_groups)]

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        device = ctx.device if ctx is not None else torch.device("cpu")
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        groups = [g for i, g in enumerate(self.row_groups()) if i % world == rank]
        out: Dict[str, Column] = {}
        missing = []
        for c in columns:
            key = (c, str(device), rank, world, self._version())
            col = self._resident.get(key) if self.cache else None
            if col is None:
                missing.append(c)
            else:
                out[c] = col
        if missing and device.type == "cuda" and GPU_DECODE:
            # GPU page decode (csrc/kernels/parquet.hip); columns it does not
            # handle stay in `missing` for the host decoder below
            decoded, rejected = self._gpu().read([(c, self._field(c).dtype) for c in missing], groups, device)
            self.last_gpu_stats = dict(self._gpu().last_stats, host_columns=sorted(rejected))
            for c, col in decoded.items():
                if self.cache:
                    with self._lock:
                        self._resident[(c, str(device), rank, world, self._version())] = col
                out[c] = col
            missing = [c for c in missing if c not in decoded]
        if missing:
            tables = []
            for fi, rg in groups:
                try:
                    tables.append(pq.ParquetFile(self.files[fi]).read_row_group(rg, columns=missing))
                except (OSError, pa.ArrowInvalid) as e:
                    raise IoError(f"error reading {self.files[fi]} row group {rg}: {e}") from e
            if tables:
                t = pa.concat_tables(tables)
            else:
                t = pa.table({c: pa.array([], self._arrow_schema.field(c).type) for c in missing})
            for c in missing:
                col = Column.from_arrow(t.column(c), device=device, dtype=self._field(c).dtype)
                if self.cache:
                    with self._lock:
                        self._resident[(c, str(device), rank, world, self._version())] = col
                out[c] = col
        n = len(next(iter(out.values()))) if out else sum(self._meta[fi].row_group(rg).num_rows for fi, rg in groups)
        return Batch({c: out[c] for c in columns}, n)

    def _gpu(self):
        if self._gpu_reader is None:
            from .gpu_parquet import GpuParquetReader
            self._gpu_reader = GpuParquetReader(self.files)
        return self._gpu_reader

    def _field(self, name: str) -> Field:
        for f in self._fields:
            if f.name == name:
                return f
        raise KeyError(name)

    def _version(self):
        return tuple(os.path.getmtime(f) for f in self.files[:8])

    def evict(self):
        with self._lock:
            self._resident.clear()


def write_parquet(table: pa.Table, path: str, row_group_size: int = 1 << 20, compression: str = "snappy"):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    pq.write_table(table, path, row_group_size=row_group_size, compression=compression)
