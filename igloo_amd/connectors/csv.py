"""CSV table source.

Parity: reference crates/connectors/filesystem/src/lib.rs —
``CsvTable::new(path)`` (header = true), ``new_with_header(path, has_header)``,
``scan() -> Iterator<Row = Vec<String>>`` reading the whole file, io/csv errors
mapped to ``Error::Unknown`` (:18-46); and the coordinator's DataFusion
ListingTable CSV with an explicit schema (reference crates/coordinator/src/main.rs:26-44).

Both shapes are provided: ``scan_rows()`` returns the reference's rows of
strings; ``scan()`` (TableSource) returns typed device columns. On a GPU the
file is staged in HBM and parsed by gfx950 kernels (igloo_amd/connectors/
gpu_csv.py: quote-aware row splitting + typed field parsing); on CPU, or when
a value does not parse as the declared type, Arrow's multithreaded CSV reader
is used. ``GPU_PARSE = False`` forces the host reader.
"""
from __future__ import annotations

import csv as _csv
import os
from typing import Iterator, List, Optional, Sequence

import pyarrow as pa
import pyarrow.csv as pacsv
import torch

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import IoError

Row = List[str]
GPU_PARSE = True
#: files up to this size infer their schema from the whole file, larger ones
#: from the first block (the GPU parse then checks every value)
FULL_INFER_BYTES = 64 << 20


class CsvTable(TableSource):
    cacheable = True   # resident copies live in the engine's cache tier

    def __init__(self, path: str, schema: Optional[List[Field]] = None, has_header: bool = True,
                 delimiter: str = ","):
        self.path = path
        self.has_header = has_header
        self.delimiter = delimiter
        self._schema = schema
        self._table: Optional[pa.Table] = None
        self._gpu_rows: Optional[int] = None
        self.last_scan = ""   # "gpu" | "host" (| "host: <reason>")

    # -------------------------------------------------------- reference API
    @staticmethod
    def new(path: str) -> "CsvTable":
        return CsvTable(path, has_header=True)

    @staticmethod
    def new_with_header(path: str, has_header: bool) -> "CsvTable":
        return CsvTable(path, has_header=has_header)

    def scan_rows(self) -> Iterator[Row]:
        """All data rows as lists of strings (header row skipped when present)."""
        try:
            with open(self.path, newline="") as f:
                rows = list(_csv.reader(f, delimiter=self.delimiter))
        except OSError as e:
            raise IoError(f"failed to open {self.path}: {e.strerror or e}") from e
        except _csv.Error as e:
            raise IoError(f"csv error in {self.path}: {e}") from e
        if self.has_header and rows:
            rows = rows[1:]
        return iter(rows)

    # ------------------------------------------------------------ TableSource
    def _load(self) -> pa.Table:
        if self._table is None:
            if not os.path.exists(self.path):
                raise IoError(f"failed to open {self.path}: No such file or directory")
            ro = pacsv.ReadOptions(autogenerate_column_names=not self.has_header)
            if self._schema and not self.has_header:
                ro = pacsv.ReadOptions(column_names=[f.name for f in self._schema])
            po = pacsv.ParseOptions(delimiter=self.delimiter)
            co = pacsv.ConvertOptions(
                column_types={f.name: f.dtype.to_arrow() for f in self._schema} if self._schema else None)
            try:
                t = pacsv.read_csv(self.path, read_options=ro, parse_options=po, convert_options=co)
            except (pa.ArrowInvalid, OSError) as e:
                raise IoError(f"csv error in {self.path}: {e}") from e
            if self._schema and self.has_header:
                t = t.rename_columns([f.name for f in self._schema][: t.num_columns])
            self._table = t
        return self._table

    def schema(self) -> List[Field]:
        if self._schema:
            return self._schema
        if os.path.exists(self.path) and os.path.getsize(self.path) > FULL_INFER_BYTES:
            sch = self._infer_first_block()
        else:
            sch = self._load().schema
        self._schema = [Field(f.name, T.from_arrow_type(f.type), True) for f in sch]
        return self._schema

    def _infer_first_block(self) -> pa.Schema:
        ro = pacsv.ReadOptions(autogenerate_column_names=not self.has_header, block_size=4 << 20)
        try:
            with pacsv.open_csv(self.path, read_options=ro,
                                parse_options=pacsv.ParseOptions(delimiter=self.delimiter)) as r:
                return r.schema
        except (pa.ArrowInvalid, OSError) as e:
            raise IoError(f"csv error in {self.path}: {e}") from e

    def num_rows(self) -> int:
        if self._gpu_rows is not None:
            return self._gpu_rows
        return self._load().num_rows

    def _scan_gpu(self, columns: Sequence[str], device):
        from .gpu_csv import CsvParseError, read_csv_gpu
        fields = self.schema()
        try:
            cols = read_csv_gpu(self.path, fields, columns, device, has_header=self.has_header,
                                delimiter=self.delimiter)
        except CsvParseError as e:
            self.last_scan = f"host: {e}"
            return None
        self.last_scan = "gpu"
        if cols:
            self._gpu_rows = len(next(iter(cols.values())))
        return cols

    @property
    def version(self):
        """CDC probe: the file's mtime and size (a rewrite drops cached columns)."""
        try:
            st = os.stat(self.path)
        except OSError:
            return None
        if self._table is not None and getattr(self, "_ver", None) not in (None, (st.st_mtime_ns, st.st_size)):
            self._table = None   # host copy of the old contents
        self._ver = (st.st_mtime_ns, st.st_size)
        return self._ver

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        device = ctx.device if ctx is not None else torch.device("cpu")
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        out = {}
        missing = list(columns)
        if missing and device.type == "cuda" and GPU_PARSE:
            cols = self._scan_gpu(missing, device)
            if cols is not None:
                n = len(next(iter(cols.values()))) if cols else 0
                lo, hi = 0, n
                if world > 1:  # contiguous row ranges per rank
                    per = (n + world - 1) // world
                    lo, hi = min(rank * per, n), min((rank + 1) * per, n)
                for c in missing:
                    col = cols[c]
                    if world > 1:
                        from ..ops.gather import take
                        col = take(col, torch.arange(lo, hi, dtype=torch.int64, device=device))
                    out[c] = col
                missing = []
        if missing:
            t = self._load()
            if world > 1:  # contiguous row ranges per rank
                per = (t.num_rows + world - 1) // world
                t = t.slice(rank * per, per)
            types = {f.name: f.dtype for f in self.schema()}
            for c in missing:
                out[c] = Column.from_arrow(t.column(c), device=device, dtype=types[c])
            if not self.last_scan.startswith("host"):
                self.last_scan = "host"
        n = len(next(iter(out.values()))) if out else self.num_rows()
        return Batch({c: out[c] for c in columns}, n)
