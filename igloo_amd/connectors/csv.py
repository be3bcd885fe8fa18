"""CSV table source.

Parity: reference crates/connectors/filesystem/src/lib.rs —
``CsvTable::new(path)`` (header = true), ``new_with_header(path, has_header)``,
``scan() -> Iterator<Row = Vec<String>>`` reading the whole file, io/csv errors
mapped to ``Error::Unknown`` (:18-46); and the coordinator's DataFusion
ListingTable CSV with an explicit schema (reference crates/coordinator/src/main.rs:26-44).

Both shapes are provided: ``scan_rows()`` returns the reference's rows of
strings; ``scan()`` (TableSource) returns typed device columns, parsed with
Arrow's multithreaded CSV reader and uploaded to HBM once.
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


class CsvTable(TableSource):
    def __init__(self, path: str, schema: Optional[List[Field]] = None, has_header: bool = True,
                 delimiter: str = ","):
        self.path = path
        self.has_header = has_header
        self.delimiter = delimiter
        self._schema = schema
        self._table: Optional[pa.Table] = None
        self._resident = {}

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
        t = self._load()
        self._schema = [Field(f.name, T.from_arrow_type(f.type), True) for f in t.schema]
        return self._schema

    def num_rows(self) -> int:
        return self._load().num_rows

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        device = ctx.device if ctx is not None else torch.device("cpu")
        t = self._load()
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        if world > 1:  # contiguous row ranges per rank
            per = (t.num_rows + world - 1) // world
            t = t.slice(rank * per, per)
        out = {}
        types = {f.name: f.dtype for f in self.schema()}
        for c in columns:
            key = (c, str(device), rank, world)
            if key not in self._resident:
                self._resident[key] = Column.from_arrow(t.column(c), device=device, dtype=types[c])
            out[c] = self._resident[key]
        return Batch(out, t.num_rows)
