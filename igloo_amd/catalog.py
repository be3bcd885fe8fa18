"""Catalog and table sources.

Parity: reference crates/common/src/catalog.rs:5-27 — ``MemoryCatalog`` is a
``HashMap<String, Arc<dyn TableProvider>>`` with ``register_table`` (overwrite)
/ ``get_table`` (Option) and a public ``tables`` field that callers iterate
(reference crates/igloo/src/main.rs:83-85). This catalog keeps that API, is
thread-safe, and its sources expose schema, row counts and the partitioning
the distributed planner needs.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import pyarrow as pa
import torch

from . import types as T
from .columnar import Batch, Column
from .types import DataType
from .utils.errors import PlanError


@dataclass(frozen=True)
class Field:
    name: str
    dtype: DataType
    nullable: bool = True


class TableSource:
    """A scannable table. ``scan`` returns a device Batch keyed by column name."""

    #: column the rows are hash-partitioned on across ranks (None = arbitrary split)
    partitioned_by: Optional[str] = None
    #: every rank holds the full table
    replicated: bool = False
    #: integer column the rows are stored in ascending order of (SPMD: a
    #: replicated table splits by ranges of it, parallel/slicing.py)
    cluster_key: Optional[str] = None

    def schema(self) -> List[Field]:
        raise NotImplementedError

    def num_rows(self) -> Optional[int]:
        return None

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        raise NotImplementedError

    def field(self, name: str) -> Field:
        for f in self.schema():
            if f.name == name:
                return f
        raise PlanError(f"column {name} not in table")

    def arrow_schema(self) -> pa.Schema:
        return pa.schema([pa.field(f.name, f.dtype.to_arrow(), f.nullable) for f in self.schema()])


def _mark_resident(c: Column) -> None:
    """Flag a table column's data tensor as long-lived, so per-tensor derived
    structures (narrow copies for the fused scans) are worth building."""
    try:
        c.data._igloo_resident = True
    except (AttributeError, RuntimeError):
        pass


class MemoryTable(TableSource):
    """Device-resident table (the HBM tier): columns stay in GPU memory and a
    scan hands out the resident columns without copying."""

    def __init__(self, columns: Dict[str, Column], num_rows: Optional[int] = None,
                 partitioned_by: Optional[str] = None, replicated: bool = False,
                 fields: Optional[List[Field]] = None, resident: bool = True, cluster_key: Optional[str] = None):
        self.columns = dict(columns)
        # resident=False: columns stay where they are (e.g. host memory under a
        # small device budget) and each scan moves a transient copy
        self.resident = resident
        for c in self.columns.values():
            _mark_resident(c)
        self._n = num_rows if num_rows is not None else (len(next(iter(columns.values()))) if columns else 0)
        self.partitioned_by = partitioned_by
        self.replicated = replicated
        self.cluster_key = cluster_key
        self._fields = fields or [Field(k, c.dtype, c.valid is not None) for k, c in self.columns.items()]

    @staticmethod
    def from_arrow(table: pa.Table, device="cpu", **kw) -> "MemoryTable":
        cols = {name: Column.from_arrow(table.column(name), device=device) for name in table.column_names}
        fields = [Field(f.name, T.from_arrow_type(f.type), f.nullable) for f in table.schema]
        return MemoryTable(cols, table.num_rows, fields=fields, **kw)

    def schema(self) -> List[Field]:
        return self._fields

    def num_rows(self) -> int:
        return self._n

    def scan(self, columns, ctx) -> Batch:
        dev = ctx.device if ctx is not None else None
        out = {}
        for c in columns:
            col = self.columns[c]
            if dev is not None and col.device != dev:
                col = col.to(dev)
                if self.resident:
                    self.columns[c] = col  # promote to the execution device once (cache tier)
            out[c] = col
        return Batch(out, self._n)

    #: ``scan_morsels`` available (exec/morsel.py)
    can_stream = True

    def scan_morsels(self, columns, ctx, filters=None, max_rows: int = 1 << 20):
        """Row ranges of at most ``max_rows`` rows, each moved to the execution
        device on its own (exec/morsel.py): a host-resident table streams
        through a bounded device working set."""
        from .cache.cdc import _slice
        dev = ctx.device if ctx is not None else None
        for a in range(0, self._n, max(1, max_rows)):
            z = min(self._n, a + max_rows)
            out = {}
            for c in columns:
                col = _slice(self.columns[c], a, z)
                out[c] = col.to(dev) if dev is not None and col.device != dev else col
            yield Batch(out, z - a)

    @property
    def nbytes(self) -> int:
        return sum(c.nbytes for c in self.columns.values())


class Catalog:
    """Thread-safe name -> TableSource map (+ views)."""

    def __init__(self):
        self._lock = threading.RLock()
        self.tables: Dict[str, TableSource] = {}
        self.views: Dict[str, str] = {}
        #: bumped by every DDL change (plan caches key on it)
        self.version = 0

    def register_table(self, name: str, source: TableSource) -> Optional[TableSource]:
        with self._lock:
            old = self.tables.get(name)
            self.tables[name] = source
            self.version += 1
            return old

    def get_table(self, name: str) -> Optional[TableSource]:
        with self._lock:
            return self.tables.get(name)

    def deregister_table(self, name: str) -> Optional[TableSource]:
        with self._lock:
            self.version += 1
            self.views.pop(name, None)
            return self.tables.pop(name, None)

    def register_view(self, name: str, sql: str):
        with self._lock:
            self.version += 1
            self.views[name] = sql

    def drop_view(self, name: str):
        with self._lock:
            self.version += 1
            return self.views.pop(name, None)

    def view_names(self) -> List[str]:
        with self._lock:
            return sorted(self.views)

    def get_view(self, name: str) -> Optional[str]:
        with self._lock:
            return self.views.get(name)

    def table_names(self) -> List[str]:
        with self._lock:
            return sorted(self.tables)

    def __iter__(self) -> Iterator[Tuple[str, TableSource]]:
        with self._lock:
            return iter(list(self.tables.items()))

    def __contains__(self, name: str) -> bool:
        return self.get_table(name) is not None


# reference name
MemoryCatalog = Catalog
