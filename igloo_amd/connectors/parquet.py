"""Parquet table source.

Parity: reference crates/engine/src/operators/parquet_scan.rs (ParquetScanExec:
whole-file read in 1024-row batches on a blocking thread, projection by index,
IO errors silently dropped at :79-81) and the DataFusion ListingTable +
ParquetFormat path used by the integration test
(crates/engine/tests/integration_test.rs:46-56), which prunes row groups by
their min/max statistics.

Here: a path may be a file, a directory (recursive *.parquet) or a glob;
footer metadata gives schema/row counts without reading data; only projected
columns are read; row groups whose min/max statistics prove a pushed
conjunct false are skipped (``scan(..., filters=...)``; the counts land in
``last_gpu_stats``); on N ranks each rank reads its share of the row groups,
or — for a ``local`` dataset whose files already hold this rank's hash
partition (models/tpch/parquet_gen.py) — all of them. On a GPU the column
chunks are staged with native preads + one H2D copy and their pages are
decompressed and decoded by gfx950 kernels (connectors/gpu_parquet.py);
columns that decoder does not handle (nested, INT96, non-snappy codecs, DELTA
encodings) and CPU scans use the host decoder (pyarrow). IO errors raise.
``GPU_DECODE = False`` forces the host decoder.

The source itself keeps nothing resident: the engine wraps it in the cache
tier (cache/cdc.py CachedTable) whose CDC probe is ``version`` — the listed
file set with every file's mtime and size, so a rewritten, added or removed
file anywhere in the dataset invalidates the cached columns.
"""
from __future__ import annotations

import glob
import os
import threading
from fractions import Fraction
from typing import Dict, List, Optional, Sequence, Tuple

import pyarrow as pa
import pyarrow.parquet as pq
import torch

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import IoError

GPU_DECODE = True
_FLIP = {"=": "=", "<": ">", "<=": ">=", ">": "<", ">=": "<="}


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


def _file_version(files: Sequence[str]) -> tuple:
    out = []
    for f in files:
        try:
            st = os.stat(f)
            out.append((f, st.st_mtime_ns, st.st_size))
        except OSError:
            out.append((f, None, None))
    return tuple(out)


class ParquetTable(TableSource):
    cacheable = True
    #: ``scan`` takes pushed filters for row-group statistics pruning
    prunes = True
    #: ``scan_morsels`` available (exec/morsel.py)
    can_stream = True

    def __init__(self, path: str, files: Optional[List[str]] = None, local: bool = False,
                 partitioned_by: Optional[str] = None, replicated: bool = False, cache: Optional[bool] = None,
                 cluster_key: Optional[str] = None):
        self.path = path
        self._fixed_files = files is not None
        self.files = files if files is not None else list_files(path)
        if not self.files:
            raise IoError(f"no parquet files under {path}")
        self.local = local
        self.partitioned_by = partitioned_by
        self.replicated = replicated
        self.cluster_key = cluster_key
        if cache is not None:
            self.cacheable = cache
        self._lock = threading.Lock()
        self._gpu_reader = None
        self.last_gpu_stats: Dict[str, object] = {}
        self._load_meta()

    def _load_meta(self):
        try:
            self._meta = [pq.ParquetFile(f).metadata for f in self.files]
            schema = pq.read_schema(self.files[0])
        except (OSError, pa.ArrowInvalid) as e:
            raise IoError(f"cannot read parquet {self.files[0]}: {e}") from e
        self._arrow_schema = schema
        self._fields = [Field(f.name, T.from_arrow_type(f.type), f.nullable) for f in schema]
        self._stat_version = _file_version(self.files)
        self._gpu_reader = None
        self._bounds: Dict[str, Dict[Tuple[int, int], object]] = {}   # column -> row group -> bounds

    def schema(self) -> List[Field]:
        return self._fields

    def num_rows(self) -> int:
        return sum(m.num_rows for m in self._meta)

    @property
    def version(self) -> tuple:
        """CDC probe: the dataset's file set with mtimes and sizes (re-listed,
        so added / removed files count too). A change reloads the footers."""
        files = self.files if self._fixed_files else list_files(self.path)
        v = _file_version(files)
        if v != self._stat_version:
            with self._lock:
                self.files = files
                self._load_meta()
        return self._stat_version

    def row_groups(self):
        """(file index, row group index) in global order."""
        return [(fi, rg) for fi, m in enumerate(self._meta) for rg in range(m.num_row_groups)]

    def my_row_groups(self, ctx) -> List[Tuple[int, int]]:
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        groups = self.row_groups()
        if self.local or world == 1:
            return groups
        return [g for i, g in enumerate(groups) if i % world == rank]

    # ------------------------------------------------------------ pruning
    def prune(self, groups: List[Tuple[int, int]], filters) -> List[Tuple[int, int]]:
        """Drop row groups whose min/max statistics prove some conjunct false.
        ``filters``: [(column name, op, [values])] with op in = < <= > >= in."""
        if not filters or not groups:
            return groups
        # decoded footer bounds per column, built once per metadata version:
        # a filter set the engine has not seen (new substitution parameters)
        # costs one comparison per row group, not a walk over footer objects
        checks = [(self._column_bounds(name), op, values) for name, op, values in filters]
        return [g for g in groups if not any(_bounds_refute(b.get(g), op, values) for b, op, values in checks)]

    def group_rows(self) -> Dict[Tuple[int, int], int]:
        """Row count of every (file, row group), kept per metadata version."""
        r = self._bounds.get("\0rows")
        if r is None:
            r = self._bounds["\0rows"] = {(fi, rg): m.row_group(rg).num_rows
                                          for fi, m in enumerate(self._meta) for rg in range(m.num_row_groups)}
        return r

    def _column_bounds(self, name: str) -> Dict[Tuple[int, int], object]:
        b = self._bounds.get(name)
        if b is None:
            b = {}
            for fi, m in enumerate(self._meta):
                idx = _leaf_index(m, name)
                for rg in range(m.num_row_groups):
                    b[(fi, rg)] = _group_bounds(m, m.row_group(rg), idx)
            self._bounds[name] = b
        return b

    # ------------------------------------------------------------- scan
    def scan_morsels(self, columns: Sequence[str], ctx, filters=None, max_rows: int = 1 << 20):
        """This rank's row groups (after statistics pruning) in runs of whole
        row groups of about ``max_rows`` rows, each decoded on its own
        (exec/morsel.py)."""
        groups = self.prune(self.my_row_groups(ctx), filters)
        run, rows = [], 0
        for fi, rg in groups:
            n = self._meta[fi].row_group(rg).num_rows
            if run and rows + n > max_rows:
                yield self.scan(columns, ctx, groups=run)
                run, rows = [], 0
            run.append((fi, rg))
            rows += n
        if run:
            yield self.scan(columns, ctx, groups=run)

    def scan(self, columns: Sequence[str], ctx, filters=None, groups=None) -> Batch:
        device = ctx.device if ctx is not None else torch.device("cpu")
        all_groups = self.my_row_groups(ctx) if groups is None else list(groups)
        groups = self.prune(all_groups, filters)
        stats = {"row_groups": len(all_groups), "row_groups_read": len(groups),
                 "row_groups_pruned": len(all_groups) - len(groups)}
        out: Dict[str, Column] = {}
        missing = list(columns)
        if missing and device.type == "cuda" and GPU_DECODE:
            # GPU page decode (csrc/kernels/parquet.hip); columns it does not
            # handle stay in `missing` for the host decoder below
            decoded, rejected = self._gpu().read([(c, self._field(c).dtype) for c in missing], groups, device)
            stats.update(self._gpu().last_stats, host_columns=sorted(rejected))
            out.update(decoded)
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
                out[c] = Column.from_arrow(t.column(c), device=device, dtype=self._field(c).dtype)
        self.last_gpu_stats = stats
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

    def evict(self):
        """Nothing is held by the source (the cache tier owns resident columns)."""


# ---------------------------------------------------------------- statistics
def _stat_value(raw, phys: str, dec_scale: Optional[int]) -> Optional[object]:
    """One min/max statistic (physical value, ``Statistics.min_raw``) as a
    comparable Python value in the units of ``pushable_filters``."""
    if raw is None:
        return None
    if phys in ("INT32", "INT64"):
        v = int(raw)
    elif phys in ("FLOAT", "DOUBLE"):
        return float(raw)
    elif phys == "BYTE_ARRAY":
        try:
            return raw.decode("utf-8") if isinstance(raw, (bytes, bytearray)) else str(raw)
        except UnicodeDecodeError:
            return None
    elif phys == "FIXED_LEN_BYTE_ARRAY" and isinstance(raw, (bytes, bytearray)):
        v = int.from_bytes(raw, "big", signed=True)
    else:
        return None
    if dec_scale is not None:
        return Fraction(v, 10 ** dec_scale)
    return v


_ALL_NULL = "all-null"


def _group_bounds(m, g, idx):
    """Row group ``g``'s statistics for leaf column ``idx``: (min, max), the
    marker _ALL_NULL, or None (no usable statistics)."""
    if idx is None:
        return None
    cm = g.column(idx)
    st = cm.statistics
    if st is None:
        return None
    if st.has_null_count and st.null_count == g.num_rows and g.num_rows > 0:
        return _ALL_NULL
    if not st.has_min_max:
        return None
    sc = m.schema.column(idx)
    lt = sc.logical_type
    scale = sc.scale if lt is not None and lt.type == "DECIMAL" else None
    lo = _stat_value(st.min_raw, cm.physical_type, scale)
    hi = _stat_value(st.max_raw, cm.physical_type, scale)
    if lo is None or hi is None:
        return None
    return lo, hi


def _refuted(g, m, f) -> bool:
    """True when row group ``g`` cannot hold a row satisfying ``f``."""
    name, op, values = f
    return _bounds_refute(_group_bounds(m, g, _leaf_index(m, name)), op, values)


def _bounds_refute(b, op, values) -> bool:
    if b is None:
        return False
    if b is _ALL_NULL:
        return True     # only NULLs: no comparison can be true
    lo, hi = b
    try:
        if op == "in":
            return all(v < lo or v > hi for v in values)
        v = values[0]
        if op == "=":
            return v < lo or v > hi
        if op == "<":
            return lo >= v
        if op == "<=":
            return lo > v
        if op == ">":
            return hi <= v
        if op == ">=":
            return hi < v
    except TypeError:
        return False
    return False


def _leaf_index(m, name: str) -> Optional[int]:
    sch = m.schema
    for i in range(len(sch)):
        if sch.column(i).path == name:
            return i
    return None


def pushable_filters(filters, name_of) -> List[tuple]:
    """Scan conjuncts usable for statistics pruning: ``col OP literal`` and
    ``col IN (literals)`` (non-null literals), as (column name, op, values)
    with literals in the units of ``_stat_value`` (decimals as Fractions)."""
    from ..sql.expr import BinOp, ColRef, InList, Lit
    out = []

    def lit(e):
        if not isinstance(e, Lit) or e.value is None:
            return None
        if e.dtype.is_decimal:
            return Fraction(int(e.value), 10 ** e.dtype.scale)
        if e.dtype.is_string or e.dtype.kind in ("int8", "int16", "int32", "int64", "date32", "float32", "float64"):
            return e.value
        return None

    for f in filters or []:
        if isinstance(f, BinOp) and f.op in _FLIP:
            a, b, op = f.left, f.right, f.op
            if isinstance(b, ColRef) and isinstance(a, Lit):
                a, b, op = b, a, _FLIP[op]
            if isinstance(a, ColRef) and a.cid in name_of:
                v = lit(b)
                if v is not None and a.dtype.kind != "bool":
                    out.append((name_of[a.cid], op, [v]))
        elif isinstance(f, InList) and not f.negated and isinstance(f.x, ColRef) and f.x.cid in name_of:
            vals = [lit(v) for v in f.values]
            if vals and all(v is not None for v in vals):
                out.append((name_of[f.x.cid], "in", vals))
    return out


def write_parquet(table: pa.Table, path: str, row_group_size: int = 1 << 20, compression: str = "snappy"):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    pq.write_table(table, path, row_group_size=row_group_size, compression=compression)
