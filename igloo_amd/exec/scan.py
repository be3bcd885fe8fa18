"""Scan, values, filter and projection operators.

One of the five operator modules (context, scan, joins, aggregate, sorting)."""
from __future__ import annotations

import math
import os
import re
import time
from fractions import Fraction
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import torch

from .. import types as T
from ..columnar import Batch, Column, batch_device
from ..ops import agg as A
from ..ops import hashing as H
from ..ops import misc as M
from ..ops import strings as S
from ..ops._lib import (check_not_capturing, device_ints, launch, ptr, stream, to_host_f64s, to_host_int,
                       to_host_ints, unlogged)
from ..utils import trace as _trace
from ..ops.gather import gather_tensor, take, take_many
from ..ops.select import MaskRows, compact_columns, exclusive_scan, mask_to_indices
from ..sql import logical as L
from ..sql.expr import AggCall, BinOp, ColRef, Expr, Lit, and_all, col_refs, conjuncts
from ..utils.errors import ExecutionError, NotSupported
from . import fused
from .expr_eval import Evaluator, Scalar, _convert_tensor
from .context import ExecContext, ExecNode, _NOSPAN, _sync


# ============================================================================ scan
_CID = re.compile(r"#\d+")

LATE_SCAN = True
NDV_DERIVED = True



#: fused mask compaction of a filtered scan's columns (COMPACT = False: mask ->
#: indices -> gather, the A/B baseline)
COMPACT = True


def _tag_base(col: Column, src: Column, n_src: int):
    if NDV_DERIVED and col.valid is None and not col.is_dict:
        try:   # filtered subset of a source column: its NDV derives from the source's
            col.data._igloo_base = (src, n_src)
        except (AttributeError, RuntimeError):
            pass


class ScanExec(ExecNode):
    #: set by a parent multi-way join: a filtered scan may hand over its rows
    #: as indices into the source (LateBatch) instead of gathered columns
    late_ok = False
    #: set by a parent semi / anti join: the subquery side of EXISTS may stay
    #: in index form too (its filter mask then decides which rows exist,
    #: exec/joins.py _in_place_semi); single-process, unbudgeted runs only
    late_semi = False

    def __init__(self, logical: L.Scan):
        self.logical = logical
        self.children = []

    def describe(self):
        s = self.logical
        f = f", filters=[{', '.join(x.sql() for x in s.filters)}]" if s.filters else ""
        return f"{s.table} projection=[{', '.join(c.name for c in s.schema)}]{f}"

    def column_names(self):
        """(source column names to read, their cids, cid -> ColInfo): the
        projection plus every filter input."""
        s = self.logical
        table_cols = getattr(s, "table_cols", s.schema)
        by_cid = {c.cid: c for c in table_cols}
        for c in s.schema:
            by_cid[c.cid] = c
        need = {c.cid for c in s.schema}
        for f in s.filters:
            need |= col_refs(f)
        return [by_cid[cid].name for cid in sorted(need)], need, by_cid

    def pushable(self):
        """Filters the source can test against row-group statistics (or None)."""
        s = self.logical
        if not (s.filters and getattr(s.source, "prunes", False)):
            return None
        from ..connectors.parquet import pushable_filters
        _, need, by_cid = self.column_names()
        return pushable_filters(s.filters, {cid: by_cid[cid].name for cid in need})

    def scan_raw(self, ctx) -> Batch:
        """Scanned columns (projection + filter inputs) before filtering, keyed by cid."""
        if ctx.morsel is None and id(self) in ctx.raw_peeks:
            return ctx.raw_peeks.pop(id(self))
        s = self.logical
        table_cols = getattr(s, "table_cols", s.schema)
        names, need, by_cid = self.column_names()
        slice_key = ctx.slices.get(id(s.source)) if ctx.morsel is None else None
        if ctx.morsel is not None and ctx.morsel[0] == id(self):
            raw = ctx.morsel[1]          # the current morsel of a pipeline (exec/morsel.py)
        elif slice_key is not None:
            # a query over replicated tables only: this rank's key-range
            # slice of the largest one (parallel/slicing.py); read whole
            # (no row-group pruning), so every scan of the table slices alike
            from ..parallel.slicing import slice_columns
            with ctx.span("scan.source"):
                full = s.source.scan(names + ([slice_key] if slice_key not in names else []), ctx)
                ctx.note_scan(s.source, full.num_rows)
                scols, n, tag = slice_columns(full.columns, full.num_rows, slice_key, ctx.world, ctx.comm.rank)
            cols = {cid: scols[by_cid[cid].name] for cid in sorted(need)}
            kc = [cid for cid in sorted(need) if by_cid[cid].name == slice_key]
            # (an unsorted key column splits by rows: partitioned, placed by no key)
            return Batch(cols, n, (tag,) + tuple(kc) if tag is not None and kc else None)
        else:
            with ctx.span("scan.source"):
                pf = self.pushable()
                # row-group statistics pruning (the filter is still applied below)
                raw = s.source.scan(names, ctx, filters=pf) if pf is not None else s.source.scan(names, ctx)
            ctx.note_scan(s.source, raw.num_rows)
        cols = {cid: raw.columns[by_cid[cid].name] for cid in sorted(need)}
        dist = None
        if ctx.spmd:
            if getattr(s.source, "replicated", False):
                dist = ("replicated",)
            elif getattr(s.source, "partitioned_by", None):
                pc = [c.cid for c in table_cols if c.name == s.source.partitioned_by]
                dist = ("hash", pc[0]) if pc else None
        return Batch(cols, raw.num_rows, dist)

    def peek_raw(self, ctx) -> Batch:
        """``scan_raw`` for a fast-path check that may still fall back to the
        general path: the batch is kept so the scan is not read (decoded,
        copied to the device) a second time when the check fails."""
        raw = self.scan_raw(ctx)
        if ctx.morsel is None:
            ctx.raw_peeks[id(self)] = raw
        return raw

    @property
    def predicate(self) -> Optional[Expr]:
        return and_all(self.logical.filters) if self.logical.filters else None

    def finish(self, b: Batch, ctx) -> Batch:
        """Apply the fused scan filter and the projection to a ``scan_raw`` batch."""
        s = self.logical
        out_cids = [c.cid for c in s.schema]
        if s.filters:
            # one query scanning a table twice under the same filter (Q21's l1 and
            # l3, Q11/Q15 view repeats) evaluates it and gathers each column once
            name = {c.cid: c.name for c in getattr(s, "table_cols", s.schema)}
            name.update({c.cid: c.name for c in s.schema})
            fsql = tuple(sorted(_CID.sub("", f.sql()) for f in s.filters))
            key = (id(s.source), b.num_rows, fsql, ctx.morsel[2] if ctx.morsel is not None else None)
            hit = None if any("random" in x.lower() for x in fsql) else ctx.scan_cache.get(key)
            late = (self.late_ok or (self.late_semi and not ctx.spmd and ctx.budget is None)) and LATE_SCAN \
                and ctx.device.type == "cuda"
            if hit is None:
                with ctx.span("scan.filter_eval"):
                    m = predicate_mask(self.predicate, b, ctx)
                if COMPACT and not late and ctx.device.type == "cuda":
                    # every projected column in the same pass as the mask's
                    # compaction (select.hip tile_compact): no index vector
                    # between the mask and the column copies
                    with ctx.span("scan.filter_compact"):
                        idx, cols = compact_columns(m, [b.columns[c] for c in out_cids])
                    taken = {}
                    for c, col in zip(out_cids, cols):
                        _tag_base(col, b.columns[c], b.num_rows)
                        taken[name[c]] = col
                    hit = ctx.scan_cache[key] = (idx, taken)
                else:
                    with ctx.span("scan.filter_eval"):
                        # (index form: the count's readback may wait for the
                        # parent join's, MaskRows.resolve)
                        rows = MaskRows(m, defer=late)
                    # (the mask stays with the index form: a join may probe the
                    # table's own key column under it instead of gathering it,
                    # and then the index vector is never written)
                    hit = ctx.scan_cache[key] = (rows, {})
            rows, taken_by_name = hit
            if late:
                # index form: the join gathers its key columns now and payload
                # columns only for the rows that survive it
                src = Batch({c: b.columns[c] for c in out_cids}, b.num_rows, b.dist)
                return _LazyScanBatch(src, rows, name, taken_by_name, ctx)
            todo = [c for c in out_cids if name[c] not in taken_by_name]
            if todo:
                with ctx.span("scan.filter_gather"):
                    if isinstance(rows, MaskRows) and COMPACT and rows.mask.is_cuda:
                        # the index form of an earlier scan (Q21's l1 for l3):
                        # the columns compacted straight from its mask
                        taken = compact_columns(rows.mask, [b.columns[c] for c in todo], total=rows.total,
                                                want_idx=False)[1]
                    else:
                        taken = take_many([b.columns[c] for c in todo],
                                          rows.idx if isinstance(rows, MaskRows) else rows)
                    for c, col in zip(todo, taken):
                        _tag_base(col, b.columns[c], b.num_rows)
                        taken_by_name[name[c]] = col
            n_rows = rows.total if isinstance(rows, MaskRows) else rows.numel()
            return Batch({c: taken_by_name[name[c]] for c in out_cids}, n_rows, b.dist)
        return Batch({c: b.columns[c] for c in out_cids}, b.num_rows, b.dist)

    def _run(self, ctx):
        # (under SPMD too: a filtered scan is rank-local, so each rank may stream
        # its own rows or not without changing any collective)
        if ctx.budget is not None and self.logical.filters \
                and not (ctx.morsel is not None and ctx.morsel[0] == id(self)):
            from .morsel import streamed_scan
            out = streamed_scan(self, ctx)
            if out is not None:
                return out
        return self.finish(self.scan_raw(ctx), ctx)


def predicate_mask(pred: Expr, b: Batch, ctx) -> torch.Tensor:
    """Filter mask: one fused VM kernel on the GPU when the predicate fits, else
    node-by-node evaluation."""
    if ctx.device.type == "cuda":
        m = fused.predicate_mask(pred, b, ctx.evaluator)
        if m is not None:
            return m
    return ctx.evaluator.mask(pred, b)


class LazyBatch(Batch):
    """A Batch materialised on first access (lets the aggregate fuse the scan
    filter and skip building the filtered batch altogether)."""

    def __init__(self, thunk, dist):  # noqa: D401 - no Batch.__init__: attributes are lazy
        self._thunk = thunk
        self._b = None
        self.dist = dist

    def _get(self) -> Batch:
        if self._b is None:
            self._b = self._thunk()
        return self._b

    @property
    def columns(self):  # type: ignore[override]
        return self._get().columns

    @property
    def num_rows(self):  # type: ignore[override]
        return self._get().num_rows


class FragmentInputExec(ExecNode):
    """Output of another query fragment, materialized by the fragment scheduler."""

    def __init__(self, logical: L.FragmentRef):
        self.logical = logical
        self.children = []

    def _run(self, ctx):
        inputs = getattr(ctx, "fragment_inputs", None) or {}
        if self.logical.fragment_id not in inputs:
            raise ExecutionError(f"input of fragment {self.logical.fragment_id} is not available")
        return inputs[self.logical.fragment_id]


class ValuesExec(ExecNode):
    def __init__(self, logical: L.Values):
        self.logical = logical
        self.children = []

    def _run(self, ctx):
        v = self.logical
        n = len(v.rows)
        cols = {}
        for j, ci in enumerate(v.schema):
            vals = []
            for r in v.rows:
                e = ctx.evaluator.eval(r[j], Batch({}, 1))
                vals.append(e.value if isinstance(e, Scalar) else e.to_pylist()[0])
            cols[ci.cid] = _column_from_values(vals, ci.dtype, ctx.device)
        return Batch(cols, n, ("replicated",) if ctx.spmd else None)


class UnnestExec(ExecNode):
    """Rows of the child repeated once per element of a list column
    (ops/nested.py unnest_rows: the range-expansion kernel over the lists'
    (start, length) pairs, then one gather per column)."""

    def __init__(self, logical: L.Unnest, child: ExecNode):
        self.logical = logical
        self.children = [child]

    def _run(self, ctx):
        from ..ops import nested as NS
        b = self.children[0].execute(ctx)
        u = self.logical
        lst = b.columns[u.list_col.cid]
        parent, vals = NS.unnest_rows(lst)
        keys = [k for k in b.columns if k != u.list_col.cid]
        cols = dict(zip(keys, take_many([b.columns[k] for k in keys], parent))) if keys else {}
        cols[u.list_col.cid] = take(lst, parent)
        cols[u.out.cid] = vals
        return Batch(cols, parent.numel(), b.dist)


class TableFunctionExec(ExecNode):
    """generate_series / range rows made on the device (one arange), unnest
    of a constant list: the list's child values."""

    def __init__(self, logical: L.TableFunction):
        self.logical = logical
        self.children = []

    def _run(self, ctx):
        t = self.logical
        ci = t.schema[0]
        dist = ("replicated",) if ctx.spmd else None
        if t.name in ("generate_series", "range"):
            start, stop, step = t.args
            if step == 0:
                raise ExecutionError(f"{t.name}: step cannot be zero")
            if t.name == "generate_series":
                stop = stop + (1 if step > 0 else -1)
            n = max(0, -(-(stop - start) // step)) if step > 0 else max(0, -(-(start - stop) // -step))
            vals = torch.arange(n, dtype=torch.int64, device=ctx.device) * step + start if n else \
                torch.zeros(0, dtype=torch.int64, device=ctx.device)
            return Batch({ci.cid: Column(ci.dtype, vals)}, n, dist)
        if t.name == "unnest":
            from ..ops import nested as NS
            v = ctx.evaluator.eval(t.args[0], Batch({}, 1))
            lst = v if isinstance(v, Column) else NS.scalar_to_column(v.value, t.args[0].dtype, 1, ctx.device)
            child = NS.unnest_values(lst, ctx.device)
            return Batch({ci.cid: child}, len(child), dist)
        raise NotSupported(f"table function {t.name}")


def _column_from_values(vals, dtype, device) -> Column:
    if dtype.is_decimal:
        t = torch.tensor([0 if v is None else int(v) for v in vals], dtype=torch.int64)
        valid = None if all(v is not None for v in vals) else torch.tensor([v is not None for v in vals])
        return Column(dtype, t, valid).to(device)
    if dtype.kind == "date32":
        t = torch.tensor([0 if v is None else int(v) for v in vals], dtype=torch.int32)
        valid = None if all(v is not None for v in vals) else torch.tensor([v is not None for v in vals])
        return Column(dtype, t, valid).to(device)
    if dtype.kind == "null":
        return Column.full(None, T.NULL, len(vals), device)
    return Column.from_arrow(pa.array(vals, dtype.to_arrow()), device=device, dtype=dtype,
                             dict_encode=False if dtype.is_string else None)


# ================================================================ filter / project
class FilterExec(ExecNode):
    def __init__(self, logical: L.Filter, child: ExecNode):
        self.logical = logical
        self.children = [child]
        from .aggregate import HashAggExec
        if isinstance(child, HashAggExec):
            child.having = logical.pred     # HAVING: the aggregate may apply it while grouping

    def describe(self):
        return self.logical.pred.sql()

    def _run(self, ctx):
        b = self.children[0].execute(ctx)
        return filter_batch(b, self.logical.pred, ctx)


def filter_batch(b: Batch, pred: Expr, ctx) -> Batch:
    with ctx.span("filter.eval"):
        m = predicate_mask(pred, b, ctx)
        idx = mask_to_indices(m)
    if idx.numel() == b.num_rows:
        return b
    keys = list(b.columns)
    with ctx.span("filter.gather"):
        taken = take_many([b.columns[k] for k in keys], idx)
    return Batch(dict(zip(keys, taken)), idx.numel(), b.dist)


class ProjectExec(ExecNode):
    def __init__(self, logical: L.Project, child: ExecNode):
        self.logical = logical
        self.children = [child]

    def describe(self):
        return ", ".join(e.sql() if isinstance(e, ColRef) and e.cid == c.cid else f"{e.sql()} AS {c.name}"
                         for c, e in self.logical.exprs)

    def identity(self) -> bool:
        """Every output column is an input column under its own id."""
        return all(isinstance(e, ColRef) and e.cid == ci.cid for ci, e in self.logical.exprs)

    def _run(self, ctx):
        b = self.children[0].execute(ctx)
        if isinstance(b, _LazyScanBatch) and self.identity():
            return b        # a filtered scan in index form stays so (its extra columns go unread)
        from ..parallel.exchange import keyed
        cols = {}
        d = b.dist
        # replicated / arbitrary carry over; a key placement keeps the
        # output columns that are its key columns (renamed or not)
        dist = d if d == ("replicated",) else None
        placed = []
        for ci, e in self.logical.exprs:
            cols[ci.cid] = ctx.evaluator.column(e, b)
            if keyed(d) and isinstance(e, ColRef) and e.cid in d[1:]:
                placed.append(ci.cid)
        if placed:
            dist = (d[0],) + tuple(placed)
        elif keyed(d):
            dist = None
        return Batch(cols, b.num_rows, dist)



class _ScanColumns:
    """Mapping view of a _LazyScanBatch: gathers a column on first read."""

    def __init__(self, b: "_LazyScanBatch"):
        self._b = b

    def __getitem__(self, cid):
        return self._b.gather(cid)

    def get(self, cid, default=None):
        return self._b.gather(cid) if cid in self._b.src.columns else default

    def __contains__(self, cid):
        return cid in self._b.src.columns

    def __iter__(self):
        return iter(self._b.src.columns)

    def __len__(self):
        return len(self._b.src.columns)

    def keys(self):
        return list(self._b.src.columns)

    def values(self):
        return (self._b.gather(c) for c in list(self._b.src.columns))

    def items(self):
        return ((c, self._b.gather(c)) for c in list(self._b.src.columns))


class _LazyScanBatch(Batch):
    """A filtered scan whose columns are gathered on first read (shared with
    other scans of the same table under the same filter in the query). A
    LateBatch over it gathers never-read payload columns straight from the
    source through the composed row index — only for rows that survive the
    join — while its own row indices stay those of the filtered scan."""

    def __init__(self, src: Batch, rows, names: dict, shared: dict, ctx):  # noqa: D401
        """rows: the surviving row ids (tensor) or ops/select.py MaskRows."""
        self.src, self._rows, self._names, self._shared, self._ctx = src, rows, names, shared, ctx
        # bool[src rows]: the filter the rows came from (None: not kept)
        self.mask = rows.mask if isinstance(rows, MaskRows) else None
        self.dist = src.dist
        self.out_dist = None
        self.columns = _ScanColumns(self)

    @property
    def num_rows(self) -> int:  # type: ignore[override]
        r = self._rows
        return r.total if isinstance(r, MaskRows) else r.numel()

    @property
    def pending_rows(self):
        """The MaskRows whose count is not read back yet (or None)."""
        r = self._rows
        return r if isinstance(r, MaskRows) and r._total is None else None

    @property
    def idx(self) -> torch.Tensor:
        """Row ids into ``src`` (written on first use)."""
        return self._rows.idx if isinstance(self._rows, MaskRows) else self._rows

    @property
    def device(self):
        return self._rows.mask.device if isinstance(self._rows, MaskRows) else self._rows.device

    def has(self, cid) -> bool:
        return self._names[cid] in self._shared

    def gather(self, cid) -> Column:
        c = self._shared.get(self._names[cid])
        if c is None:
            with self._ctx.span("scan.filter_gather"):
                c = take(self.src.columns[cid], self.idx)
            _tag_base(c, self.src.columns[cid], self.src.num_rows)
            self._shared[self._names[cid]] = c
        return c

    def take_rows(self, cids, rows: torch.Tensor) -> List[Column]:
        """Columns at filtered-scan rows ``rows``; unread ones via the source."""
        have = [c for c in cids if self.has(c)]
        pend = [c for c in cids if not self.has(c)]
        out = dict(zip(have, take_many([self._shared[self._names[c]] for c in have], rows))) if have else {}
        if pend:
            comp = gather_tensor(self.idx, rows)
            out.update(zip(pend, take_many([self.src.columns[c] for c in pend], comp)))
        return [out[c] for c in cids]
