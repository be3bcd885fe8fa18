"""Execution context and the physical operator base class.

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
from ..ops.select import exclusive_scan, mask_to_indices
from ..sql import logical as L
from ..sql.expr import AggCall, BinOp, ColRef, Expr, Lit, and_all, col_refs, conjuncts
from ..utils.errors import ExecutionError, NotSupported
from . import fused
from .expr_eval import Evaluator, Scalar, _convert_tensor



class ExecContext:
    """Per-query execution state: device, communicator, metrics, subquery cache."""

    def take_deferred(self):
        """The deferred device error flags as ONE device tensor plus their
        messages (None when there are none), handed to the result's host copy
        (engine.py _host_columns) instead of a readback of their own."""
        if not self.deferred_checks:
            return None
        import torch
        checks, self.deferred_checks = self.deferred_checks, []
        return torch.cat([f.reshape(-1).to(torch.int64) for f, _ in checks]), [m for _, m in checks]

    def check_deferred(self) -> None:
        """Raise the first deferred device error whose flag is set (ONE
        readback for all of them, at the end of the query)."""
        if not self.deferred_checks:
            return
        import torch
        from ..ops._lib import to_host_ints
        from ..utils.errors import ExecutionError
        flags = to_host_ints(torch.cat([f.reshape(-1).to(torch.int64) for f, _ in self.deferred_checks]))
        checks, self.deferred_checks = self.deferred_checks, []
        for v, (_, msg) in zip(flags, checks):
            if v:
                raise ExecutionError(msg)

    def __init__(self, engine=None, device="cpu", comm=None, analyze: bool = False):
        self.engine = engine
        self.device = torch.device(device)
        self.comm = comm
        self.analyze = analyze
        self.metrics: Dict[int, dict] = {}
        self._subq: Dict[int, object] = {}
        self.evaluator = Evaluator(self)
        self.spans: Dict[str, list] = {}  # phase -> [total ms, calls] (EXPLAIN ANALYZE only)
        self.scan_cache: Dict[tuple, tuple] = {}  # (source, filters) -> (row ids, gathered columns by name)
        # device working-memory budget of the join operators (bytes, None =
        # unbounded): a join whose inputs exceed it runs partitioned, spilling
        # partitions to pinned host memory (``grace_join``)
        sess = getattr(engine, "session", None) or {}
        gb = sess.get("device_budget_gb", os.environ.get("IGLOO_DEVICE_BUDGET_GB"))
        self.budget = int(float(gb) * 2**30) if gb not in (None, "", 0, "0") else None
        self.spill = {"joins": 0, "partitions": 0, "bytes": 0}
        # rows of base tables this query read (each table once; index / range
        # searches into a resident column subtract the rows they skipped)
        self.rows_scanned = 0
        self._scanned_sources: set = set()
        # table sources this query read (engine.py polls their CDC probes before
        # replaying the query's graph) and the cache-tier keys it was served
        # from (a graph replay refreshes their LRU position)
        self.sources: list = []
        self.cache_keys: list = []
        # morsel pipelines (exec/morsel.py): the streamed scan's current morsel
        # (scan node id, raw batch, tag), results of the operators a pipeline
        # computes once (node id -> Batch, for the node ids in memo_ids)
        self.morsel = None
        self.memo: Optional[dict] = None
        self.memo_ids: set = set()
        self.morsel_depth = 0
        self.morsels = {"pipelines": 0, "morsels": 0, "rows": 0, "bytes": 0}
        self.semi_builds: dict = {}   # aggregated SEMI / ANTI build sides (exec/morsel.py)
        # raw scans a fast-path check already read (ScanExec.peek_raw): the
        # general path that runs when the check fails reuses them
        self.raw_peeks: Dict[int, Batch] = {}
        # device error flags checked once when the query's result is ready
        # (generated kernels' decimal-overflow flags: no mid-query sync)
        self.deferred_checks: list = []
        # aggregate subtrees computed once per query (exec/aggregate.py _subtree_key)
        self.subplans: Dict[str, tuple] = {}
        # SPMD: {id(source): key column} of the replicated table this query
        # splits by key range (parallel/slicing.py plan_slices)
        self.slices: Dict[int, str] = {}

    def note_scan(self, source, rows: int) -> None:
        if id(source) not in self._scanned_sources:
            self._scanned_sources.add(id(source))
            self.sources.append(source)
            self.rows_scanned += rows

    def note_partial_read(self, t: torch.Tensor, rows_read: int) -> None:
        """A join searched resident column ``t`` and touched only ``rows_read`` rows."""
        if getattr(t, "_igloo_resident", False):
            self.rows_scanned -= max(0, t.numel() - rows_read)

    def span(self, name: str):
        """Time a phase inside an operator (device-synchronised; no-op unless
        analyzing); a roctx range under IGLOO_DEBUG=roctx (utils/trace.py)."""
        if self.analyze:
            return _Span(self, name)
        return _trace.Range(name) if _trace.ENABLED else _NOSPAN

    def span_report(self) -> str:
        rows = sorted(self.spans.items(), key=lambda kv: -kv[1][0])
        return "\n".join(f"  {k:<28} {v[0]:10.3f} ms  x{v[1]}" for k, v in rows)

    @property
    def world(self) -> int:
        return self.comm.world_size if self.comm is not None else 1

    @property
    def spmd(self) -> bool:
        """Rows are spread over ranks: exchanges run (also a forced world of
        one, parallel/comm.py ``force_spmd``, which runs every collective)."""
        return self.comm is not None and self.comm.spmd

    def scalar_subquery(self, e) -> object:
        key = id(e.plan)
        if key not in self._subq:
            from .planner import execute_plan
            b = execute_plan(e.plan, self)
            if self.spmd:
                from ..parallel.exchange import gather_all
                b = gather_all(b, self)
            if b.num_rows > 1:
                raise ExecutionError("scalar subquery returned more than one row")
            if b.num_rows == 0:
                self._subq[key] = None
            else:
                col = b.columns[e.plan.schema[0].cid]
                t = e.plan.schema[0].dtype
                dv = _device_scalar(col, t)
                if dv is not _NO_SCALAR:
                    self._subq[key] = dv
                    return dv
                v = col.to_arrow()[0].as_py()
                if t.is_decimal and v is not None:
                    from decimal import Decimal
                    v = int(Decimal(v).scaleb(t.scale))
                elif t.kind == "date32" and v is not None:
                    import datetime
                    v = (v - datetime.date(1970, 1, 1)).days
                self._subq[key] = v
        return self._subq[key]


_NO_SCALAR = object()


def _device_scalar(col: Column, t):
    """First value of a device column through the replayable readback path
    (ops/_lib.py to_host_ints): integers, dates (days) and decimals (scaled
    integers) as int, floats bit-exact, NULL as None. Other types return
    ``_NO_SCALAR`` (host conversion)."""
    d = col.data
    if not d.is_cuda or col.offsets is not None or col.dictionary is not None or t.kind in ("null", "timestamp") \
            or t.is_string:
        return _NO_SCALAR
    if col.valid is not None and not to_host_int(col.valid[:1]):
        return None
    if d.dim() == 2:
        lo, hi = to_host_ints(d[:1].reshape(-1))
        return (hi << 64) | (lo & 0xFFFFFFFFFFFFFFFF)
    if d.dtype.is_floating_point:
        return to_host_f64s(d[:1])[0]
    if d.dtype == torch.bool:
        return bool(to_host_int(d[:1]))
    return to_host_int(d[:1])


class _Span:
    __slots__ = ("ctx", "name", "t0")

    def __init__(self, ctx, name):
        self.ctx, self.name = ctx, name

    def __enter__(self):
        _sync(self.ctx)
        self.t0 = time.perf_counter()

    def __exit__(self, *exc):
        _sync(self.ctx)
        v = self.ctx.spans.setdefault(self.name, [0.0, 0])
        v[0] += (time.perf_counter() - self.t0) * 1e3
        v[1] += 1
        return False


class _NoSpan:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NOSPAN = _NoSpan()


def _sync(ctx):
    if ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


class ExecNode:
    children: List["ExecNode"]
    logical: L.Plan

    def execute(self, ctx: ExecContext) -> Batch:
        if ctx.memo is not None and id(self) in ctx.memo_ids:
            # computed once per morsel pipeline (exec/morsel.py)
            hit = ctx.memo.get(id(self))
            if hit is None:
                hit = ctx.memo[id(self)] = self._execute_traced(ctx)
            return hit
        return self._execute_traced(ctx)

    def _execute_traced(self, ctx: ExecContext) -> Batch:
        if _trace.ENABLED:
            _trace.push(type(self).__name__)
            try:
                return self._execute(ctx)
            finally:
                _trace.pop()
        return self._execute(ctx)

    def _execute(self, ctx: ExecContext) -> Batch:
        if ctx.analyze:
            _sync(ctx)
            t0 = time.perf_counter()
        c0 = (ctx.comm.calls, ctx.comm.bytes_sent) if ctx.analyze and ctx.comm is not None else (0, 0)
        out = self._run(ctx)
        if ctx.analyze:
            _sync(ctx)
            m = {"ms": (time.perf_counter() - t0) * 1e3, "rows": out.num_rows, "dist": getattr(out, "dist", None)}
            if ctx.comm is not None:
                m["collectives"] = ctx.comm.calls - c0[0]
                m["bytes"] = ctx.comm.bytes_sent - c0[1]
            ctx.metrics[id(self)] = m
        return out

    def _run(self, ctx: ExecContext) -> Batch:  # pragma: no cover
        raise NotImplementedError

    def name(self) -> str:
        return type(self).__name__

    def describe(self) -> str:
        return self.logical.label()

    def explain(self, ctx: Optional[ExecContext] = None, indent: int = 0) -> str:
        m = ""
        if ctx is not None and id(self) in ctx.metrics:
            mm = ctx.metrics[id(self)]
            m = f"  [rows={mm['rows']}, time={mm['ms']:.3f}ms]"
        lines = ["  " * indent + f"{self.name()}: {self.describe()}{m}"]
        for c in self.children:
            lines.append(c.explain(ctx, indent + 1))
        return "\n".join(lines)
