"""Morsel-driven streaming and external sort under a device memory budget.

The reference streams 1024-row record batches from its Parquet scan through
bounded channels into the operators above it (reference
crates/engine/src/operators/parquet_scan.rs:44-66; the hash join's probe
channel, crates/engine/src/operators/hash_join.rs:136-138), so no operator
holds a whole table. Here operators normally take whole device-resident
columns (the HBM tier holds the tables: 288 GB per GPU). When a session sets a
device budget (``device_budget_gb`` / IGLOO_DEVICE_BUDGET_GB) and a scan's
columns exceed a fraction of it, the aggregation above that scan runs as a
morsel pipeline instead:

* the scan is read in morsels of whole row groups (Parquet) or row ranges
  (host-resident memory tables), each sized to ``budget / MORSEL_FRACTION``
  bytes, and moved to the device one at a time;
* every morsel flows through the operators between the scan and the
  aggregate (filters, projections, joins whose other side is built once and
  memoised for the whole pipeline) and ends as PARTIAL aggregate states — the
  same phase-1 states the SPMD exchange merges across ranks
  (parallel/exchange.py ``partial_plan`` / ``merge_partials``);
* the partial states of all morsels are concatenated and merged once.

A scan can stream when every operator between it and the aggregate
distributes over a union of row sets: filters, projections, inner joins (either
side), the preserved side of left joins, the probe side of semi / anti joins,
and inner multi-way joins. Anything else (a scan under another aggregate, a
sort, a limit, the build side of an outer / semi join) runs whole, where the
grace join (joins.py ``grace_join``) bounds its joins.

``external_sort`` is the ORDER BY counterpart: an input over the budget is
range-partitioned on its leading sort key by sampled splitters, the partitions
are staged in pinned host memory, and each is brought back, sorted on the
device and staged again; their concatenation is the sorted result.

EXPLAIN ANALYZE reports both ("morsels: ..." and "spill: ...").
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from ..columnar import Batch

#: a morsel's scanned bytes are at most budget / MORSEL_FRACTION
MORSEL_FRACTION = 8
#: stream a scan whose columns exceed budget / STREAM_FRACTION
STREAM_FRACTION = 4
MORSEL_MIN_ROWS = 1 << 14
#: bytes per row assumed for a string column without statistics
STRING_ROW_BYTES = 40


# --------------------------------------------------------------- planning
def _walk(node):
    yield node
    for c in node.children:
        yield from _walk(c)


def _contains(node, target) -> bool:
    return any(n is target for n in _walk(node))


def stream_path_ok(node, target) -> bool:
    """Every operator on the path from ``node`` down to scan ``target``
    distributes over a union of the scan's rows (see the module docstring)."""
    from .scan import FilterExec, ProjectExec
    from .joins import HashJoinExec, MultiJoinExec
    if node is target:
        return True
    if isinstance(node, (FilterExec, ProjectExec)):
        return stream_path_ok(node.children[0], target)
    if isinstance(node, HashJoinExec):
        kind = node.logical.kind
        left, right = node.children
        if _contains(left, target):
            return kind in ("inner", "left", "semi", "anti") and stream_path_ok(left, target)
        if _contains(right, target):
            return kind in ("inner", "right") and stream_path_ok(right, target)
        return False
    if isinstance(node, MultiJoinExec):
        # the inner-join inputs only: the trailing children are SEMI / ANTI build sides
        nin = len(node.logical.children)
        if any(_contains(c, target) for c in node.children[nin:]):
            return False
        inside = [c for c in node.children[:nin] if _contains(c, target)]
        return len(inside) == 1 and stream_path_ok(inside[0], target)
    return False


def scan_bytes(scan) -> int:
    """Bytes the scan's columns occupy (row count x column widths)."""
    src = scan.logical.source
    n = src.num_rows() if hasattr(src, "num_rows") else None
    if not n:
        return 0
    names, _, _ = scan.column_names()
    width = 0
    for name in names:
        try:
            t = src.field(name).dtype
        except Exception:  # noqa: BLE001 - sources without field lookup
            width += 8
            continue
        if t.is_string:
            width += STRING_ROW_BYTES
        else:
            width += max(1, getattr(t, "byte_width", None) or 8) + 1
    return int(n) * width


def pick_stream_scan(agg, ctx):
    """The largest streamable scan below aggregate ``agg`` whose columns exceed
    budget / STREAM_FRACTION, or None."""
    from .scan import ScanExec
    best, best_bytes = None, ctx.budget // STREAM_FRACTION
    for n in _walk(agg.children[0]):
        if not isinstance(n, ScanExec) or not getattr(n.logical.source, "can_stream", False):
            continue
        b = scan_bytes(n)
        if b > best_bytes and stream_path_ok(agg.children[0], n):
            best, best_bytes = n, b
    return best


#: morsels prepared ahead of the one being processed (0: serial)
PREFETCH_DEPTH = 1


def prefetched(gen, ctx):
    """The morsels of ``gen`` with the next ones produced ahead, on a helper
    thread and a side HIP stream: the host slice / Parquet read, its H2D copy
    and (Parquet) the page decode of morsel k+1 overlap the operators running
    on morsel k on the compute stream. Each morsel is handed over behind an
    event the compute stream waits on, and its tensors are recorded on the
    compute stream so the caching allocator does not recycle them early.
    At most PREFETCH_DEPTH morsels wait in the queue (device memory: the
    current morsel, the queued ones and the one being produced)."""
    from ..ops._lib import capturing
    if PREFETCH_DEPTH <= 0 or ctx.device.type != "cuda" or capturing():
        yield from gen
        return
    import queue
    import threading
    side = torch.cuda.Stream(device=ctx.device)
    q: "queue.Queue" = queue.Queue(maxsize=PREFETCH_DEPTH)
    stop = threading.Event()
    end = object()

    def work():
        try:
            with torch.cuda.device(ctx.device), torch.cuda.stream(side):
                for b in gen:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    while not stop.is_set():
                        try:
                            q.put((b, ev), timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
        except BaseException as e:  # noqa: BLE001 - re-raised on the consumer side
            q.put(e)
        finally:
            q.put(end)

    t = threading.Thread(target=work, name="igloo-morsel-prefetch", daemon=True)
    t.start()
    cur = torch.cuda.current_stream(ctx.device)
    try:
        while True:
            item = q.get()
            if item is end:
                break
            if isinstance(item, BaseException):
                raise item
            b, ev = item
            cur.wait_event(ev)
            for c in b.columns.values():
                for x in (c.data, c.valid, c.offsets):
                    if x is not None and x.is_cuda:
                        x.record_stream(cur)
            yield b
    finally:
        stop.set()
        while t.is_alive():
            try:
                q.get(timeout=0.1)
            except queue.Empty:
                pass
        t.join()


# -------------------------------------------------------------- execution
def streamed_aggregate(agg, ctx) -> Optional[Batch]:
    """Run aggregate node ``agg`` as a morsel pipeline when the budget calls
    for it; None when it does not (or the aggregates do not decompose)."""
    from ..parallel.exchange import _TmpIds, decomposable, partial_plan
    from .scan import ScanExec
    from .aggregate import aggregate
    from .joins import apply_key_filters
    lg = agg.logical
    if ctx.budget is None or not decomposable(lg.aggs):
        return None
    if any(getattr(a, "filter", None) is not None and _has_subquery(a.filter) for _, a in lg.aggs):
        return None
    scan = pick_stream_scan(agg, ctx)
    if ctx.spmd:
        # every rank takes the same path with the same morsel count: the
        # subtree below the aggregate may exchange rows once per morsel
        return _spmd_streamed_aggregate(agg, scan, ctx)
    if scan is None:
        return None
    child = agg.children[0]
    names, _, _ = scan.column_names()
    src = scan.logical.source
    row_bytes = max(1, scan_bytes(scan) // max(1, src.num_rows() or 1))
    max_rows = max(MORSEL_MIN_ROWS, ctx.budget // MORSEL_FRACTION // row_bytes)
    ids = _TmpIds()
    partial, plan = partial_plan(lg.aggs, ids)
    # everything below the aggregate that does not read the streamed scan is
    # computed once and reused by every morsel
    on_path = {id(n) for n in _walk(child) if _contains(n, scan)}
    saved = (ctx.memo, ctx.memo_ids, ctx.morsel)
    ctx.memo, ctx.memo_ids = {}, {id(n) for n in _walk(child) if id(n) not in on_path}
    ctx.morsel_depth += 1
    parts: List[Batch] = []
    acc = _PartialStates(lg.groups, partial, plan, ids, ctx, max(1, (src.num_rows() or 1) // max_rows + 1))
    stats = ctx.morsels
    stats["pipelines"] += 1
    try:
        with ctx.span("morsel.pipeline"):
            for k, raw in enumerate(prefetched(src.scan_morsels(names, ctx, scan.pushable(), max_rows), ctx)):
                ctx.morsel = (id(scan), raw, ("morsel", stats["pipelines"], k))
                stats["morsels"] += 1
                stats["rows"] += raw.num_rows
                stats["bytes"] += raw.nbytes
                ctx.rows_scanned += raw.num_rows
                if isinstance(child, ScanExec):
                    pb = None
                    if ctx.device.type == "cuda" and not agg.runtime_filters:
                        from . import fused
                        pb = fused.fused_scan_aggregate(lg.groups, partial, scan.scan_raw(ctx), scan.predicate, ctx)
                    b = child.execute(ctx) if pb is None else None
                else:
                    pb, b = None, child.execute(ctx)
                if pb is None:
                    if agg.runtime_filters:
                        b = apply_key_filters(b, list(agg.runtime_filters), ctx)
                    pb = aggregate(lg.groups, partial, b, ctx)
                acc.add(pb)
                ctx.scan_cache = {k2: v for k2, v in ctx.scan_cache.items() if k2[-1] != ctx.morsel[2]}
                ctx.morsel = None
    finally:
        ctx.memo, ctx.memo_ids, ctx.morsel = saved
        ctx.morsel_depth -= 1
        agg.runtime_filters = []
    with ctx.span("morsel.merge"):
        return acc.finish()


def _morsel_rows(scan, ctx) -> int:
    src = scan.logical.source
    row_bytes = max(1, scan_bytes(scan) // max(1, src.num_rows() or 1))
    return max(MORSEL_MIN_ROWS, ctx.budget // MORSEL_FRACTION // row_bytes)


def _agreed_morsels(gen_fn, scan, count: int, ctx):
    """This rank's morsels, padded with empty ones to ``count`` (every rank
    runs the same number of pipeline iterations: each may hold collectives)."""
    n = 0
    first = None
    for raw in gen_fn():
        if first is None:
            first = raw
        n += 1
        yield raw
    if n >= count:
        return
    empty = _empty_morsel(scan, first, ctx)
    for _ in range(count - n):
        yield empty


def _empty_morsel(scan, like, ctx) -> Batch:
    from ..ops.gather import take_many
    if like is None:
        names, _, _ = scan.column_names()
        like = scan.logical.source.scan(names, ctx)
    keys = list(like.columns)
    dev = next(iter(like.columns.values())).device if keys else ctx.device
    idx = torch.zeros(0, dtype=torch.int64, device=dev)
    return Batch(dict(zip(keys, take_many([like.columns[k] for k in keys], idx))) if keys else {}, 0, like.dist)


def _spmd_streamed_aggregate(agg, scan, ctx) -> Optional[Batch]:
    """Bounded-memory aggregation under SPMD: ranks agree (one all-reduce) on
    whether to stream and on the morsel count; each rank folds its morsels
    into partial states (compacted under the budget like the single-rank
    pipeline), and ``distributed_aggregate`` exchanges and merges them."""
    from ..parallel.exchange import distributed_aggregate
    from .scan import ScanExec
    from .aggregate import aggregate
    from .joins import apply_key_filters
    lg = agg.logical
    from .joins import MultiJoinExec
    if any(isinstance(n, MultiJoinExec) for n in _walk(agg.children[0])):
        # a multi-way join re-planned per morsel under SPMD carries
        # rank-dependent column sets into its exchanges: not streamed (a
        # plan-only test, alike on every rank)
        return None
    want = 0
    if scan is not None:
        src = scan.logical.source
        want = max(1, -(-(src.num_rows() or 0) // _morsel_rows(scan, ctx)))
    count = max(x[0] for x in ctx.comm.allgather_ints([want]))
    if count == 0:
        return None                   # no rank streams: the plain path on every rank
    if scan is None:
        # this rank's data fits but another's does not: stream anyway (one
        # morsel per pipeline step) so the collective sequences match
        scan = _any_stream_scan(agg)
        if scan is None:
            raise RuntimeError("SPMD morsel pipeline: no streamable scan on this rank")
    child = agg.children[0]
    names, _, _ = scan.column_names()
    src = scan.logical.source
    max_rows = _morsel_rows(scan, ctx)

    def local(groups, partial, plan):
        from ..parallel.exchange import _TmpIds
        on_path = {id(n) for n in _walk(child) if _contains(n, scan)}
        saved = (ctx.memo, ctx.memo_ids, ctx.morsel)
        ctx.memo, ctx.memo_ids = {}, {id(n) for n in _walk(child) if id(n) not in on_path}
        ctx.morsel_depth += 1
        acc = _PartialStates(groups, partial, plan, _TmpIds(), ctx, count)
        stats = ctx.morsels
        stats["pipelines"] += 1
        try:
            gen = _agreed_morsels(lambda: src.scan_morsels(names, ctx, scan.pushable(), max_rows), scan, count, ctx)
            for k, raw in enumerate(prefetched(gen, ctx)):
                ctx.morsel = (id(scan), raw, ("morsel", stats["pipelines"], k))
                stats["morsels"] += 1
                stats["rows"] += raw.num_rows
                ctx.rows_scanned += raw.num_rows
                b = child.execute(ctx)
                if agg.runtime_filters:
                    b = apply_key_filters(b, list(agg.runtime_filters), ctx)
                acc.add(aggregate(groups, partial, b, ctx))
                ctx.scan_cache = {k2: v for k2, v in ctx.scan_cache.items() if k2[-1] != ctx.morsel[2]}
                ctx.morsel = None
        finally:
            ctx.memo, ctx.memo_ids, ctx.morsel = saved
            ctx.morsel_depth -= 1
        out = acc.partials()
        return out if out is not None else _empty_partials(groups, partial, ctx)
    try:
        return distributed_aggregate(lg, Batch({}, 0, None), ctx, local=local)
    finally:
        agg.runtime_filters = []


def _empty_partials(groups, partial, ctx) -> Batch:
    from .aggregate import _empty_col
    return Batch({ci.cid: _empty_col(ci.dtype, ctx.device) for ci, _ in list(groups) + list(partial)}, 0)


def _any_stream_scan(agg):
    from .scan import ScanExec
    best, best_bytes = None, -1
    for n in _walk(agg.children[0]):
        if isinstance(n, ScanExec) and getattr(n.logical.source, "can_stream", False) \
                and stream_path_ok(agg.children[0], n):
            b = scan_bytes(n)
            if b > best_bytes:
                best, best_bytes = n, b
    return best


class _PartialStates:
    """Partial aggregate states of a morsel pipeline, bounded in device memory:

    * they accumulate on the device; past budget / 4 bytes they are compacted
      (re-aggregated into one partial state per group: SUM of sums and
      counts, MIN of mins, ...), which bounds them by the group count when
      groups repeat across morsels (TPC-H Q17: parts over lineitem);
    * when compaction cannot shrink them (groups aligned with the stream,
      Q18's orders over lineitem), every later partial is hash-partitioned on
      the group keys into pinned host memory, and the final merge runs one
      partition at a time (a grace aggregation).
    """

    def __init__(self, groups, partial, plan, ids, ctx, morsels_expected: int):
        self.groups, self.partial, self.plan, self.ids, self.ctx = groups, partial, plan, ids, ctx
        self.parts: List[Batch] = []
        self.bytes = 0
        self.limit = ctx.budget // 4
        self.spill = None          # P lists of host batches once partitioned
        self.expected = morsels_expected
        self.seen = 0

    def add(self, pb: Batch) -> None:
        from .joins import _batch_bytes, concat_batches
        self.seen += 1
        if self.spill is not None:
            self._distribute(pb)
            return
        self.parts.append(pb)
        self.bytes += _batch_bytes(pb)
        if self.bytes <= self.limit or not self.groups or len(self.parts) < 2:
            return
        with self.ctx.span("morsel.compact"):
            c = self._compact(concat_batches(self.parts))
        cb = _batch_bytes(c)
        self.ctx.morsels["compactions"] = self.ctx.morsels.get("compactions", 0) + 1
        self.parts, self.bytes = [c], cb
        if cb > self.limit // 2:
            # groups do not repeat enough: partition everything to host memory
            per = cb / max(1, self.seen)
            total = per * max(self.expected, self.seen)
            P = 2
            while total / P > self.ctx.budget / 8 and P < 1024:
                P *= 2
            self.spill = [[] for _ in range(P)]
            parts, self.parts, self.bytes = self.parts, [], 0
            for b in parts:
                self._distribute(b)
        else:
            self.limit = max(self.limit, 2 * cb)

    def _compact(self, rb: Batch) -> Batch:
        """Re-aggregate partial states into one partial row per group (same column ids)."""
        from ..parallel.exchange import _join_wide_finals, _split_wide_partials, _wide_finals
        from ..sql.expr import AggCall
        from .aggregate import aggregate
        fgroups = [(ci, ci.ref()) for ci, _ in self.groups]
        rb, wide = _split_wide_partials(rb, self.plan, self.ids)
        merge = {"sum": "sum", "count": "sum", "min": "min", "max": "max", "bool_and": "bool_and",
                 "bool_or": "bool_or"}
        final = [(pci, AggCall(merge[call.func], pci.ref(), False, pci.dtype)) for pci, call in self.partial]
        final, rec = _wide_finals(final, wide, self.ids)
        return _join_wide_finals(aggregate(fgroups, final, rb, self.ctx), rec)

    def _distribute(self, b: Batch) -> None:
        from ..ops import misc as M
        from ..parallel.exchange import partition_keys
        from ..ops.gather import take_many
        from .joins import _batch_bytes, _to_host
        P = len(self.spill)
        key = None
        for ci, _ in self.groups:
            k = partition_keys(b.columns[ci.cid]).to(torch.int64)
            key = k if key is None else (key * 1000003) ^ k
        perm, counts = M.hash_partition(key.contiguous(), P)
        keys = list(b.columns)
        start = 0
        for p, c in enumerate(counts):
            idx = perm[start:start + c]
            start += c
            if c == 0:
                continue
            piece = Batch(dict(zip(keys, take_many([b.columns[k] for k in keys], idx))), c)
            self.ctx.spill["bytes"] += _batch_bytes(piece)
            self.spill[p].append(_to_host(piece) if self.ctx.device.type == "cuda" else piece)
        self.ctx.spill["aggregate_partitions"] = P

    def partials(self) -> Optional[Batch]:
        """The partial states compacted to one row per group (not finalised:
        an SPMD exchange merges them across ranks)."""
        from .joins import _to_device, _to_host, concat_batches
        if self.spill is None:
            if not self.parts:
                return None
            return self._compact(concat_batches(self.parts)) if self.groups and len(self.parts) > 1 \
                else concat_batches(self.parts)
        dev = self.ctx.device
        outs = []
        for plist in self.spill:
            if plist:
                d = concat_batches([_to_device(b, dev) if dev.type == "cuda" else b for b in plist])
                o = self._compact(d)
                outs.append(_to_host(o) if dev.type == "cuda" else o)
        if not outs:
            return None
        return concat_batches([_to_device(o, dev) if dev.type == "cuda" else o for o in outs])

    def finish(self) -> Optional[Batch]:
        from ..parallel.exchange import merge_partials
        from .joins import _to_device, _to_host, concat_batches
        if self.spill is None:
            if not self.parts:
                return None
            return merge_partials(self.groups, self.plan, concat_batches(self.parts), self.ids, self.ctx)
        dev = self.ctx.device
        outs = []
        for plist in self.spill:
            if not plist:
                continue
            d = concat_batches([_to_device(b, dev) if dev.type == "cuda" else b for b in plist])
            o = merge_partials(self.groups, self.plan, d, self.ids, self.ctx)
            outs.append(_to_host(o) if dev.type == "cuda" else o)
            del d
        if not outs:
            return None
        return concat_batches([_to_device(o, dev) if dev.type == "cuda" else o for o in outs])


def streamed_scan(scan, ctx) -> Optional[Batch]:
    """A filtered scan over the budget, materialised morsel by morsel: each
    morsel is filtered and projected on its own and only the surviving rows
    are kept (concatenated at the end), so the device never holds the
    unfiltered columns. None when the scan fits (or cannot stream)."""
    from .joins import concat_batches
    src = scan.logical.source
    if not getattr(src, "can_stream", False):
        return None
    nbytes = scan_bytes(scan)
    if nbytes <= ctx.budget // STREAM_FRACTION:
        return None
    names, _, _ = scan.column_names()
    row_bytes = max(1, nbytes // max(1, src.num_rows() or 1))
    max_rows = max(MORSEL_MIN_ROWS, ctx.budget // MORSEL_FRACTION // row_bytes)
    stats = ctx.morsels
    stats["pipelines"] += 1
    saved = ctx.morsel
    outs = []
    late, scan.late_ok = scan.late_ok, False
    try:
        with ctx.span("morsel.scan"):
            for k, raw in enumerate(prefetched(src.scan_morsels(names, ctx, scan.pushable(), max_rows), ctx)):
                ctx.morsel = (id(scan), raw, ("morsel", stats["pipelines"], k))
                stats["morsels"] += 1
                stats["rows"] += raw.num_rows
                stats["bytes"] += raw.nbytes
                ctx.rows_scanned += raw.num_rows
                outs.append(scan.finish(scan.scan_raw(ctx), ctx))
                ctx.scan_cache = {k2: v for k2, v in ctx.scan_cache.items() if k2[-1] != ctx.morsel[2]}
    finally:
        ctx.morsel = saved
        scan.late_ok = late
    if not outs:
        return None
    out = concat_batches(outs) if len(outs) > 1 else outs[0]
    return out


def big_streamable(node, ctx) -> bool:
    """``node``'s output derives from a scan too big for the budget that
    could stream (an aggregate over ``node`` would run as a morsel pipeline)."""
    from .scan import ScanExec
    lim = ctx.budget // STREAM_FRACTION
    return any(isinstance(n, ScanExec) and getattr(n.logical.source, "can_stream", False) and scan_bytes(n) > lim
               and stream_path_ok(node, n) for n in _walk(node))


def semi_aggregate(kind, on, residual, null_aware, left_cids, right_plan, right_node, ctx, key):
    """Build side of a SEMI / ANTI join that is too big for the budget,
    replaced by an aggregate of it that streams in morsels:

    * no residual: the build side's distinct keys (GROUP BY the keys);
    * residual ``l.x <> r.y`` (TPC-H Q21's "another supplier of the same
      order"): GROUP BY the keys with MIN(y), MAX(y) — some non-NULL y differs
      from x exactly when MIN(y) <> x or MAX(y) <> x.

    The aggregate holds one row per distinct key instead of the whole build
    side, and is computed once per query (``key``: the join's identity; a
    join inside a morsel pipeline runs once per morsel). Returns (aggregate
    batch, spec for ``apply_semi_aggregate``) or None when the join does not
    have this shape (NOT IN's NULL rules included) or its build side fits."""
    from ..parallel.exchange import _TmpIds
    from ..sql import logical as L
    from ..sql.expr import AggCall, BinOp, ColRef
    from .aggregate import HashAggExec
    if ctx.budget is None or ctx.spmd or kind not in ("semi", "anti") or not on or null_aware:
        return None
    hit = ctx.semi_builds.get(key)
    if hit is not None:
        return hit
    rcids = {c.cid for c in right_plan.schema}
    ineq = None
    if residual is not None:
        r = residual
        if not (isinstance(r, BinOp) and r.op == "<>" and isinstance(r.left, ColRef) and isinstance(r.right, ColRef)):
            return None
        x, y = (r.left, r.right) if r.left.cid in left_cids else (r.right, r.left)
        if x.cid not in left_cids or y.cid not in rcids or x.dtype.is_string or y.dtype.is_string:
            return None
        if x.dtype != y.dtype or x.dtype.is_float:
            # MIN/MAX(y) are compared with x as raw values: decimals of
            # different scales (or int vs decimal) are in different units
            return None
        ineq = (x, y)
    if not big_streamable(right_node, ctx):
        return None
    ids = _TmpIds()
    groups = [(L.ColInfo(ids(), f"__k{i}", rk.dtype, rk.nullable), rk) for i, (_, rk) in enumerate(on)]
    aggs = []
    if ineq is not None:
        y = ineq[1]
        aggs = [(L.ColInfo(ids(), "__mn", y.dtype), AggCall("min", y, False, y.dtype)),
                (L.ColInfo(ids(), "__mx", y.dtype), AggCall("max", y, False, y.dtype))]
    ab = HashAggExec(L.Aggregate(right_plan, groups, aggs), right_node).execute(ctx)
    spec = {"kind": kind, "lkeys": [le for le, _ in on], "kcids": [ci.cid for ci, _ in groups],
            "x": ineq[0] if ineq else None, "mn": aggs[0][0].cid if aggs else None,
            "mx": aggs[1][0].cid if aggs else None}
    ctx.semi_builds[key] = (ab, spec)
    ctx.morsels["semi_aggregates"] = ctx.morsels.get("semi_aggregates", 0) + 1
    return ab, spec


def apply_semi_aggregate(lb: Batch, ab: Batch, spec, ctx) -> Batch:
    """The rows of ``lb`` the SEMI (ANTI: not) join keeps, from the aggregated
    build side of ``semi_aggregate``."""
    from ..ops import hashing as H
    from ..ops.select import mask_to_indices
    from .joins import _take_batch, key_tensors
    ev = ctx.evaluator
    with ctx.span("join.aggregated_semi"):
        if ab.num_rows == 0 or lb.num_rows == 0:
            hit = torch.zeros(lb.num_rows, dtype=torch.bool, device=ctx.device)
        else:
            lk, rk, lvalid, rvalid = key_tensors([ev.column(le, lb) for le in spec["lkeys"]],
                                                 [ab.columns[c] for c in spec["kcids"]])
            lim = ctx.budget // 4 if ctx.budget else None
            table_bytes = 12 * (1 << max(1, (2 * rk.numel() - 1).bit_length()))
            if lim and table_bytes > lim:
                first = _partitioned_probe_first(lk, lvalid, rk, rvalid, table_bytes, lim)
            else:
                first = H.JoinTable(rk, rvalid).probe_first(lk, lvalid)
            hit = first >= 0
            if spec["x"] is not None:
                x = ev.column(spec["x"], lb)
                safe = torch.where(hit, first, torch.zeros_like(first)).long()
                mn, mx = ab.columns[spec["mn"]], ab.columns[spec["mx"]]
                mnv, mxv = mn.data.index_select(0, safe), mx.data.index_select(0, safe)
                xv = x.data.to(mnv.dtype)
                cond = (mnv != xv) | (mxv != xv)
                if mn.valid is not None:
                    cond &= mn.valid.index_select(0, safe)
                if x.valid is not None:
                    cond &= x.valid
                hit &= cond
        keep = mask_to_indices(hit if spec["kind"] == "semi" else ~hit)
    return _take_batch(lb, keep)


def _partitioned_probe_first(lk, lvalid, rk, rvalid, table_bytes: int, lim: int) -> torch.Tensor:
    """``JoinTable(rk).probe_first(lk)`` with the table built one hash
    partition of the keys at a time, each within ``lim`` bytes (a streamed
    semi-join build side with millions of distinct keys, TPC-H Q21 under a
    device budget). Returns int64 build-row indices, -1 where absent."""
    from ..ops import hashing as H
    from ..ops import misc as M
    P = 2
    while table_bytes / P > lim and P < 1024:
        P *= 2
    first = torch.full((lk.numel(),), -1, dtype=torch.int64, device=lk.device)
    rperm, rcounts = M.hash_partition(rk.to(torch.int64).contiguous(), P)
    lperm, lcounts = M.hash_partition(lk.to(torch.int64).contiguous(), P)
    ra = la = 0
    for p in range(P):
        ri, li = rperm[ra:ra + rcounts[p]].long(), lperm[la:la + lcounts[p]].long()
        ra += rcounts[p]
        la += lcounts[p]
        if ri.numel() == 0 or li.numel() == 0:
            continue
        t = H.JoinTable(rk.index_select(0, ri), None if rvalid is None else rvalid.index_select(0, ri))
        f = t.probe_first(lk.index_select(0, li), None if lvalid is None else lvalid.index_select(0, li)).long()
        ok = f >= 0
        first.index_put_((li[ok],), ri.index_select(0, f[ok]))
        del t
    return first


def aggregated_semi_join(join, ctx) -> Optional[Batch]:
    """HashJoinExec SEMI / ANTI through ``semi_aggregate`` (None: not applicable)."""
    j = join.logical
    r = semi_aggregate(j.kind, j.on, j.residual, j.null_aware, {c.cid for c in j.left.schema}, j.right,
                       join.children[1], ctx, ("join", id(join)))
    if r is None:
        return None
    return apply_semi_aggregate(join.children[0].execute(ctx), r[0], r[1], ctx)


def _has_subquery(e) -> bool:
    from ..sql.expr import has_subquery
    return has_subquery(e)


# ------------------------------------------------------------ external sort
#: rows sampled per partition when choosing range splitters
SAMPLE_PER_PART = 64
#: a sort's working memory is taken as this multiple of its input bytes
SORT_MEM_FACTOR = 3


def external_sort(b: Batch, keys, fetch, ctx) -> Optional[Batch]:
    """ORDER BY over an input whose working memory exceeds the budget: range
    partitions on the leading key (sampled splitters), staged in host memory,
    each sorted on the device; None when the input fits (or the leading key
    is not a plain fixed-width column)."""
    from .joins import _batch_bytes, _take_batch, _to_device, _to_host, concat_batches
    from .sorting import sort_batch
    if ctx.budget is None or fetch is not None or b.num_rows < 2:
        return None
    need = SORT_MEM_FACTOR * _batch_bytes(b)
    if need <= ctx.budget:
        return None
    e, asc, nulls_first = keys[0]
    lead = ctx.evaluator.column(e, b)
    if lead.dtype.is_string or lead.is_wide or lead.data.dim() != 1 or lead.dictionary is not None:
        return None
    P = 2
    while need / P > ctx.budget / 2 and P < 4096:
        P *= 2
    n = b.num_rows
    v = lead.data.to(torch.float64) if lead.data.dtype.is_floating_point else lead.data.to(torch.int64)
    valid = lead.valid
    # splitters: quantiles of a strided sample of the non-NULL leading keys
    step = max(1, n // (P * SAMPLE_PER_PART))
    samp = v[::step] if valid is None else v[::step][valid[::step]]
    if samp.numel() == 0:
        return None
    samp, _ = torch.sort(samp)
    q = torch.linspace(0, samp.numel() - 1, P + 1, device=samp.device)[1:-1].round().long()
    split = torch.unique(samp.index_select(0, q))
    # partition id: searchsorted on the splitters; descending order flips it;
    # NULLs form their own partition at the requested end
    pid = torch.searchsorted(split, v, right=True)
    nparts = split.numel() + 1
    if not asc:
        pid = nparts - 1 - pid
    if valid is not None:
        pid = torch.where(valid, pid + (1 if nulls_first else 0),
                          torch.full_like(pid, 0 if nulls_first else nparts))
        nparts += 1
    order = torch.argsort(pid, stable=True)
    counts = torch.bincount(pid, minlength=nparts).tolist()
    dev = ctx.device
    outs, start = [], 0
    ctx.spill["sorts"] = ctx.spill.get("sorts", 0) + 1
    saved, ctx.budget = ctx.budget, None      # each partition sorts in memory
    try:
        with ctx.span("sort.spill_partitions"):
            parts = []
            for c in counts:
                if c == 0:
                    continue
                piece = _take_batch(b, order[start:start + c])
                start += c
                ctx.spill["sort_runs"] = ctx.spill.get("sort_runs", 0) + 1
                ctx.spill["bytes"] += _batch_bytes(piece)
                parts.append(_to_host(piece) if dev.type == "cuda" else piece)
            del order, pid
        with ctx.span("sort.spill_runs"):
            for p in parts:
                d = _to_device(p, dev) if dev.type == "cuda" else p
                s = sort_batch(d, keys, None, ctx)
                outs.append(_to_host(s) if dev.type == "cuda" else s)
    finally:
        ctx.budget = saved
    return concat_batches([_to_device(o, dev) if dev.type == "cuda" else o for o in outs])

