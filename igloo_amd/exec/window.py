"""Window functions and recursive CTEs (DataFusion's
WindowAggExec / BoundedWindowAggExec and RecursiveQueryExec, which the
reference reaches through ``SessionContext::sql``: reference
crates/engine/src/lib.rs:40, :54-57; Cargo.lock datafusion-functions-window).

A window spec (PARTITION BY + ORDER BY) costs one sort: partition keys are
encoded to dense group ids (the GROUP BY machinery), rows are radix-sorted
by (group id, ORDER BY keys), and every function of that spec is then a
segmented scan or an elementwise pass over the sorted order
(ops/window.py -> csrc/kernels/window.hip):

* partition / peer-group starts and ends: max / min scans of head indices;
* row_number / rank / percent_rank / cume_dist / ntile: one elementwise
  kernel over those bounds; dense_rank: a segmented count of peer heads;
* running aggregates (the default RANGE UNBOUNDED PRECEDING .. CURRENT ROW
  frame): one segmented scan, read at each row's last peer;
* whole-partition aggregates: the same scan read at the partition end;
* sliding ROWS / RANGE / GROUPS frames: per-row [lo, hi] bounds (RANGE
  offsets binary-search the sorted key), sums and counts as differences of
  global prefixes, min / max by a frame loop (or a one-sided scan when the
  frame is unbounded on one side);
* lag / lead / first_value / last_value / nth_value: a source-row index
  per row and one gather.

The output keeps the sorted row order (SQL leaves it unspecified); an ORDER
BY above sorts again. Under SPMD the rows are first hash-partitioned by a
PARTITION BY key every call shares (all-to-all), so each rank owns whole
partitions; without one, all rows are gathered (replicated).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch

from .. import types as T
from ..columnar import Batch, Column
from ..ops import window as W
from ..ops import strings as S
from ..ops._lib import to_host_int
from ..ops.gather import gather_tensor, take_many
from ..sql import logical as L
from ..sql.expr import ColRef, WindowCall
from ..utils.errors import ExecutionError, NotSupported
from .context import ExecNode
from .expr_eval import _convert_tensor
from .joins import _take_batch, concat_batches


class WindowExec(ExecNode):
    def __init__(self, logical: L.Window, child: ExecNode):
        self.logical = logical
        self.children = [child]

    def describe(self):
        return ", ".join(f"{w.sql()} AS {c.name}#{c.cid}" for c, w in self.logical.wexprs)

    def _run(self, ctx):
        b = self.children[0].execute(ctx)
        if ctx.spmd and b.dist != ("replicated",):
            b = _distribute(b, self.logical, ctx)
        dist = b.dist
        b = Batch({k: b.columns[k] for k in b.columns}, b.num_rows, dist)
        specs: "OrderedDict[str, list]" = OrderedDict()
        for ci, w in self.logical.wexprs:
            specs.setdefault(w.spec_sql(), []).append((ci, w))
        for calls in specs.values():
            with ctx.span("window.spec"):
                b = _apply_spec(b, calls, ctx)
        b.dist = dist
        return b


def _distribute(b: Batch, lw: L.Window, ctx) -> Batch:
    """SPMD: co-locate each partition on one rank (hash shuffle by a
    PARTITION BY column every call shares), else gather every row."""
    from ..parallel.exchange import gather_all, partition_keys, shuffle
    common = None
    for _, w in lw.wexprs:
        ks = [e.cid for e in w.partition if isinstance(e, ColRef)]
        common = ks if common is None else [k for k in common if k in ks]
    if common:
        cid = common[0]
        if b.dist == ("hash", cid):
            return b
        key = partition_keys(b.columns[cid])
        return shuffle(b, key, ctx, key_cid=cid)
    return gather_all(b, ctx)


class _Sorted:
    """Per-spec sorted state: partition ids and lazily computed bounds."""

    def __init__(self, n, pid, peer, dev):
        self.n, self.pid, self.peer, self.dev = n, pid, peer, dev
        self._c: Dict[str, Optional[torch.Tensor]] = {}

    def _get(self, name, fn):
        if name not in self._c:
            self._c[name] = fn()
        return self._c[name]

    @property
    def ss(self):
        if self.pid is None:
            return None
        return self._get("ss", lambda: W.seg_scan(self.pid, None, W.V_HEADIDX, W.MAX_I, self.n, ids2=self.pid))

    @property
    def se(self):
        if self.pid is None:
            return None
        return self._get("se", lambda: W.seg_scan(self.pid, None, W.V_HEADIDX, W.MIN_I, self.n, ids2=self.pid,
                                                  reverse=True))

    @property
    def ps(self):
        if self.peer is None:
            return self.ss if self.pid is not None else self._zeros()
        return self._get("ps", lambda: W.seg_scan(None, None, W.V_HEADIDX, W.MAX_I, self.n, ids2=self.peer,
                                                  device=self.dev))

    @property
    def pe(self):
        if self.peer is None:
            return self.se if self.pid is not None else self._last()
        return self._get("pe", lambda: W.seg_scan(None, None, W.V_HEADIDX, W.MIN_I, self.n, ids2=self.peer,
                                                  reverse=True, device=self.dev))

    def _zeros(self):
        return self._get("zeros", lambda: torch.zeros(self.n, dtype=torch.int64, device=self.dev))

    def _last(self):
        return self._get("last", lambda: torch.full((self.n,), self.n - 1, dtype=torch.int64, device=self.dev))

    @property
    def dense(self):
        if self.peer is None:
            return self._get("dense", lambda: torch.ones(self.n, dtype=torch.int64, device=self.dev))
        return self._get("dense", lambda: W.seg_scan(self.pid, None, W.V_HEAD2, W.SUM_I, self.n, ids2=self.peer,
                                                     device=self.dev))

    def groups(self):
        """GROUPS frames: global peer-group number per row and first row per group."""
        def build():
            peer = self.peer if self.peer is not None else self.pid
            if peer is None:
                return (torch.zeros(self.n, dtype=torch.int64, device=self.dev),
                        torch.zeros(1, dtype=torch.int64, device=self.dev), 1)
            gnum = W.seg_scan(None, None, W.V_HEAD2, W.SUM_I, self.n, ids2=peer, device=self.dev) - 1
            ng = to_host_int(gnum[-1:]) + 1
            gpos = torch.empty(ng, dtype=torch.int64, device=self.dev)
            heads = torch.ones(self.n, dtype=torch.bool, device=self.dev)
            if self.n > 1:
                heads[1:] = peer[1:] != peer[:-1]
            from ..ops.select import mask_to_indices
            gpos[:] = mask_to_indices(heads, total=ng).to(torch.int64)
            return gnum, gpos, ng
        return self._get("groups", build)


def _sort_value(c: Column) -> torch.Tensor:
    if c.dtype.is_string:
        return S.sort_ranks(c)
    if c.is_wide:
        return _convert_tensor(c, T.FLOAT64)
    if c.data.dtype == torch.bool:
        return c.data.to(torch.int8)
    return c.data


def _apply_spec(b: Batch, calls, ctx) -> Batch:
    from ..ops import sort as SO
    from .aggregate import _encode_groups
    w0: WindowCall = calls[0][1]
    n = b.num_rows
    dev = ctx.device
    ev = ctx.evaluator
    if n == 0:
        out = dict(b.columns)
        for ci, w in calls:
            out[ci.cid] = _empty(w.dtype, dev)
        return Batch(out, 0, b.dist)
    pcols = [ev.column(e, b) for e in w0.partition]
    ocols = [(ev.column(e, b), asc, nf) for e, asc, nf in w0.order]
    gid = None
    if pcols:
        gid, ng, _, _ = _encode_groups(pcols, ctx)
        if ng <= 1:
            gid = None
    keys = []
    if gid is not None:
        keys.append((gid, False, False, None))
    okeys = [(_sort_value(c), not asc, nf, c.valid) for c, asc, nf in ocols]
    keys += okeys
    if keys:
        perm = SO.argsort(keys, n, dev)
        b = _take_batch(b, perm)
        pid = gather_tensor(gid, perm) if gid is not None else None
        taken = take_many([c for c, _, _ in ocols], perm) if ocols else []
        ocols = [(t, asc, nf) for t, (_, asc, nf) in zip(taken, ocols)]
        okeys = [(gather_tensor(v, perm), d, nf,
                  gather_tensor(vv.to(torch.uint8), perm).to(torch.bool) if vv is not None else None)
                 for v, d, nf, vv in okeys]
    else:
        pid = None
    if pid is not None and pid.dtype not in (torch.int32, torch.int64):
        pid = pid.to(torch.int64)
    peer = None
    if okeys:
        # peer groups: rows equal on partition and every ORDER BY key
        h = torch.zeros(n, dtype=torch.bool, device=dev)
        h[0] = True
        if n > 1:
            if pid is not None:
                h[1:] |= pid[1:] != pid[:-1]
            for v, _, _, vv in okeys:
                if vv is None:
                    h[1:] |= v[1:] != v[:-1]
                else:
                    # NULL keys are peers whatever value sits under them
                    h[1:] |= ((v[1:] != v[:-1]) & vv[1:] & vv[:-1]) | (vv[1:] != vv[:-1])
        peer = torch.cumsum(h.to(torch.int64), 0)
    st = _Sorted(n, pid, peer, dev)
    out = dict(b.columns)
    for ci, w in calls:
        with ctx.span(f"window.{w.func}"):
            out[ci.cid] = _compute(w, b, st, ocols, ctx)
    return Batch(out, n, b.dist)


def _empty(t, dev) -> Column:
    if t.is_string:
        return Column(t, torch.zeros(0, dtype=torch.uint8, device=dev), None,
                      offsets=torch.zeros(1, dtype=torch.int64, device=dev))
    return Column(t, torch.zeros(0, dtype=t.torch_dtype if t.kind != "null" else torch.bool, device=dev))


_RANK_FN = {"row_number": W.ROW_NUMBER, "rank": W.RANK, "dense_rank": W.DENSE_RANK, "percent_rank": W.PERCENT_RANK,
            "cume_dist": W.CUME_DIST, "ntile": W.NTILE}


def _compute(w: WindowCall, b: Batch, st: _Sorted, ocols, ctx) -> Column:
    n, dev = st.n, st.dev
    f = w.func
    if f in _RANK_FN:
        fn = _RANK_FN[f]
        arg = w.options[0] if f == "ntile" else 0
        dense = st.dense if f == "dense_rank" else None
        need_peer = f in ("rank", "percent_rank", "cume_dist")
        v = W.rank(fn, arg, n, st.ss, st.se, st.ps if need_peer else None, st.pe if f == "cume_dist" else None,
                   dense, dev)
        return Column(w.dtype, v)
    ev = ctx.evaluator
    if f == "lag":
        x = ev.column(w.args[0], b)
        idx = W.index(W.LAG, w.options[0], n, st.ss, st.se, None, None, dev)
        res = take_many([x], idx, neg=True)[0]
        if len(w.args) > 1:
            res = _fill_default(res, idx < 0, ev.eval(w.args[1], b), w.dtype, n, dev)
        return res
    lo, hi = _frame_bounds(w, st, ocols)
    if f in ("first_value", "last_value", "nth_value"):
        x = ev.column(w.args[0], b)
        fn = {"first_value": W.FIRST, "last_value": W.LAST, "nth_value": W.NTH}[f]
        idx = W.index(fn, w.options[0] if w.options else 0, n, None, None, lo, hi, dev)
        return take_many([x], idx, neg=True)[0]
    return _aggregate(w, b, st, lo, hi, ctx)


def _fill_default(res: Column, oob: torch.Tensor, dflt, t, n, dev) -> Column:
    from .expr_eval import Scalar, _convert_scalar
    if isinstance(dflt, Scalar):
        if dflt.value is None:
            return res
        if t.is_string:
            const = S.const_column(str(dflt.value), dev)
            src = res if res.valid is not None else Column(res.dtype, res.data, None, res.offsets, res.dictionary)
            return S.select_rows([src, const], oob.to(torch.int64), n)
        val = _convert_scalar(dflt.value, dflt.dtype, t)
        data = torch.where(oob, torch.full_like(res.data, val), res.data)
        valid = None if res.valid is None else (res.valid | oob)
        return Column(t, data, valid)
    raise NotSupported("lag/lead with a non-constant default")


def _frame_bounds(w: WindowCall, st: _Sorted, ocols):
    fr = w.frame
    n = st.n
    if fr.unit == "range" and (fr.start in ("preceding", "following") or fr.end in ("preceding", "following")):
        c, asc, _ = ocols[0]
        key = c.data if not c.is_wide else _convert_tensor(c, T.FLOAT64)
        if key.dtype == torch.bool:
            key = key.to(torch.int64)
        soff = fr.start_off.value if hasattr(fr.start_off, "value") else fr.start_off
        eoff = fr.end_off.value if hasattr(fr.end_off, "value") else fr.end_off
        return W.bounds(n, st.ss, st.se, st.ps, st.pe, "range", fr.start, soff, fr.end, eoff, key, c.valid,
                        not asc, device=st.dev)
    if fr.unit == "groups" and (fr.start in ("preceding", "following") or fr.end in ("preceding", "following")):
        gnum, gpos, ng = st.groups()
        return W.bounds(n, st.ss, st.se, st.ps, st.pe, "groups", fr.start, fr.start_off, fr.end, fr.end_off,
                        gnum=gnum, gpos=gpos, ngroups=ng, device=st.dev)
    unit = fr.unit if fr.unit == "rows" else "range"
    return W.bounds(n, st.ss, st.se, st.ps if unit == "range" else None, st.pe if unit == "range" else None, unit,
                    fr.start, fr.start_off, fr.end, fr.end_off, device=st.dev)


def _at(t: torch.Tensor, idx: Optional[torch.Tensor]) -> torch.Tensor:
    return t if idx is None else gather_tensor(t, idx)


def _aggregate(w: WindowCall, b: Batch, st: _Sorted, lo, hi, ctx) -> Column:
    from .aggregate import _avg
    n, dev = st.n, st.dev
    ev = ctx.evaluator
    f = w.func
    fr = w.frame
    col = ev.column(w.args[0], b) if w.args else None
    valid = col.valid if col is not None else None
    if w.filter is not None:
        m = ev.mask(w.filter, b)
        valid = m if valid is None else (valid & m)
    # frame shape: scans serve frames anchored at the partition start or end
    whole = fr.start == "unbounded_preceding" and fr.end == "unbounded_following"
    running = fr.start == "unbounded_preceding" and fr.end == "current"
    if whole:
        read = st.se if st.pid is not None else st._last()
    elif running:
        read = st.pe if fr.unit != "rows" else None
    else:
        read = "frame"
    pid = st.pid
    err = torch.zeros(1, dtype=torch.int32, device=dev) if dev.type == "cuda" else None

    def scan(vals, vkind, op, vv=valid):
        if read == "frame":
            return None
        r = W.seg_scan(pid, vals, vkind, op, n, valid=vv, device=dev, err=err)
        return _at(r, read)

    def prefix(vals, vkind, op, vv=valid):
        return W.seg_scan(None, vals, vkind, op, n, valid=vv, device=dev, err=err)

    def counts():
        if read != "frame":
            return scan(None, W.V_ONE, W.SUM_I)
        return W.frame_sum(None, prefix(None, W.V_ONE, W.SUM_I), lo, hi, n)[1]

    if err is not None:
        ctx.deferred_checks.append((err, f"window {f}() overflowed 64-bit integer arithmetic"))
    if f == "count":
        return Column(T.INT64, counts())
    src = col.dtype
    if src.is_string and f in ("min", "max"):
        return _string_minmax(w, col, valid, st, lo, hi, read, ctx)
    if f in ("sum", "avg") and (col.is_wide or (w.dtype.is_decimal and w.dtype.precision > 18)):
        # exact 128-bit sums: three limb sums (32 + 32 + signed high word)
        # with the int64 scans, recombined with carries
        lo_w, hi_w = (col.data[:, 0], col.data[:, 1]) if col.is_wide else (col.data.to(torch.int64),
                                                                            col.data.to(torch.int64) >> 63)
        mask32 = 0xFFFFFFFF
        limbs = [(lo_w & mask32).contiguous(), ((lo_w >> 32) & mask32).contiguous(), hi_w.contiguous()]
        if read != "frame":
            sums = [scan(x, W.V_I64, W.SUM_I) for x in limbs]
        else:
            sums = [W.frame_sum(prefix(x, W.V_I64, W.SUM_I), None, lo, hi, n)[0] for x in limbs]
        s0, s1, s2 = sums
        a0, a1 = s0 & mask32, s0 >> 32
        mid = a1 + (s1 & mask32)
        lo_r = a0 | ((mid & mask32) << 32)
        hi_r = (mid >> 32) + (s1 >> 32) + s2
        c = counts()
        vv = c > 0
        wide = torch.stack([lo_r, hi_r], 1).contiguous()
        if f == "sum":
            return Column(w.dtype, wide, vv)
        return Column(w.dtype, _avg(wide, c, src, w.dtype), vv)
    if f in ("sum", "avg"):
        fl = src.is_float
        vals = col.data.to(torch.float64) if fl else col.data
        if not fl and vals.dtype not in (torch.int32, torch.int64):
            vals = vals.to(torch.int64)
        vk = W.V_F64 if fl else (W.V_I32 if vals.dtype == torch.int32 else W.V_I64)
        op = W.SUM_F if fl else W.SUM_I
        if read != "frame":
            s = scan(vals, vk, op)
        else:
            s = W.frame_sum(prefix(vals, vk, op), None, lo, hi, n)[0]
        c = counts()
        vv = c > 0
        if f == "sum":
            t = w.dtype
            data = s if t.is_float else s.to(torch.int64)
            return Column(t, data, vv)
        return Column(w.dtype, _avg(s, c, src, w.dtype), vv)
    if f in ("min", "max") and col.is_wide:
        # 128-bit decimals: min / max of their ranks, mapped back to a value
        from ..ops import sort as SO
        hi_k = col.data[:, 1].contiguous()
        lo_k = (col.data[:, 0] ^ (-(2**63))).contiguous()      # unsigned order of the low word
        perm = SO.argsort([(hi_k, False, False, None), (lo_k, False, False, None)], n, dev).to(torch.int64)
        ranks = torch.empty(n, dtype=torch.int64, device=dev)
        ranks.scatter_(0, perm, torch.arange(n, dtype=torch.int64, device=dev))
        is_max = f == "max"
        op = W.MAX_I if is_max else W.MIN_I
        if read != "frame":
            r = scan(ranks, W.V_I64, op)
            vv = counts() > 0
        else:
            r, vv = W.frame_minmax(ranks, valid, lo, hi, n, is_max)
        src_rows = gather_tensor(perm, r.clamp(0, max(n - 1, 0)))
        vals = gather_tensor(col.data, src_rows)
        return Column(w.dtype, vals, vv)
    if f in ("min", "max", "bool_and", "bool_or"):
        is_max = f in ("max", "bool_or")
        fl = src.is_float
        vals = col.data.to(torch.float64) if fl else col.data.to(torch.int64)
        if read != "frame":
            op = (W.MAX_F if is_max else W.MIN_F) if fl else (W.MAX_I if is_max else W.MIN_I)
            r = scan(vals, W.V_F64 if fl else W.V_I64, op)
            vv = counts() > 0
        elif fr.start == "unbounded_preceding" or fr.end == "unbounded_following":
            # one-sided frame: a (reverse) segmented scan read at the open end
            rev = fr.end == "unbounded_following"
            op = (W.MAX_F if is_max else W.MIN_F) if fl else (W.MAX_I if is_max else W.MIN_I)
            full = W.seg_scan(pid, vals, W.V_F64 if fl else W.V_I64, op, n, valid=valid, reverse=rev, device=dev)
            idx = (lo if rev else hi).clamp(0, n - 1)
            r = gather_tensor(full, idx)
            vv = W.frame_sum(None, prefix(None, W.V_ONE, W.SUM_I), lo, hi, n)[1] > 0
        else:
            r, vv = W.frame_minmax(vals, valid, lo, hi, n, is_max)
        t = w.dtype
        if t.kind == "bool":
            return Column(t, r != 0, vv)
        return Column(t, r.to(t.torch_dtype) if not t.is_decimal else r.to(torch.int64), vv)
    if f in ("stddev", "stddev_samp", "stddev_pop", "var", "var_samp", "var_pop"):
        x = _convert_tensor(col, T.FLOAT64).contiguous()
        if read != "frame":
            s1 = scan(x, W.V_F64, W.SUM_F)
            s2 = scan(x * x, W.V_F64, W.SUM_F)
        else:
            s1 = W.frame_sum(prefix(x, W.V_F64, W.SUM_F), None, lo, hi, n)[0]
            s2 = W.frame_sum(prefix(x * x, W.V_F64, W.SUM_F), None, lo, hi, n)[0]
        c = counts().to(torch.float64)
        pop = f.endswith("_pop")
        mean = s1 / c.clamp(min=1)
        var = ((s2 - c * mean * mean) / (c if pop else (c - 1)).clamp(min=1)).clamp(min=0)
        out = var.sqrt() if f.startswith("stddev") else var
        return Column(T.FLOAT64, out, c > (0 if pop else 1))
    raise NotSupported(f"window aggregate {f}")


def _string_minmax(w, col: Column, valid, st: _Sorted, lo, hi, read, ctx) -> Column:  # noqa: C901
    """min / max over strings: on sort ranks, mapped back to a row holding the winner."""
    n, dev = st.n, st.dev
    if not col.is_dict:
        col = S.dict_encode(col)
    ranks = S.sort_ranks(col).to(torch.int64)
    is_max = w.func == "max"
    if read != "frame":
        r = W.seg_scan(st.pid, ranks, W.V_I64, W.MAX_I if is_max else W.MIN_I, n, valid=valid, device=dev)
        r = _at(r, read)
        cnt = W.seg_scan(st.pid, None, W.V_ONE, W.SUM_I, n, valid=valid, device=dev)
        vv = _at(cnt, read) > 0
    else:
        r, vv = W.frame_minmax(ranks, valid, lo, hi, n, is_max)
    # a row per rank value (any non-NULL row holding that rank carries the
    # same string; NULL rows scatter into a spare slot)
    top = len(col.dictionary)     # ranks lie in [0, dictionary size): no readback
    row_of = torch.zeros(top + 1, dtype=torch.int64, device=dev)
    slot = ranks if col.valid is None else torch.where(col.valid, ranks, torch.full_like(ranks, top))
    row_of.scatter_(0, slot, torch.arange(n, dtype=torch.int64, device=dev))
    src = torch.where(vv, gather_tensor(row_of, r.clamp(min=0, max=row_of.numel() - 1)),
                      torch.full((n,), -1, dtype=torch.int64, device=dev))
    return take_many([col], src, neg=True)[0]


# ================================================================ recursive CTE
class WorkTableExec(ExecNode):
    def __init__(self, logical: L.WorkTableScan):
        self.logical = logical
        self.children = []

    def _run(self, ctx):
        tables = getattr(ctx, "worktables", None) or {}
        b = tables.get(self.logical.table_id)
        if b is None:
            raise ExecutionError("recursive CTE work table read outside its iteration")
        cols = {ci.cid: b.columns[k] for ci, k in zip(self.logical.schema, list(b.columns))}
        return Batch(cols, b.num_rows, b.dist)


class RecursiveCTEExec(ExecNode):
    """Iterate the recursive term over the previous iteration's rows until it
    produces none (UNION: rows seen before are dropped each round)."""

    def __init__(self, logical: L.RecursiveCTE, anchor: ExecNode, rec: ExecNode):
        self.logical = logical
        self.children = [anchor, rec]

    def _rename(self, b: Batch, plan: L.Plan) -> Batch:
        cols = {o.cid: b.columns[c.cid] for o, c in zip(self.logical.schema, plan.schema)}
        return Batch(cols, b.num_rows, b.dist)

    def _run(self, ctx):
        lg = self.logical
        if not hasattr(ctx, "worktables"):
            ctx.worktables = {}
        first = self._rename(self.children[0].execute(ctx), lg.anchor)
        if ctx.spmd and first.dist != ("replicated",):
            from ..parallel.exchange import gather_all
            first = gather_all(first, ctx)
        parts = []
        seen = None
        if lg.distinct:
            first, seen = _new_rows(first, None, ctx)
        parts.append(first)
        work = first
        it = 0
        while work.num_rows:
            it += 1
            if it > lg.max_iterations:
                raise ExecutionError(f"recursive CTE exceeded {lg.max_iterations} iterations "
                                     "(SET max_recursion to raise the limit)")
            ctx.worktables[lg.table_id] = work
            # per-iteration caches keyed by plan text would replay the first
            # iteration's results: drop them between iterations
            saved = (ctx.subplans, ctx._subq, ctx.scan_cache)
            ctx.subplans, ctx._subq, ctx.scan_cache = {}, {}, {}
            try:
                nxt = self._rename(self.children[1].execute(ctx), lg.recursive)
            finally:
                ctx.subplans, ctx._subq, ctx.scan_cache = saved
            if ctx.spmd and nxt.dist != ("replicated",):
                from ..parallel.exchange import gather_all
                nxt = gather_all(nxt, ctx)
            if lg.distinct:
                nxt, seen = _new_rows(nxt, seen, ctx)
            if nxt.num_rows:
                parts.append(nxt)
            work = nxt
        ctx.worktables.pop(lg.table_id, None)
        out = concat_batches(parts)
        out.dist = ("replicated",) if ctx.spmd else None
        return out


def _new_rows(b: Batch, seen: Optional[Batch], ctx) -> Tuple[Batch, Batch]:
    """Rows of ``b`` not in ``seen`` and not repeated within ``b`` (NULLs
    equal), and the grown ``seen``."""
    from .aggregate import _encode_groups
    n_seen = seen.num_rows if seen is not None else 0
    allb = concat_batches([seen, b]) if seen is not None else b
    n = allb.num_rows
    if n == 0 or b.num_rows == 0:
        return _take_batch(b, torch.zeros(0, dtype=torch.int64, device=ctx.device)), (seen if seen is not None else b)
    keys = list(allb.columns)
    gid, ng, _, _ = _encode_groups([allb.columns[k] for k in keys], ctx)
    first = torch.full((ng,), n, dtype=torch.int64, device=gid.device)
    first.scatter_reduce_(0, gid.to(torch.int64), torch.arange(n, dtype=torch.int64, device=gid.device), "amin")
    r = torch.arange(n, dtype=torch.int64, device=gid.device)
    keep = (gather_tensor(first, gid) == r) & (r >= n_seen)
    from ..ops.select import mask_to_indices
    idx = mask_to_indices(keep).to(torch.int64) - n_seen
    fresh = _take_batch(b, idx)
    fresh.dist = b.dist
    return fresh, concat_batches([x for x in (seen, fresh) if x is not None])
