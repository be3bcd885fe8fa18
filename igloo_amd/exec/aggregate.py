"""Hash aggregation: partial / final, eager COUNT, fused sorted HAVING.

One of the five operator modules (context, scan, joins, aggregate, sorting)."""
from __future__ import annotations

from ..utils import switches as _sw
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
from ..columnar import LazyColumn, Batch, Column, batch_device
from ..ops import agg as A
from ..ops import hashing as H
from ..ops import misc as M
from ..ops import strings as S
from ..ops._lib import (capturing, check_not_capturing, device_ints, launch, ptr, stream, to_host_f64s, to_host_int,
                       to_host_ints, unlogged)
from ..utils import trace as _trace
from ..ops.gather import gather_tensor, take, take_many
from ..ops.select import count_true, exclusive_scan, mask_to_indices
from ..sql import logical as L
from ..sql.expr import AggCall, BinOp, ColRef, Expr, Lit, and_all, col_refs, conjuncts
from ..utils.errors import ExecutionError, NotSupported
from . import fused
from .expr_eval import Evaluator, Scalar, _convert_tensor
from .context import ExecContext, ExecNode
from .scan import LazyBatch, ScanExec, predicate_mask
from .joins import (HashJoinExec, LateBatch, _index_key_filter, _index_then_filter, _take_batch, apply_key_filters,
                    group_key_tensor, hash_join, key_tensors, _num_key, _resident_ndv)


# ======================================================================= aggregate
#: eager COUNT under LEFT JOIN: right-key spans up to this count with one histogram
EAGER_COUNT_DIRECT_SPAN = 1 << 27
#: HashAggExec._eager_count_masked
EAGER_COUNT_MASKED = True
#: HashAggExec._sorted_having: fused sorted GROUP BY + HAVING
SORTED_HAVING = True
SORTED_HAVING_MIN_ROWS = 1 << 16
#: the streaming sorted-HAVING kernel (csrc/kernels/agg.hip sorted_having_scan_kernel; IGLOO_DEBUG=having_general
#: takes the run-folding kernel, on the C++ side too)
HAVING_SCAN = not _sw.debug("having_general")
#: HashAggExec: a runtime key filter over a filtered resident scan takes the key index first
INDEX_THEN_FILTER = True

def having_constant(op: str, lit: Lit, src: T.DataType, func: str, float_state: bool):
    """The HAVING literal in the units of the aggregate's raw state (fused
    sorted GROUP BY + HAVING): a float for f64 states; else an int, where a
    fractional threshold is rounded so that the integer comparison keeps its
    meaning (x > 2.5 <=> x > 2, x >= 2.5 <=> x >= 3, x < 2.5 <=> x < 3,
    x <= 2.5 <=> x <= 2). None for = / <> against a fractional value."""
    lv = Fraction(lit.value, 10 ** lit.dtype.scale) if lit.dtype.is_decimal else Fraction(lit.value)
    if float_state:
        return float(lv)
    thr = lv * 10 ** (src.scale if (src.is_decimal and func != "count") else 0)
    if thr.denominator != 1:
        if op in ("=", "<>"):
            return None
        thr = math.floor(thr) if op in (">", "<=") else math.ceil(thr)
    return int(thr)


class HashAggExec(ExecNode):
    def __init__(self, logical: L.Aggregate, child: ExecNode):
        self.logical = logical
        self.children = [child]
        self.runtime_filters: list = []  # (group expr, key column) set by a parent join
        self.having = None               # predicate of a parent FilterExec (HAVING)

    def _sorted_having(self, ctx) -> Optional[Batch]:
        """GROUP BY a sorted key column HAVING <aggregate> <cmp> <constant> as
        one fused pass (ops/agg.py sorted_having): only the passing groups are
        materialised (TPC-H Q18: 6.5K of 150M l_orderkey groups at SF100). The
        parent FilterExec still applies the predicate to them (NULL groups).
        None when the shape does not apply (the general path runs)."""
        lg, pred = self.logical, self.having
        if (pred is None or ctx.device.type != "cuda" or ctx.budget is not None or self.runtime_filters
                or not SORTED_HAVING or len(lg.groups) != 1 or not 1 <= len(lg.aggs) <= 4
                or not isinstance(lg.groups[0][1], ColRef) or not isinstance(pred, BinOp)):
            return None
        if any(a.func not in ("sum", "count", "min", "max") or a.distinct or a.filter is not None for _, a in lg.aggs):
            return None
        flip = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "<>": "<>"}
        if pred.op not in flip:
            return None
        agg_cids = {ci.cid: i for i, (ci, _) in enumerate(lg.aggs)}
        if isinstance(pred.left, ColRef) and pred.left.cid in agg_cids and isinstance(pred.right, Lit):
            ref, lit, op = pred.left, pred.right, pred.op
        elif isinstance(pred.right, ColRef) and pred.right.cid in agg_cids and isinstance(pred.left, Lit):
            ref, lit, op = pred.right, pred.left, flip[pred.op]
        else:
            return None
        if lit.value is None or not (lit.dtype.is_integer or lit.dtype.is_decimal or lit.dtype.is_float):
            return None
        if any(a.func in ("min", "max") and a.arg is not None and a.arg.dtype.is_string for _, a in lg.aggs):
            return None
        # an unfiltered scan whose group key column is sorted (decided before
        # running anything, so every other aggregate path stays available)
        child = self.children[0]
        if not isinstance(child, ScanExec) or child.predicate is not None:
            return None
        gci, gexpr = lg.groups[0]
        if ctx.spmd and not self._group_local(child, gexpr, ctx):
            return None
        raw = child.peek_raw(ctx)
        if ctx.spmd:
            from ..parallel.exchange import REPLICATED, placed_on
            if raw.dist != REPLICATED and not placed_on(raw.dist, gexpr.cid):
                return None      # (alike on every rank: placements follow from plan and catalog)
        kc = raw.columns.get(gexpr.cid) if hasattr(raw, "columns") else None
        if kc is None or kc.valid is not None or kc.data.dtype not in (torch.int32, torch.int64) \
                or kc.data.dim() != 1 or kc.dtype.is_string or raw.num_rows < SORTED_HAVING_MIN_ROWS \
                or not H.is_sorted(kc.data):
            return None
        b = child.finish(raw, ctx)
        n = b.num_rows
        kcol = ctx.evaluator.column(gexpr, b)
        if kcol.data.data_ptr() != kc.data.data_ptr() or n != raw.num_rows:
            return self._finish_general(b, ctx)
        specs, finals, vidx = [], [], {}
        for i, (ci, a) in enumerate(lg.aggs):
            _plan_agg(ci, a, b, None, 1, n, ctx, specs, finals)
            vidx[i] = len(specs) - 1          # the aggregate's value spec (sum/min/max/count)
        if len(specs) > 4:
            return self._finish_general(b, ctx)
        hidx = vidx[agg_cids[ref.cid]]
        hop_spec = specs[hidx][0]
        a = lg.aggs[agg_cids[ref.cid]][1]
        src = a.arg.dtype if a.arg is not None else T.INT64
        const = having_constant(op, lit, src, a.func, hop_spec in ("sum_f64", "min_f64", "max_f64"))
        if const is None:
            return self._finish_general(b, ctx)
        specs = [sp[:3] for sp in specs]
        if HAVING_SCAN and all(sp[2] is None and sp[0] in ("count", "sum_int") for sp in specs) \
                and sum(sp[0] == "sum_int" for sp in specs) <= 1:
            # the streaming kernel reads the summed column at its narrow width
            # (Q18's l_quantity as int16: 1.2 GB instead of 4.8 GB at SF100)
            from .fused import narrow
            specs = [(o, narrow(v) if o == "sum_int" else v, vv) for o, v, vv in specs]
        with ctx.span("agg.sorted_having"):
            got = A.sorted_having(kcol.data, specs, hidx, op, const)
        if got is None:
            return self._finish_general(b, ctx)
        rep, results = got
        out = {gci.cid: take(kcol, rep)}
        for fin in finals:
            ci, col = fin(results)
            out[ci.cid] = col
        return Batch(out, rep.numel(), self._local_dist(raw.dist, gci) if ctx.spmd else None)

    @staticmethod
    def _group_local(scan: "ScanExec", gexpr, ctx) -> bool:
        """SPMD: every group of GROUP BY ``gexpr`` over ``scan`` lives on one
        rank (the scan's table is placed by that column -- hash-partitioned,
        or a replicated table this query splits by ranges of it -- or is
        replicated whole), so an aggregate over the rank's rows is final.
        Decided from the plan and catalog, alike on every rank."""
        src = scan.logical.source
        names = {c.cid: c.name for c in getattr(scan.logical, "table_cols", scan.logical.schema)}
        names.update({c.cid: c.name for c in scan.logical.schema})
        col = names.get(gexpr.cid) if isinstance(gexpr, ColRef) else None
        if getattr(src, "replicated", False):
            sk = ctx.slices.get(id(src))
            return sk is None or (col is not None and col == sk)
        pk = getattr(src, "partitioned_by", None)
        return pk is not None and col == pk

    @staticmethod
    def _local_dist(d, gci):
        from ..parallel.exchange import REPLICATED, keyed
        if d == REPLICATED:
            return REPLICATED
        return (d[0], gci.cid) if keyed(d) else None

    def _finish_general(self, b, ctx) -> Batch:
        lg = self.logical
        out = aggregate(lg.groups, lg.aggs, b, ctx)
        if ctx.spmd:
            out.dist = self._local_dist(b.dist, lg.groups[0][0])
        return out

    def describe(self):
        a = self.logical
        return (f"gby=[{', '.join(e.sql() for _, e in a.groups)}], "
                f"aggr=[{', '.join(x.sql() for _, x in a.aggs)}]")

    def _eager_count(self, ctx) -> Optional[Batch]:
        """GROUP BY <left join key>, COUNT(<right column>)... over a LEFT JOIN on
        that key (TPC-H Q13: customer LEFT JOIN orders, count per customer):
        count the right side per key first, then look the counts up per left row
        and sum them per group — a group-by over the right input plus a probe of
        the left keys, instead of materialising and re-grouping the join
        (150M-row join output at SF100). Exact: a left row with k partners
        contributes k to COUNT(x) exactly when x is non-NULL on each partner."""
        lg, child = self.logical, self.children[0]
        if not isinstance(child, HashJoinExec) or len(lg.groups) != 1 or not lg.aggs:
            return None
        j = child.logical
        if j.kind != "left" or j.residual is not None or len(j.on) != 1:
            return None
        lkey, rkey = j.on[0]
        gci, gexpr = lg.groups[0]
        if not (isinstance(gexpr, ColRef) and isinstance(lkey, ColRef) and gexpr.cid == lkey.cid):
            return None
        right_cids = {c.cid for c in j.right.schema}
        for _, a in lg.aggs:
            if not (a.func == "count" and not a.distinct and a.filter is None and isinstance(a.arg, ColRef)
                    and a.arg.cid in right_cids):
                return None
        ev = ctx.evaluator
        if ctx.budget is not None and not ctx.spmd:
            from .morsel import big_streamable
            if big_streamable(child.children[1], ctx):
                return self._eager_count_streamed(lkey, rkey, ctx)
        if ctx.device.type != "cuda" and not ctx.spmd:
            return None     # (the CPU engine stays the plain join + aggregate: the GPU tests' reference)
        lb = child.children[0].execute(ctx)
        masked = self._eager_count_masked(lg, lb, lkey, rkey, ctx)
        if masked is not None:
            return masked
        rb = child.children[1].execute(ctx)
        with ctx.span("agg.eager_count"):
            lk, rk, lvalid, rvalid = key_tensors([ev.column(lkey, lb)], [ev.column(rkey, rb)])
            if rvalid is not None:  # NULL keys never match
                keep = mask_to_indices(rvalid)
                rk = gather_tensor(rk, keep)
                rb = _take_batch(rb, keep)
            cnt_cols = {}
            if ctx.spmd:
                out = self._spmd_counts(lg, lb, lkey, lk, lvalid, rk,
                                        [ev.column(a.arg, rb).valid for _, a in lg.aggs], ctx)
                return out if out is not None else self._spmd_join_aggregate(lb, rb, ctx)
            rng = H.key_range(rk) if rk.numel() else None
            span = rng[1] - rng[0] + 1 if rng else 0
            if rng and span <= EAGER_COUNT_DIRECT_SPAN:
                # dense key domain: one histogram pass over the right keys, then a
                # direct lookup per left key (no hash table, no group ids)
                kmin = rng[0]
                li = lk.to(torch.int64) - kmin
                inr = (li >= 0) & (li < span)
                if lvalid is not None:
                    inr &= lvalid
                li = torch.where(inr, li, torch.zeros_like(li))
                for k, (_, a) in enumerate(lg.aggs):
                    hist = A.key_histogram(rk, kmin, span, ev.column(a.arg, rb).valid) if rk.numel() else \
                        torch.zeros(span, dtype=torch.int64, device=ctx.device)
                    cnt_cols[-(k + 1)] = torch.where(inr, hist.index_select(0, li), torch.zeros_like(li))
            elif rk.numel():
                gid, ng, rep, srt = H.group_ids_ex(rk)
                specs = [("count", None, ev.column(a.arg, rb).valid) for _, a in lg.aggs]
                counts = A.grouped_aggregate(gid, ng, specs, rk.numel(), ctx.device, sorted_gids=srt)
                first = H.JoinTable(gather_tensor(rk, rep)).probe_first(lk, lvalid)
                hit = first >= 0
                safe = torch.where(hit, first, torch.zeros_like(first)).long()
                for k, c in enumerate(counts):
                    cnt_cols[-(k + 1)] = torch.where(hit, c.index_select(0, safe), torch.zeros_like(safe))
            else:
                for k in range(len(lg.aggs)):
                    cnt_cols[-(k + 1)] = torch.zeros(lb.num_rows, dtype=torch.int64, device=ctx.device)
        return self._count_sums(lg, lb, [cnt_cols[-(k + 1)] for k in range(len(lg.aggs))], ctx)

    def _count_sums(self, lg, lb: Batch, counts, ctx, dist=None) -> Batch:
        """GROUP BY <left key> SUM(per-row partner count) -- the eager COUNT's
        final step over the left rows and their looked-up counts."""
        cols = dict(lb.columns)
        aggs = []
        for k, (ci, _) in enumerate(lg.aggs):
            tmp = -(10**9) - k  # temporary column ids (binder ids are positive)
            cols[tmp] = Column(T.INT64, counts[k].to(torch.int64).contiguous())
            aggs.append((ci, AggCall("sum", ColRef(tmp, "__cnt", T.INT64, False), False, T.INT64)))
        if ctx.spmd:
            from ..parallel.exchange import distributed_aggregate
            return distributed_aggregate(L.Aggregate(None, lg.groups, aggs),
                                         Batch(cols, lb.num_rows, dist if dist is not None else lb.dist), ctx)
        return aggregate(lg.groups, aggs, Batch(cols, lb.num_rows), ctx)

    def _spmd_counts(self, lg, lb: Batch, lkey, lk, lvalid, rk, rmasks, ctx, rcol: Optional[Column] = None
                     ) -> Optional[Batch]:
        """SPMD eager COUNT: each rank histograms its right rows' keys over the
        GLOBAL key range (one tiny all-gather of the ranges), then

        * replicated left side (TPC-H Q13: customer against orders placed by
          order key): ONE reduce-scatter sums the histograms and leaves rank r
          the counts of key chunk r only (1/world of the bytes of an
          all-reduce, which would hand every rank all 15M counts at SF100);
          each rank keeps the left rows of its chunk, so the result is
          partitioned by key range and the GROUP BY that follows is rank-local;
        * partitioned left side: an all-reduce (every rank's left keys may
          fall anywhere in the range).

        Counts travel as int32 (half the bytes) when the global right row
        count fits. None when the global key span is too large for dense
        histograms (decided alike on every rank)."""
        from ..parallel.exchange import REPLICATED
        from ..parallel.slicing import range_chunk, range_tag
        comm = ctx.comm
        W = comm.world_size
        dev = ctx.device
        masks = list(rmasks)
        rng = H.key_range(rk, masks[0] if len(set(map(id, masks))) == 1 else None) if rk.numel() else None
        g = comm.allgather_ints([rng[0], rng[1], rk.numel()] if rng else [2**62, -2**62, rk.numel()])
        g0, g1 = min(r[0] for r in g), max(r[1] for r in g)
        if g0 > g1:
            return self._count_sums(lg, lb, [torch.zeros(lb.num_rows, dtype=torch.int64, device=dev)] * len(masks), ctx)
        span = g1 - g0 + 1
        if span > EAGER_COUNT_DIRECT_SPAN:
            return None
        wide = sum(r[2] for r in g) >= 2**31
        rep = lb.dist == REPLICATED
        chunk = range_chunk(g0, g1, W) if rep else span
        width = W * chunk if rep else span
        hdt = torch.int64 if wide else torch.int32
        hists = torch.zeros((len(masks), width), dtype=hdt, device=dev)
        full = _full_key_hist(rcol, g0, span) if rcol is not None and rk.numel() else None
        for k, m in enumerate(masks):
            if rk.numel():
                if full is not None and m is not None and 2 * count_true(m) > m.numel():
                    # most of this rank's rows pass (Q13): subtract the few
                    # that fail from the resident column's remembered per-key
                    # counts (as on one rank; a local choice, no collective)
                    hists[k, :span] = (full - A.key_histogram(rk, g0, span, ~m, sparse=True)).to(hdt)
                else:
                    hists[k, :span] = A.key_histogram(rk, g0, span, m).to(hdt)
        lkey64 = lk.to(torch.int64)
        if rep:
            # [world, aggs, chunk]: rank r's share is one contiguous block
            mine = comm.reduce_scatter_tensor(hists.view(len(masks), W, chunk).transpose(0, 1).contiguous(), "sum")
            mine = mine.view(len(masks), chunk)
            # the left rows of this rank's key chunk (keys outside the right
            # side's range clamp to the first / last chunk; NULL keys: rank 0)
            owner = torch.clamp(torch.div(lkey64 - g0, chunk, rounding_mode="floor"), 0, W - 1)
            own = owner == comm.rank
            if lvalid is not None:
                own = torch.where(lvalid, own, torch.full_like(own, comm.rank == 0))
            if W > 1:
                sel = mask_to_indices(own)
                lb = _take_batch(lb, sel)
                lkey64 = gather_tensor(lkey64, sel)
                lvalid = gather_tensor(lvalid, sel) if lvalid is not None else None
            base, size, table = g0 + comm.rank * chunk, chunk, mine
            dist = (range_tag(W, g0, chunk), lkey.cid) if isinstance(lkey, ColRef) else None
        else:
            table = comm.allreduce_tensor(hists, "sum")
            base, size, dist = g0, span, None
        li = lkey64 - base
        inr = (li >= 0) & (li < size)
        if lvalid is not None:
            inr &= lvalid
        li = torch.where(inr, li, torch.zeros_like(li))
        counts = [torch.where(inr, table[k].index_select(0, li).to(torch.int64), torch.zeros_like(li))
                  for k in range(len(masks))]
        return self._count_sums(lg, lb, counts, ctx, dist)

    def _eager_count_masked(self, lg, lb, lkey, rkey, ctx) -> Optional[Batch]:
        """``_eager_count`` over a filtered right-side scan without
        compacting it: the per-key histogram reads the resident key column
        with the filter mask as its validity (Q13: 148M of 150M orders pass
        o_comment NOT LIKE, so the compaction and the o_custkey gather were
        pure copies). Dense key domains, single rank, no budget; None when
        the shape differs."""
        rnode = self.children[0].children[1]
        if ctx.budget is not None or not isinstance(rnode, ScanExec) or rnode.predicate is None \
                or not EAGER_COUNT_MASKED or not isinstance(rkey, ColRef) \
                or any(not isinstance(a.arg, ColRef) for _, a in lg.aggs):
            return None
        ev = ctx.evaluator
        raw = rnode.peek_raw(ctx)
        for _, a in lg.aggs:
            # COUNT(x) counts the same rows as the key histogram when x holds
            # no NULLs: a NOT NULL column, or one declared nullable that has no
            # validity (Parquet fields are nullable by default)
            c = raw.columns.get(a.arg.cid)
            if getattr(a.arg, "nullable", True) and (c is None or c.valid is not None):
                return None
        rcol = raw.columns.get(rkey.cid)
        lcol = ev.column(lkey, lb)
        if rcol is None or rcol.dtype.is_string or lcol.dtype.is_string or rcol.is_dict \
                or rcol.data.dtype not in (torch.int32, torch.int64) or lcol.data.dtype not in (torch.int32, torch.int64):
            return None
        if ctx.spmd:
            # (the global key span decides, alike on every rank)
            with ctx.span("agg.eager_count"):
                m = predicate_mask(rnode.predicate, raw, ctx)
                if rcol.valid is not None:
                    m = m & rcol.valid
                return self._spmd_counts(lg, lb, lkey, lcol.data, lcol.valid, rcol.data, [m] * len(lg.aggs), ctx,
                                         rcol=rcol)
        rng = H.key_range(rcol.data, rcol.valid)
        span = rng[1] - rng[0] + 1 if rng else 0
        if not rng or span > EAGER_COUNT_DIRECT_SPAN:
            return None
        with ctx.span("agg.eager_count"):
            m = predicate_mask(rnode.predicate, raw, ctx)
            if rcol.valid is not None:
                m = m & rcol.valid
            kmin = rng[0]
            li = lcol.data.to(torch.int64) - kmin
            inr = (li >= 0) & (li < span)
            if lcol.valid is not None:
                inr &= lcol.valid
            li = torch.where(inr, li, torch.zeros_like(li))
            full = _full_key_hist(rcol, kmin, span)
            if full is not None and 2 * count_true(m) > m.numel():
                # most rows pass (Q13: 148M of 150M orders): count the few
                # that fail and subtract them from the column's remembered
                # per-key counts instead of histogramming the many
                hist = full - A.key_histogram(rcol.data, kmin, span, ~m, sparse=True)
            else:
                hist = A.key_histogram(rcol.data, kmin, span, m)
            cnt = torch.where(inr, hist.index_select(0, li), torch.zeros_like(li))
        cols = dict(lb.columns)
        aggs = []
        for k, (ci, _) in enumerate(lg.aggs):
            tmp = -(10**9) - k  # temporary column ids (binder ids are positive)
            cols[tmp] = Column(T.INT64, cnt.contiguous())
            aggs.append((ci, AggCall("sum", ColRef(tmp, "__cnt", T.INT64, False), False, T.INT64)))
        return aggregate(lg.groups, aggs, Batch(cols, lb.num_rows), ctx)

    def _eager_count_streamed(self, lkey, rkey, ctx) -> Batch:
        """``_eager_count`` with a right side over the device budget: the
        per-key counts come from an aggregate of the right side (GROUP BY the
        join key, one COUNT per aggregate), which streams in morsels
        (exec/morsel.py), instead of the materialised right side."""
        from ..parallel.exchange import _TmpIds
        lg, child = self.logical, self.children[0]
        j = child.logical
        ids = _TmpIds()
        kci = L.ColInfo(ids(), "__k", rkey.dtype, rkey.nullable)
        cnt = [(L.ColInfo(ids(), "__c", T.INT64, False), AggCall("count", a.arg, False, T.INT64)) for _, a in lg.aggs]
        ab = HashAggExec(L.Aggregate(j.right, [(kci, rkey)], cnt), child.children[1]).execute(ctx)
        lb = child.children[0].execute(ctx)
        ev = ctx.evaluator
        with ctx.span("agg.eager_count"):
            lk, rk, lvalid, rvalid = key_tensors([ev.column(lkey, lb)], [ab.columns[kci.cid]])
            cols = dict(lb.columns)
            aggs = []
            if ab.num_rows and lb.num_rows:
                first = H.JoinTable(rk, rvalid).probe_first(lk, lvalid)
                hit = first >= 0
                safe = torch.where(hit, first, torch.zeros_like(first)).long()
            for k, (ci, _) in enumerate(lg.aggs):
                if ab.num_rows and lb.num_rows:
                    c = ab.columns[cnt[k][0].cid].data
                    v = torch.where(hit, c.index_select(0, safe), torch.zeros_like(safe))
                else:
                    v = torch.zeros(lb.num_rows, dtype=torch.int64, device=ctx.device)
                tmp = -(10**9) - k
                cols[tmp] = Column(T.INT64, v.contiguous())
                aggs.append((ci, AggCall("sum", ColRef(tmp, "__cnt", T.INT64, False), False, T.INT64)))
        return aggregate(lg.groups, aggs, Batch(cols, lb.num_rows), ctx)

    def _spmd_join_aggregate(self, lb: Batch, rb: Batch, ctx) -> Batch:
        """SPMD fallback after the inputs were computed: the plain exchange +
        join + distributed aggregation."""
        from ..parallel.exchange import distributed_aggregate, prepare_join
        j = self.children[0].logical
        lb, rb = prepare_join(lb, rb, j, ctx)
        out = hash_join(lb, rb, j.kind, j.on, j.residual, ctx, null_aware=j.null_aware)
        out.dist = lb.out_dist
        return distributed_aggregate(self.logical, out, ctx)

    def _run(self, ctx):
        lg = self.logical
        child = self.children[0]
        if self.having is not None and ctx.budget is None and ctx.device.type == "cuda" \
                and not self.runtime_filters:
            out = self._sorted_having(ctx)
            if out is not None:
                return out
        # the same aggregate subtree twice in one query (TPC-H Q15's revenue
        # view, read by the outer query and by its max() subquery) runs once
        key = _subtree_key(lg) if not self.runtime_filters and ctx.morsel is None and ctx.memo is None \
            and ctx.budget is None else None
        if key is not None:
            hit = ctx.subplans.get(key)
            if hit is not None:
                return _rekeyed(hit, lg)
        out = self._run_agg(ctx, child)
        if key is not None:
            ctx.subplans[key] = (out, [c.cid for c in lg.schema])
        return out

    def _run_agg(self, ctx, child):
        lg = self.logical
        if ctx.budget is not None:
            from .morsel import streamed_aggregate
            out = streamed_aggregate(self, ctx)
            if out is not None:
                return out
        if (ctx.device.type == "cuda" or ctx.budget is not None or ctx.spmd) and not self.runtime_filters:
            out = self._eager_count(ctx)
            if out is not None:
                return out
        local = None
        if isinstance(child, ScanExec) and ctx.device.type == "cuda" and not self.runtime_filters:
            # scan -> filter -> aggregate in one fused kernel when the shape allows
            raw = child.scan_raw(ctx)
            pred = child.predicate

            def local(groups, aggs, plan=None, raw=raw, pred=pred):
                return fused.fused_scan_aggregate(groups, aggs, raw, pred, ctx)
            if not ctx.spmd:
                out = local(lg.groups, lg.aggs)
                if out is not None:
                    return out
            b = LazyBatch(lambda: child.finish(raw, ctx), raw.dist)
        elif self.runtime_filters and isinstance(child, ScanExec) and child.predicate is not None \
                and ctx.device.type == "cuda" and ctx.budget is None and INDEX_THEN_FILTER:
            # decided before the scan filter runs over the whole table
            raw = child.scan_raw(ctx)
            filters, self.runtime_filters = self.runtime_filters, []
            pre = _index_then_filter(child, raw, filters, ctx)
            if pre is not None:
                b, filters = pre
            else:
                b = child.finish(raw, ctx)
            self.runtime_filters = filters
        else:
            b = child.execute(ctx)
        if self.runtime_filters:
            filters, self.runtime_filters = self.runtime_filters, []
            b = apply_key_filters(b, filters, ctx)
        if ctx.spmd:
            from ..parallel.exchange import distributed_aggregate
            return distributed_aggregate(lg, b, ctx, local=local)
        return aggregate(lg.groups, lg.aggs, b, ctx)


_CIDNUM = re.compile(r"#(\d+)")


def _subtree_key(plan) -> Optional[str]:
    """Text of a logical subtree with its column ids renumbered in order of
    appearance: two subtrees with equal keys compute the same rows (same
    tables, filters, expressions). None for subtrees holding a subquery
    (its plan is not part of the text)."""
    txt = plan.explain()
    if "subquery" in txt or "WorkTable" in txt:
        return None
    seen: Dict[str, int] = {}

    def ren(m):
        return "#" + str(seen.setdefault(m.group(1), len(seen)))
    return _CIDNUM.sub(ren, txt)


def _rekeyed(hit, lg) -> Batch:
    """A cached aggregate result under this subtree's output column ids."""
    out, cids = hit
    mine = [c.cid for c in lg.schema]
    m = dict(zip(cids, mine))
    d = out.dist
    if isinstance(d, tuple) and len(d) > 1:          # key placements name output columns
        d = (d[0],) + tuple(m.get(c, c) for c in d[1:])
    return Batch({m[c]: out.columns[c] for c in cids}, out.num_rows, d)


def aggregate(groups, aggs, b: Batch, ctx, row_parts: Optional[Dict[int, int]] = None, fd: bool = False,
              skip: Optional[set] = None) -> Batch:
    """GROUP BY ``groups`` computing ``aggs`` over ``b``. ``row_parts``
    ({output cid: part index} of a LateBatch ``b``): when the grouping runs
    on the join result's index form (``_late_group_keys``: every other key is
    functionally dependent on the leading integer key), each group's row in
    those parts is added as an int64 column -- the SPMD exchange ships that
    row instead of the part's string columns (parallel/exchange.py). The
    columns are absent when the dependency did not hold; group keys in
    ``skip`` (output cids the caller replaces by those rows) are then not
    materialised at all. ``fd``: the keys are
    expected to depend on one integer key (the exchange's merge of such
    partial groups): ``_encode_groups`` tries that shortcut even without
    plain string keys."""
    ev = ctx.evaluator
    n = b.num_rows
    dev = ctx.device
    late = None
    if groups and n and isinstance(b, LateBatch) and (dev.type == "cuda" or row_parts):
        with ctx.span("agg.late_keys"):
            late = _late_group_keys(groups, b, ctx, skip if row_parts else None)
    if late is not None:
        gid, ng, rep, taken = late
    else:
        with ctx.span("agg.eval_keys"):
            gcols = [ev.column(e, b) for _, e in groups]
        if groups:
            if n == 0:
                return Batch({ci.cid: _empty_col(ci.dtype, dev) for ci, _ in list(groups) + list(aggs)}, 0)
            with ctx.span("agg.group_ids"):
                ctx.sorted_gids = False
                gid, ng, rep, reps_src = _encode_groups(gcols, ctx, fd)
        else:
            gid, ng, rep = None, 1, None
        if groups:
            with ctx.span("agg.take_keys"):
                taken = take_many(reps_src, rep)
    out: Dict[int, Column] = {}
    if groups:
        for (ci, _), c in zip(groups, taken):
            if c is not None:
                out[ci.cid] = c
        if len(groups) == 1 and taken[0] is not None and not getattr(taken[0], "pending", False) \
                and taken[0].valid is None and not taken[0].is_plain_string:
            # one row per group: a single key's values are distinct (a join
            # building on them skips its duplicate check, ops/hashing.py key_unique)
            try:
                taken[0].data._igloo_distinct = True
            except (AttributeError, RuntimeError):
                pass
    if late is not None and row_parts:
        for cid, k in row_parts.items():
            idx = b.parts[k][1]
            out[cid] = Column(T.INT64, gather_tensor(idx, rep).to(torch.int64))
    specs, finals = [], []
    with ctx.span("agg.eval_args"):
        ev.prefetch([a.arg for _, a in aggs] + [getattr(a, "arg2", None) for _, a in aggs], b)
        for ci, a in aggs:
            _plan_agg(ci, a, b, gid, ng, n, ctx, specs, finals)
    with ctx.span("agg.kernel"):
        results = A.grouped_aggregate(gid, ng, [s[:3] for s in specs], n, dev,
                                      sorted_gids=gid is not None and getattr(ctx, "sorted_gids", False)) \
            if specs else []
        for fin in finals:
            ci, col = fin(results)
            out[ci.cid] = col
    return Batch(out, ng)


def _full_key_hist(rcol: Column, kmin: int, span: int) -> Optional[torch.Tensor]:
    """Rows per key of a resident NULL-free key column over [kmin, kmin +
    span), computed once and remembered on the column (None otherwise)."""
    t = rcol.data
    if rcol.valid is not None or not getattr(t, "_igloo_resident", False) or not t.is_cuda:
        return None
    hit = getattr(t, "_igloo_key_hist", None)
    if hit is not None and hit[0] == kmin and hit[1] == span:
        return hit[2]
    if capturing():
        return None
    with unlogged():     # a one-time build on a resident column (ops/_lib.py unlogged)
        h = A.key_histogram(t, kmin, span)
    try:
        t._igloo_key_hist = (kmin, span, h)
    except (AttributeError, RuntimeError):
        return None
    return h


def _diff_bounds(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Device int64 [min, max] of a - b (both 0 <=> a == b everywhere) from
    the two-stage column_stats kernel: an ATen ``(a != b).sum()`` is a
    multi-block reduction whose semaphore memset does not replay inside a HIP
    graph (the query would never graph)."""
    d = (a.to(torch.int64) - b.to(torch.int64)).contiguous()
    if not d.is_cuda:
        return torch.stack([d.min(), d.max()]) if d.numel() else torch.zeros(2, dtype=torch.int64)
    N = launch("column_stats")
    buf = torch.empty(N.STATS_SLOTS, dtype=torch.int64, device=d.device)
    if d.numel() == 0:
        return torch.zeros(2, dtype=torch.int64, device=d.device)
    N.column_stats(ptr(d), True, 0, d.numel(), ptr(buf), stream(d))
    return buf[:2]


def _differs_from_rep(a: torch.Tensor, rr: torch.Tensor) -> torch.Tensor:
    """Device int32 flag: some a[i] != a[rr[i]] (csrc/kernels/util.hip
    differs_from_rep: one pass, no gathered copy)."""
    a = a.contiguous()
    flag = torch.empty(1, dtype=torch.int32, device=a.device)
    esz = a.element_size() * (a.shape[1] if a.dim() == 2 else 1)
    if esz not in (1, 2, 4, 8):
        d = _diff_bounds(a.reshape(a.shape[0], -1)[:, 0], a.reshape(a.shape[0], -1)[:, 0].index_select(0, rr))
        return (d != 0).any().to(torch.int32).reshape(1)
    launch("differs_from_rep").differs_from_rep(ptr(a), esz, ptr(rr), rr.dtype == torch.int64, a.shape[0],
                                                ptr(flag), stream(flag))
    return flag


def _late_group_keys(groups, b: "LateBatch", ctx, skip: Optional[set] = None):
    """GROUP BY over a join result still in index form, with plain string keys
    (TPC-H Q10: c_custkey plus six customer/nation attributes over 11M joined
    rows). Group by the widest integer key, then check per join input that its
    row index is constant within every group: a key whose source row is fixed
    by the group is functionally dependent on it, so it is dropped from the
    grouping and gathered only for the ng representative rows — the strings
    are never materialised for all joined rows. Returns (gid, ng, rep, taken)
    or None (shape does not apply or a dependency fails: the caller groups
    normally)."""
    cids = [e.cid if isinstance(e, ColRef) else None for _, e in groups]
    if any(c is None or c not in b.owner for c in cids):
        return None
    base = [b.parts[b.owner[c]][0].columns[c] for c in cids]
    plain = [i for i, c in enumerate(base) if c.dtype.is_string and not c.is_dict]
    others = [i for i in range(len(cids)) if i not in plain]
    if not plain or not others:
        return None
    keys = {i: group_key_tensor(b.gather(cids[i]))[0] for i in others}
    spans = _span_hints(keys, others)
    lead = _lead_key(others, spans, base)
    gid, ng, rep, srt = H.group_ids_ex(keys[lead])
    rr = gather_tensor(rep, gid)
    checks, parts = [], set()
    for i in range(len(cids)):
        k = b.owner[cids[i]]
        if i == lead or k in parts:
            continue
        idx = b.parts[k][1]
        if idx is None:
            return None
        parts.add(k)
        checks.append(_differs_from_rep(idx, rr) if idx.is_cuda else _diff_bounds(idx, gather_tensor(idx, rr)))
    if checks and any(to_host_ints(torch.cat([c.to(torch.int64) for c in checks]))):
        return None
    ctx.sorted_gids = srt
    taken = []
    for i, c in enumerate(cids):
        if skip and groups[i][0].cid in skip:
            taken.append(None)          # the caller ships this part's row instead
        elif i == lead:
            taken.append(take(b.gather(c), rep))
        else:
            bb, idx = b.parts[b.owner[c]]
            if i in plain:
                # strings are gathered when read: an ORDER BY ... LIMIT above
                # takes only its rows (columnar.py LazyColumn)
                taken.append(LazyColumn(base[i].dtype, bb, c, gather_tensor(idx, rep)))
            else:
                taken.append(take(bb.columns[c], gather_tensor(idx, rep)))
    return gid, ng, rep, taken


def _span_hints(keys, others):
    """Key ranges for ranking the lead key: resident-derived bounds where
    known (ops/hashing.py key_bound), the rest read back together."""
    spans = {i: H.key_bound(keys[i]) for i in others}
    todo = [i for i in others if spans[i] is None]
    if todo:
        for i, r in zip(todo, H.key_ranges([keys[i] for i in todo])):
            spans[i] = r
    return spans


def _lead_key(others, spans, cols) -> int:
    """The grouping key the others are tested to depend on: the widest-range
    plain integer key (a key column, e.g. c_custkey), before decimals and
    dictionary codes (an account balance spans more values than 150K
    customer keys at SF1, but identifies nothing)."""
    def rank(i):
        t = cols[i].dtype
        intlike = (t.is_integer and not t.is_decimal) and not cols[i].is_dict
        return (1 if intlike else 0, spans[i][1] - spans[i][0] if spans[i] else -1)
    return max(others, key=rank)


def _encode_groups(gcols: List[Column], ctx, fd: bool = False):
    """Dense group ids for GROUP BY over ``gcols`` -> (gid, ng, rep_row, rep_source_cols).

    Functional-dependency shortcut (GPU): when plain (non-dictionary) string
    keys are present -- or ``fd`` says the keys should depend on one integer
    key -- group by the integer key with the widest domain first and verify
    on the device that every other key is constant within those groups (a
    row-vs-representative comparison, far cheaper than hashing and
    dictionary-encoding strings or packing several keys). Keys that pass are
    dropped from the grouping -- the result is identical to grouping by all
    of them. TPC-H Q10 groups by c_custkey plus six customer attributes: one
    direct-mapped integer group-by replaces seven encodings; its SPMD merge
    groups custkey, balance, nation and the customer row shipped instead of
    the strings (parallel/exchange.py _partial_by_rows) the same way."""
    plain = [i for i, c in enumerate(gcols) if c.dtype.is_string and not c.is_dict]
    others = [i for i in range(len(gcols)) if i not in plain]
    keys: Dict[int, torch.Tensor] = {}
    reps_src: List[Column] = list(gcols)
    for i in others:
        keys[i], reps_src[i] = group_key_tensor(gcols[i], narrow=True)
    needed = list(range(len(gcols)))
    if (plain or (fd and len(gcols) > 1)) and others and ctx.device.type == "cuda":
        spans = _span_hints(keys, others)
        lead = _lead_key(others, spans, gcols)
        gid, ng, rep, srt = H.group_ids_ex(keys[lead])
        ctx.sorted_gids = srt
        rr = gather_tensor(rep, gid)
        checks, owner = [], []
        for i in range(len(gcols)):
            if i == lead:
                continue
            c = gcols[i]
            if i in plain:
                m = torch.zeros(1, dtype=torch.int32, device=ctx.device)
                launch("str_eq_rows").str_eq_rows(ptr(c.offsets), ptr(c.data), 0, ptr(c.offsets), ptr(c.data),
                                                  ptr(rr), False, len(c), ptr(m), stream(m))
                checks.append(m.to(torch.int64))
                owner.append(i)
            else:
                # any key unlike its representative's (one pass, graph-safe)
                checks.append(_differs_from_rep(keys[i], rr).to(torch.int64))
                owner.append(i)
            if c.valid is not None:
                checks.append(_differs_from_rep(c.valid, rr).to(torch.int64))
                owner.append(i)
        bad = {i for i, v in zip(owner, to_host_ints(torch.cat(checks))) if v}
        needed = [lead] + [i for i in range(len(gcols)) if i != lead and i in bad]
        if len(needed) == 1:
            return gid, ng, rep, reps_src
    for i in plain:
        if i in needed:
            keys[i], _ = group_key_tensor(gcols[i], narrow=True)
    packed = H.pack_keys([keys[i] for i in needed])
    gid, ng, rep, srt = H.group_ids_ex(packed)
    ctx.sorted_gids = srt
    return gid, ng, rep, reps_src


def _empty_col(t, dev) -> Column:
    if t.is_string:
        return Column(t, torch.zeros(0, dtype=torch.uint8, device=dev), None, offsets=torch.zeros(1, dtype=torch.int64, device=dev))
    return Column(t, torch.zeros(0, dtype=t.torch_dtype if t.kind != "null" else torch.bool, device=dev))


def _plan_agg(ci, a: AggCall, b: Batch, gid, ng, n, ctx, specs, finals):
    """Append kernel specs for one aggregate and a finaliser producing its column."""
    ev = ctx.evaluator
    dev = ctx.device
    func = a.func
    col = ev.column(a.arg, b) if a.arg is not None else None
    if func == "array_agg":
        # NULL elements are kept (DataFusion's array_agg); FILTER drops rows
        fv = ev.mask(a.filter, b) if a.filter is not None else None
        if a.distinct:
            k, _ = group_key_tensor(col)
            pair = H.pack_keys([gid.to(torch.int64) if gid is not None else
                                torch.zeros(n, dtype=torch.int64, device=dev), k])
            if col.valid is not None:
                pair = torch.where(col.valid, pair.to(torch.int64), torch.full((n,), -1, dtype=torch.int64, device=dev))
            if fv is not None:
                pair = torch.where(fv, pair.to(torch.int64), torch.full((n,), -2, dtype=torch.int64, device=dev))
            first = H.first_rows_mask(pair) if n else torch.zeros(0, dtype=torch.bool, device=dev)
            fv = first if fv is None else (fv & first)
        out = _array_agg(a, col, fv, gid, ng, n, ctx, b)
        finals.append(lambda r, out=out: (ci, out))
        return
    valid = col.valid if col is not None else None
    if a.filter is not None:
        fm = ev.mask(a.filter, b)
        valid = fm if valid is None else (valid & fm)
    if a.distinct and func in ("count", "sum", "avg"):
        # de-duplicate (group, value) pairs first, then aggregate the survivors;
        # rows a FILTER (or NULL) drops share one sentinel pair, so each kept
        # pair's first row is a row that passes
        k, _ = group_key_tensor(col)
        pair = H.pack_keys([gid.to(torch.int64) if gid is not None else torch.zeros(n, dtype=torch.int64, device=dev), k])
        keep_rows = torch.ones(n, dtype=torch.bool, device=dev) if valid is None else valid
        if n:
            if valid is not None:
                pair = torch.where(valid, pair.to(torch.int64), torch.full((n,), -1, dtype=torch.int64, device=dev))
            keep_rows = keep_rows & H.first_rows_mask(pair)
        valid = keep_rows
    base = len(specs)

    def add(op, vals, vv):
        specs.append((op, vals, vv))
        return len(specs) - 1

    t = a.dtype
    if func == "count":
        i = add("count", None, valid)
        finals.append(lambda r, i=i: (ci, Column(T.INT64, r[i])))
        return
    if func in ("median", "percentile", "percentile_disc"):
        out = _order_stat(a, col, valid, gid, ng, n, ctx)
        finals.append(lambda r, out=out: (ci, out))
        return
    if func == "string_agg":
        out = _string_agg(a, col, valid, gid, ng, n, ctx, b)
        finals.append(lambda r, out=out: (ci, out))
        return
    if func in ("covar_samp", "covar_pop", "corr"):
        c2 = ev.column(a.arg2, b)
        both = valid if c2.valid is None else (c2.valid if valid is None else valid & c2.valid)
        x = _convert_tensor(col, T.FLOAT64).contiguous()
        y = _convert_tensor(c2, T.FLOAT64).contiguous()
        ids = [add("sum_f64", v.contiguous(), both) for v in (x, y, x * y, x * x, y * y)]
        ic = add("count", None, both)

        def fin(r, ids=ids, ic=ic):
            sx, sy, sxy, sxx, syy = (r[i] for i in ids)
            c = r[ic].to(torch.float64)
            if func == "corr":
                num = c * sxy - sx * sy
                den = ((c * sxx - sx * sx) * (c * syy - sy * sy)).clamp(min=0).sqrt()
                return ci, Column(T.FLOAT64, num / den.clamp(min=1e-300), (c > 1) & (den > 0))
            pop = func == "covar_pop"
            cov = (sxy - sx * sy / c.clamp(min=1)) / (c if pop else c - 1).clamp(min=1)
            return ci, Column(T.FLOAT64, cov, c > (0 if pop else 1))
        finals.append(fin)
        return
    if col is None:
        raise ExecutionError(f"{func} needs an argument")
    src = col.dtype
    cnt_i = add("count", None, valid) if (valid is not None or func in ("avg",) or n == 0 or gid is None) else None

    def null_if_empty(r, data, cnt_i=cnt_i):
        if cnt_i is None:
            return None
        return r[cnt_i] > 0

    if func in ("sum", "avg"):
        if src.is_float:
            si = add("sum_f64", col.data.to(torch.float64).contiguous(), valid)
        else:
            vals = col.data
            if vals.dtype not in (torch.int32, torch.int64):
                vals = vals.to(torch.int64)
            si = add("sum_int", vals.contiguous(), valid)
        if func == "sum":
            def fin(r, si=si):
                v = r[si]
                vv = null_if_empty(r, v)
                return ci, Column(t, v if not t.is_float else v.to(torch.float64), vv)
            finals.append(fin)
        else:
            def fin(r, si=si):
                s, c = r[si], r[cnt_i]
                vv = c > 0
                return ci, Column(t, _avg(s, c, src, t), vv)
            finals.append(fin)
        return
    if func in ("min", "max"):
        if src.is_string:
            d = col if col.is_dict else S.dict_encode(col)
            ranks = S.sort_ranks(d)
            vals = d.dictionary
            i = add("min_int" if func == "min" else "max_int", ranks.contiguous(), valid)
            # map winning rank back to a dictionary code
            from ..ops.sort import argsort as _argsort
            dranks = S.sort_ranks(Column(T.UTF8, torch.arange(len(vals), dtype=torch.int32, device=dev), None,
                                         dictionary=vals))
            order = _argsort([(dranks, False, False, None)], dranks.numel(), dev)

            def fin(r, i=i, order=order, d=d):
                rk = r[i]
                vv = null_if_empty(r, rk)
                safe = rk.clamp(0, max(len(order) - 1, 0))
                codes = gather_tensor(order, safe).to(torch.int32) if len(order) else safe.to(torch.int32)
                return ci, Column(T.UTF8, codes, vv, dictionary=d.dictionary)
            finals.append(fin)
            return
        if src.is_float:
            i = add("min_f64" if func == "min" else "max_f64", col.data.to(torch.float64).contiguous(), valid)
            finals.append(lambda r, i=i: (ci, Column(t, r[i].to(t.torch_dtype), null_if_empty(r, r[i]))))
            return
        vals = col.data
        if vals.dtype not in (torch.int32, torch.int64):
            vals = vals.to(torch.int64)
        i = add("min_int" if func == "min" else "max_int", vals.contiguous(), valid)
        finals.append(lambda r, i=i: (ci, Column(t, r[i].to(t.torch_dtype) if t.kind != "bool" else r[i] != 0,
                                                 null_if_empty(r, r[i]))))
        return
    if func in ("bit_and", "bit_or", "bit_xor"):
        vals = col.data
        if vals.dtype not in (torch.int32, torch.int64):
            vals = vals.to(torch.int64)
        i = add({"bit_and": "and_int", "bit_or": "or_int", "bit_xor": "xor_int"}[func], vals.contiguous(), valid)
        finals.append(lambda r, i=i: (ci, Column(t, r[i].to(t.torch_dtype), null_if_empty(r, r[i]))))
        return
    if func in ("bool_and", "bool_or"):
        vals = col.data.to(torch.int64)
        i = add("min_int" if func == "bool_and" else "max_int", vals.contiguous(), valid)
        finals.append(lambda r, i=i: (ci, Column(T.BOOL, r[i] != 0, null_if_empty(r, r[i]))))
        return
    if func in ("stddev", "stddev_samp", "stddev_pop", "var", "var_samp", "var_pop"):
        x = _convert_tensor(col, T.FLOAT64).contiguous()
        s1 = add("sum_f64", x, valid)
        s2 = add("sum_f64", (x * x).contiguous(), valid)
        ci_ = add("count", None, valid)

        def fin(r, s1=s1, s2=s2, ci_=ci_):
            c = r[ci_].to(torch.float64)
            mean = r[s1] / c.clamp(min=1)
            pop = func.endswith("_pop")
            denom = c if pop else (c - 1)
            var = (r[s2] - c * mean * mean) / denom.clamp(min=1)
            var = var.clamp(min=0)
            out = var.sqrt() if func.startswith("stddev") else var
            return ci, Column(T.FLOAT64, out, c > (0 if pop else 1))
        finals.append(fin)
        return
    raise NotSupported(f"aggregate {func}")


def _order_perm(order, b: Batch, n: int, ctx) -> torch.Tensor:
    """Row permutation of ``b`` by an ordered aggregate's ORDER BY keys."""
    from ..ops import sort as SO
    ks = []
    for e, asc, nf in order:
        c = ctx.evaluator.column(e, b)
        if c.dtype.is_string:
            v = S.sort_ranks(c)
        elif c.is_wide:
            v = _convert_tensor(c, T.FLOAT64)
        else:
            v = c.data
        ks.append((v, not asc, nf, c.valid))
    return SO.argsort(ks, n, ctx.device).to(torch.int64)


def _group_sorted(x: torch.Tensor, valid, gid, ng: int, n: int, ctx, by_value: bool, perm0=None):
    """Valid rows ordered by (group[, value]) -> (row ids, per-group counts,
    per-group first position). ``perm0``: rows are taken in this order
    (an ordered aggregate's ORDER BY) before the stable group sort."""
    from ..ops import sort as SO
    from ..ops.select import mask_to_indices
    dev = ctx.device
    if perm0 is not None:
        rows = perm0 if valid is None else perm0[gather_tensor(valid, perm0)]
    else:
        rows = mask_to_indices(valid).to(torch.int64) if valid is not None else \
            torch.arange(n, dtype=torch.int64, device=dev)
    m = rows.numel()
    g = gather_tensor(gid, rows).to(torch.int64) if gid is not None else torch.zeros(m, dtype=torch.int64, device=dev)
    keys = [] if gid is None else [(g, False, False, None)]
    if by_value:
        keys.append((gather_tensor(x, rows), False, False, None))
    if keys and m > 1:
        perm = SO.argsort(keys, m, dev).to(torch.int64)
        rows, g = gather_tensor(rows, perm), gather_tensor(g, perm)
    counts = torch.bincount(g, minlength=ng)[:ng] if m else torch.zeros(ng, dtype=torch.int64, device=dev)
    starts = torch.cumsum(counts, 0) - counts
    return rows, counts, starts


def _order_stat(a: AggCall, col: Column, valid, gid, ng: int, n: int, ctx) -> Column:
    """median (middle value; the mean of the two middle values, truncated in
    the input type) and approx_percentile_cont (linear interpolation) per group."""
    t = a.dtype
    fl = col.dtype.is_float or col.is_wide or a.func == "percentile"
    if a.func == "percentile_disc":
        fl = col.dtype.is_float or col.is_wide
    x = _convert_tensor(col, T.FLOAT64) if (fl or col.is_wide) else col.data.to(torch.int64)
    rows, counts, starts = _group_sorted(x, valid, gid, ng, n, ctx, True)
    xs = gather_tensor(x, rows) if rows.numel() else x[:0]
    last = max(rows.numel() - 1, 0)
    ok = counts > 0
    if not rows.numel():
        return Column(t, torch.zeros(ng, dtype=t.torch_dtype if t.kind != "decimal" else torch.int64,
                                     device=ctx.device), ok)
    if a.func == "percentile_disc":
        # the first value whose cumulative distribution reaches the fraction
        k = torch.ceil(counts.to(torch.float64) * float(a.param)).to(torch.int64) - 1
        v = gather_tensor(xs, (starts + k.clamp(min=0)).clamp(0, last))
        return Column(t, v if t.is_decimal else v.to(t.torch_dtype), ok)
    if a.func == "percentile":
        pos = (counts - 1).clamp(min=0).to(torch.float64) * float(a.param)
        lo = pos.floor().to(torch.int64)
        frac = pos - lo.to(torch.float64)
        hi_ = torch.minimum(lo + 1, (counts - 1).clamp(min=0))
        v0 = gather_tensor(xs, (starts + lo).clamp(0, last))
        v1 = gather_tensor(xs, (starts + hi_).clamp(0, last))
        return Column(T.FLOAT64, v0 + (v1 - v0) * frac, ok)
    lo = (starts + torch.div(counts - 1, 2, rounding_mode="floor")).clamp(0, last)
    hi_ = (starts + torch.div(counts, 2, rounding_mode="floor")).clamp(0, last)
    v0, v1 = gather_tensor(xs, lo), gather_tensor(xs, hi_)
    if x.dtype == torch.float64:
        med = (v0 + v1) / 2
        return Column(t, med if t.is_float else med.to(torch.int64), ok)
    med = torch.div(v0 + v1, 2, rounding_mode="trunc")
    return Column(t, med.to(t.torch_dtype) if not t.is_decimal else med, ok)


def _string_agg(a: AggCall, col: Column, valid, gid, ng: int, n: int, ctx, b=None) -> Column:
    """string_agg(s, sep): each group's strings in input order joined by sep.
    Rows are ordered by group (stable), a separator is prefixed to every row
    that does not start its group, and each group's string is then one
    contiguous byte range of the concatenated pieces: the output offsets are
    the pieces' offsets at the group starts (no per-group copy)."""
    from ..ops.gather import take
    dev = ctx.device
    perm0 = _order_perm(a.order, b, n, ctx) if a.order and b is not None and n > 1 else None
    rows, counts, starts = _group_sorted(None, valid, gid, ng, n, ctx, False, perm0)
    m = rows.numel()
    if m == 0:
        z = torch.zeros(ng + 1, dtype=torch.int64, device=dev)
        return Column(T.UTF8, torch.zeros(0, dtype=torch.uint8, device=dev), counts > 0, offsets=z)
    sv = S.decode(take(col, rows))
    sv = Column(T.UTF8, sv.data, None, offsets=sv.offsets)
    head = torch.zeros(m, dtype=torch.bool, device=dev)
    head.index_fill_(0, starts[counts > 0], True)
    sep = S.const_column(str(a.param), dev)
    empty = S.const_column("", dev)
    prefix = S.select_rows([empty, sep], (~head).to(torch.int64), m)
    pieces = S.concat(prefix, sv, m)
    off = pieces.offsets
    out_off = torch.cat([gather_tensor(off, starts.clamp(max=m)), off[m:m + 1]])
    return Column(T.UTF8, pieces.data, counts > 0, offsets=out_off)


def _array_agg(a: AggCall, col: Column, valid, gid, ng: int, n: int, ctx, b) -> Column:
    """array_agg(x [ORDER BY ...]): each group's values as one list, in input
    (or the given) order. Rows are ordered by group (stable) and gathered
    once; group g's list is the (start, count) slice of that child."""
    from ..ops import nested as NS
    perm0 = _order_perm(a.order, b, n, ctx) if a.order and n > 1 else None
    rows, counts, starts = _group_sorted(None, valid, gid, ng, n, ctx, False, perm0)
    child = take(col, rows)
    return NS.from_groups(child, starts, counts, a.dtype, counts > 0)


def _avg(s: torch.Tensor, c: torch.Tensor, src, t) -> torch.Tensor:
    cc = c.clamp(min=1)
    if t.is_decimal:
        up = 10 ** (t.scale - (src.scale if src.is_decimal else 0))
        if s.is_cuda:
            # exact rounded division of the (int64 or 128-bit) sums on the device
            out = torch.empty(s.shape[0], dtype=torch.int64, device=s.device)
            launch("avg_wide").avg_wide(ptr(s.contiguous()), s.dim() == 2, ptr(c.to(torch.int64).contiguous()),
                                        s.shape[0], up, ptr(out), stream(s))
            return out
        if s.dim() == 1:
            lim = (2**63 - 1) // up
            if to_host_int((s.abs() < lim).all().to(torch.int64)):
                num = s * up
                q = torch.div(num.abs() + cc // 2, cc, rounding_mode="floor") * torch.sign(num)
                return q
        # exact host path for huge sums (few groups)
        vals = A.wide_to_python(s)
        cs = c.cpu().tolist()
        res = []
        for v, k in zip(vals, cs):
            k = max(k, 1)
            num = v * up
            q = (abs(num) + k // 2) // k
            res.append(q if num >= 0 else -q)
        if all(-(2**63) <= q < 2**63 for q in res):
            return torch.tensor(res, dtype=torch.int64, device=s.device)
        # a decimal(38, s) average past 63 bits: the (lo, hi) 128-bit layout
        pairs = [[((q + 2**64) % 2**64) - (2**64 if ((q + 2**64) % 2**64) >= 2**63 else 0), q >> 64] for q in res]
        return torch.tensor(pairs, dtype=torch.int64, device=s.device).reshape(len(res), 2)
    if s.dim() == 2:
        lo = s[:, 0].to(torch.float64)
        lo = torch.where(lo < 0, lo + 18446744073709551616.0, lo)
        sf = s[:, 1].to(torch.float64) * 18446744073709551616.0 + lo
    else:
        sf = s.to(torch.float64)
    if src.is_decimal:
        sf = sf / 10**src.scale
    return sf / cc.to(torch.float64)
