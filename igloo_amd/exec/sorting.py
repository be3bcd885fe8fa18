"""Sort / top-k, limit and union operators.

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
from .context import ExecNode
from .joins import _take_batch, concat_batches


# ============================================================ sort / limit / union
class SortExec(ExecNode):
    def __init__(self, logical: L.Sort, child: ExecNode):
        self.logical = logical
        self.children = [child]

    def describe(self):
        s = self.logical
        k = ", ".join(f"{e.sql()} {'ASC' if a else 'DESC'} NULLS {'FIRST' if nf else 'LAST'}" for e, a, nf in s.keys)
        return k + (f", fetch={s.fetch}" if s.fetch is not None else "")

    def _run(self, ctx):
        b = self.children[0].execute(ctx)
        fetch = self.logical.fetch
        if ctx.spmd and b.dist != ("replicated",):
            from ..parallel.exchange import SMALL_GATHER_ROWS, gather_all, gather_small
            if fetch is not None:
                # distributed ORDER BY ... LIMIT k: local top-k first, then only
                # k rows per rank cross the fabric, in one fixed-size all-gather
                dist = b.dist
                b = sort_batch(b, self.logical.keys, fetch, ctx)
                b.dist = dist
            b = gather_small(b, ctx, fetch) if fetch is not None and fetch <= SMALL_GATHER_ROWS \
                else gather_all(b, ctx)
        out = None
        if ctx.budget is not None:
            from .morsel import external_sort
            out = external_sort(b, self.logical.keys, fetch, ctx)
        if out is None:
            out = sort_batch(b, self.logical.keys, fetch, ctx)
        out.dist = b.dist
        return out


def sort_batch(b: Batch, keys, fetch, ctx) -> Batch:
    """ORDER BY [LIMIT fetch]: packed keys + radix sort, or radix select +
    candidate sort for a LIMIT (ops/sort.py)."""
    from ..ops import sort as SO
    n = b.num_rows
    if n <= 1:
        return b
    ev = ctx.evaluator
    if fetch is not None and len(keys) > 1 and ctx.device.type == "cuda":
        # keep the rows the leading numeric keys can still admit to the top
        # `fetch` before ranking string tie-breakers (TPC-H Q2, Q21)
        lead = []
        for e, asc, nf in keys:
            c = ev.column(e, b)
            if c.dtype.is_string or c.is_wide or c.data.dim() != 1:
                break
            lead.append((c.data, not asc, nf, c.valid))
        if lead and len(lead) < len(keys):
            cand = SO.topk_candidates(lead, n, fetch)
            if cand is not None and cand.numel() < n:
                b = _take_batch(b, cand)
                n = b.num_rows
    ks = []
    for e, asc, nf in keys:
        c = ev.column(e, b)
        if c.dtype.is_string:
            v = S.sort_ranks(c)
        elif c.is_wide:
            v = _convert_tensor(c, T.FLOAT64)
        else:
            v = c.data
        ks.append((v, not asc, nf, c.valid))
    if fetch is not None and fetch < n:
        perm = SO.topk(ks, n, fetch, ctx.device)
    else:
        perm = SO.argsort(ks, n, ctx.device)
    return _take_batch(b, perm)


class LimitExec(ExecNode):
    def __init__(self, logical: L.Limit, child: ExecNode):
        self.logical = logical
        self.children = [child]

    def describe(self):
        return f"skip={self.logical.offset}, fetch={self.logical.limit}"

    def _run(self, ctx):
        b = self.children[0].execute(ctx)
        if ctx.spmd and b.dist != ("replicated",):
            from ..parallel.exchange import gather_all
            if self.logical.limit is not None:
                # any offset+limit rows of each rank can make the answer
                keep = min(b.num_rows, self.logical.offset + self.logical.limit)
                if keep < b.num_rows:
                    dist = b.dist
                    b = _take_batch(b, torch.arange(keep, dtype=torch.int64, device=ctx.device))
                    b.dist = dist
            b = gather_all(b, ctx)
        lo = min(self.logical.offset, b.num_rows)
        hi = b.num_rows if self.logical.limit is None else min(b.num_rows, lo + self.logical.limit)
        if lo == 0 and hi == b.num_rows:
            return b
        idx = torch.arange(lo, hi, dtype=torch.int64, device=ctx.device)
        out = _take_batch(b, idx)
        out.dist = b.dist
        return out


class UnionExec(ExecNode):
    def __init__(self, logical: L.Union, children: List[ExecNode]):
        self.logical = logical
        self.children = children

    def _run(self, ctx):
        outs = []
        for ch, p in zip(self.children, self.logical.children):
            b = ch.execute(ctx)
            outs.append(Batch({s.cid: b.columns[c.cid] for s, c in zip(self.logical.schema, p.schema)}, b.num_rows,
                              b.dist))
        if ctx.spmd:
            reps = [o.dist == ("replicated",) for o in outs]
            if all(reps):
                out = concat_batches(outs)
                out.dist = ("replicated",)
                return out
            if any(reps) and ctx.comm.rank != 0:
                # a replicated input contributes its rows once (from rank 0)
                outs = [_take_batch(o, torch.zeros(0, dtype=torch.int32, device=ctx.device)) if r else o
                        for o, r in zip(outs, reps)]
        return concat_batches(outs)
