"""Row-packed gathers of several columns of one resident table
(csrc/kernels/gather.hip ``gather_packed``).

A sparse or random gather touches one cache line per row PER COLUMN: TPC-H
Q9's final payload gather takes 32M of 600M lineitem rows (5.4 %), so four
separate 8-byte column gathers fetch close to four 128-byte lines per row. A
row-packed copy of those columns (each narrowed to its value range by
exec/fused.py ``narrow``, fields widest first, rows padded to 8 bytes, at most
32) turns that into one line per row; the kernel widens every field back to
its column's type. Measured in isolation 2.05x over four 4-byte column gathers
at 5.4 % density (scripts/bench_gather_packed.py).

The copy is built on the first request for a column set and kept on the
first member's tensor as a derived structure (``_igloo_packed``, dropped with
the cache tier's other derived structures, utils/memory.py); a later request
for a subset of a kept copy's columns reuses it. Copies are bounded by
``IGLOO_PACK_BUDGET_GB`` per process, and are never built inside a graph
capture (the gather then runs per column).

The reference materialises join output with arrow ``take`` per column
(reference crates/engine/src/operators/hash_join.rs:221-240); this layout has
no counterpart there."""
from __future__ import annotations

import os
import weakref
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..columnar import Column
from . import _lib
from ._lib import launch, ptr, stream

PACKED = True
#: fewer gathered rows than this: the per-column gather (launch-bound anyway)
MIN_ROWS = 1 << 20
#: an ascending index denser than this reads most lines of every column
#: anyway: the per-column gather
MAX_ASC_DENSITY = 0.5
MAX_ROW_BYTES = 32
BUDGET = int(float(os.environ.get("IGLOO_PACK_BUDGET_GB", "24")) * (1 << 30))

_FIXED = {torch.int8: True, torch.int16: True, torch.int32: True, torch.int64: True, torch.bool: False,
          torch.uint8: False, torch.float32: False, torch.float64: False}
_live: "weakref.WeakSet[torch.Tensor]" = weakref.WeakSet()

Member = Tuple[int, int]                     # (data pointer, validity pointer or 0)
# members: {member: (value offset, value width, signed, validity offset or -1)}
Pack = Tuple[torch.Tensor, Dict[Member, Tuple[int, int, bool, int]], int]
STATS = {"builds": 0, "gathers": 0, "refused_budget": 0}


def _member(c: Column) -> Member:
    return (c.data.data_ptr(), c.valid.data_ptr() if c.valid is not None else 0)


def _eligible(c: Column, rows: int) -> bool:
    d = c.data
    return (not c.is_plain_string and not c.dtype.is_nested and d.dim() == 1 and d.dtype in _FIXED and d.is_cuda
            and len(d) == rows
            and getattr(d, "_igloo_resident", False) and (c.valid is None or c.valid.numel() == rows))


def _find(cands: Sequence[Column], want: List[Member]) -> Optional[Pack]:
    """The kept copy holding the most of ``want`` (at least two), or None."""
    best, hit = None, 1
    for c in cands:
        for pk in getattr(c.data, "_igloo_packed", None) or ():
            k = sum(m in pk[1] for m in want)
            if k > hit:
                best, hit = pk, k
    return best


def _value_tensor(c: Column) -> torch.Tensor:
    from ..exec.fused import narrow
    return narrow(c.data)


def _build(cols: Sequence[Column]) -> Optional[Pack]:
    """Packed copy of ``cols`` (all eligible, same length), None past the budget."""
    vals = [_value_tensor(c) for c in cols]
    tensors: List[torch.Tensor] = []
    spec = []
    for c, v in zip(cols, vals):
        spec.append((len(tensors), len(tensors) + 1 if c.valid is not None else -1))
        tensors.append(v)
        if c.valid is not None:
            tensors.append(c.valid.view(torch.uint8))
    from .pack import layout, pack_rows
    lay = layout(tensors)
    rb = lay[0]
    if rb > MAX_ROW_BYTES:
        return None
    rows = len(cols[0].data)
    need = rows * rb
    if sum(t.numel() for t in _live) + need > BUDGET:
        STATS["refused_budget"] += 1
        return None
    offs = {i: off for i, _, off in lay[1]}
    packed, _ = pack_rows(tensors, None, rows, lay)
    members = {}
    for c, v, (vi, vv) in zip(cols, vals, spec):
        members[_member(c)] = (offs[vi], v.element_size(), _FIXED[v.dtype], offs[vv] if vv >= 0 else -1)
    pk: Pack = (packed, members, rb)
    owner = cols[0].data
    try:
        owner._igloo_packed = list(getattr(owner, "_igloo_packed", None) or ()) + [pk]
    except (AttributeError, RuntimeError):
        return None
    _live.add(packed)
    STATS["builds"] += 1
    return pk


def _fit(cands: List[Column]) -> List[Column]:
    """Narrowest columns first, as many as fit in one packed row."""
    from .pack import layout

    def fields(c: Column) -> List[torch.Tensor]:
        v = _value_tensor(c)
        return [v] if c.valid is None else [v, c.valid.view(torch.uint8)]
    out: List[Column] = []
    tensors: List[torch.Tensor] = []
    for c in sorted(cands, key=lambda c: sum(t.element_size() for t in fields(c))):
        if layout(tensors + fields(c))[0] <= MAX_ROW_BYTES:
            out.append(c)
            tensors += fields(c)
    return out


def packed_take(cols: Sequence[Column], idx: torch.Tensor, neg: bool) -> Dict[int, Column]:
    """Columns of ``cols`` (by position) gathered through a row-packed copy;
    the positions not in the result are left to the caller's per-column path."""
    n = idx.numel()
    if not PACKED or n < MIN_ROWS or not idx.is_cuda:
        return {}
    rows = next((len(c.data) for c in cols if not c.is_plain_string and c.data.dim() == 1), -1)
    pos = [i for i, c in enumerate(cols) if rows > 0 and _eligible(c, rows)]
    if len(pos) < 2:
        return {}
    if getattr(idx, "_igloo_incr", False) and n > MAX_ASC_DENSITY * rows:
        return {}
    cand = [cols[i] for i in pos]
    want = [_member(c) for c in cand]
    pk = _find(cand, want)
    if (pk is None or not all(m in pk[1] for m in want)) and not getattr(_lib._capture, "on", False):
        # no kept copy holds every column: one for the columns that fit a row
        chosen = _fit(cand)
        if len(chosen) >= 2 and (pk is None or not all(_member(c) in pk[1] for c in chosen)):
            pk = _build(chosen) or pk
    if pk is None:
        return {}
    packed, members, rb = pk
    fields, out = [], {}
    for i in pos:
        c = cols[i]
        m = members.get(_member(c))
        if m is None:
            continue
        off, w, signed, voff = m
        data = torch.empty(n, dtype=c.data.dtype, device=idx.device)
        fields.append((ptr(data), off, w, data.element_size(), 1 if signed else 0))
        valid = None
        if c.valid is not None:
            valid = torch.empty(n, dtype=torch.bool, device=idx.device)
            fields.append((ptr(valid), voff, 1, 1, 0))
        elif neg:
            valid = torch.empty(n, dtype=torch.bool, device=idx.device)
            fields.append((ptr(valid), 0, 1, 1, 2))
        if not neg:
            from .gather import _inherit
            _inherit(data, c.data, idx)
            if getattr(idx, "_igloo_incr", False) and getattr(c.data, "_igloo_distinct", False):
                data._igloo_distinct = True
        out[i] = Column(c.dtype, data, valid, dictionary=c.dictionary)
    if len(out) < 2:
        return {}
    N = launch("gather_packed")
    s = stream(idx)
    for k in range(0, len(fields), 16):
        N.gather_packed(ptr(idx), idx.dtype == torch.int64, n, ptr(packed), packed.shape[0], rb, fields[k:k + 16], s)
    STATS["gathers"] += 1
    return out
