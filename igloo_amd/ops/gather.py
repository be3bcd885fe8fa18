"""Gathers by row index (csrc/kernels/gather.hip).

``take_many`` gathers several columns with ONE launch for all fixed-width
columns (plus validity), which is the late-materialisation step after a
join/filter/sort. Negative indices produce NULL rows (outer-join padding).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ..columnar import Column
from ._lib import is_gpu, launch, ptr, stream, to_host_ints
from .packed_gather import packed_take
from .select import offsets_from_lengths


def origin(t: torch.Tensor) -> Optional[torch.Tensor]:
    """The resident table column every value of ``t`` was gathered from (no
    negative rows), or None: ``t`` itself, a filtered scan's source
    (exec/scan.py _tag_base) or the origin a gather inherited (take_many).
    ops/hashing.py key_bound derives key ranges from it without a readback."""
    if getattr(t, "_igloo_resident", False):
        return t
    o = getattr(t, "_igloo_origin", None)
    if o is not None:
        return o
    base = getattr(t, "_igloo_base", None)
    if base is not None and base[0].data.dtype == t.dtype:
        return origin(base[0].data)
    return None


def _inherit(dst: torch.Tensor, src: torch.Tensor, idx: Optional[torch.Tensor] = None) -> None:
    o = origin(src)
    if o is not None:
        dst._igloo_origin = o
    if idx is not None and getattr(idx, "_igloo_incr", False) and getattr(src, "_igloo_sorted", False) is True:
        # rows of a sorted column taken in row order stay sorted: later
        # sorted-join / run-grouping checks need no pass (ops/hashing.py is_sorted)
        dst._igloo_sorted = True


def _cpu_take_tensor(t: torch.Tensor, idx: torch.Tensor, neg: bool) -> torch.Tensor:
    if not neg:
        return t.index_select(0, idx.long())
    ii = idx.long()
    safe = ii.clamp(min=0)
    out = t.index_select(0, safe) if t.numel() else torch.zeros((ii.numel(),) + tuple(t.shape[1:]), dtype=t.dtype)
    out[ii < 0] = 0
    return out


def _take_plain_strings(col: Column, idx: torch.Tensor, neg: bool) -> Column:
    n = idx.numel()
    if not is_gpu(idx):
        ii = idx.long()
        off = col.offsets
        safe = ii.clamp(min=0)
        starts = off.index_select(0, safe) if n else torch.zeros(0, dtype=torch.int64)
        lens = (off.index_select(0, safe + 1) - starts) if n else torch.zeros(0, dtype=torch.int64)
        if neg:
            lens = torch.where(ii < 0, torch.zeros_like(lens), lens)
        new_off, total = offsets_from_lengths(lens)
        if total:
            # byte positions: for each output byte, source = start[row] + (pos - new_off[row])
            rows = torch.repeat_interleave(torch.arange(n), lens)
            pos = torch.arange(total) - new_off[:-1].index_select(0, rows) + starts.index_select(0, rows)
            chars = col.data.index_select(0, pos)
        else:
            chars = torch.zeros(0, dtype=torch.uint8)
        return Column(col.dtype, chars, None, offsets=new_off)
    return _take_strings_gpu([col], idx)[0]


def _take_strings_gpu(cols: Sequence[Column], idx: torch.Tensor) -> List[Column]:
    """Plain string gathers of several columns by one index: the lengths and
    offsets of every column first, then ONE readback of all their byte totals
    (to size the character buffers), then the copies."""
    n = idx.numel()
    N = launch("str_gather")
    s = stream(idx)
    idx64 = idx.dtype == torch.int64
    offs = []
    for col in cols:
        lens = torch.empty(n, dtype=torch.int64, device=idx.device)
        N.str_gather_lengths(ptr(col.offsets), len(col), ptr(idx), idx64, n, ptr(lens), s)
        offs.append(offsets_from_lengths(lens, host_total=False)[0])
    totals = to_host_ints(torch.cat([o[-1:] for o in offs]) if len(offs) > 1 else offs[0][-1:])
    out = []
    for col, new_off, total in zip(cols, offs, totals):
        chars = torch.empty(max(total, 0), dtype=torch.uint8, device=idx.device)
        if total:
            N.str_gather_copy(ptr(col.offsets), len(col), ptr(col.data), ptr(idx), idx64, n, ptr(new_off),
                              ptr(chars), chars.numel(), s)
        out.append(Column(col.dtype, chars, None, offsets=new_off))
    return out


def _src_ptr(t) -> int:
    """Source pointer for gather_multi: 0 for an empty (or absent) column, so
    the kernel's unconditional loads of NULL rows read its zero page instead of
    whatever lies at an empty tensor's address."""
    return ptr(t) if t is not None and t.numel() else 0


def take_many(cols: Sequence[Column], idx: torch.Tensor, neg: bool = False) -> List[Column]:
    """Gather rows ``idx`` of every column. ``neg=True``: idx may hold -1 (NULL row)."""
    assert idx.dim() == 1 and idx.dtype in (torch.int32, torch.int64)
    from ..columnar import LazyColumn
    if not neg and any(isinstance(c, LazyColumn) and c.pending for c in cols):
        # deferred columns stay deferred: only their row index is composed
        lazy = {i: c.taken(idx) for i, c in enumerate(cols) if isinstance(c, LazyColumn) and c.pending}
        rest = [c for i, c in enumerate(cols) if i not in lazy]
        done = iter(take_many(rest, idx, neg) if rest else [])
        return [lazy[i] if i in lazy else next(done) for i in range(len(cols))]
    n = idx.numel()
    gpu = is_gpu(idx)
    out: List[Column] = []
    # GPU: (src, dst, elem_bytes, src_valid, dst_valid, src_rows) -> one gather_multi launch; indices
    # outside the source (a replayed size can leave an index tail unwritten) gather NULL / zero
    descs = []
    keepalive = []  # temporaries that must outlive the (stream-ordered) launch
    strs = [c for c in cols if c.is_plain_string]
    pre = iter(_take_strings_gpu(strs, idx) if gpu and strs else [])
    # several resident columns at sparse / random rows: one row-packed gather
    packed = packed_take(cols, idx, neg) if gpu and len(cols) > 1 else {}
    for k, c in enumerate(cols):
        if k in packed:
            out.append(packed[k])
            continue
        need_valid = neg or c.valid is not None
        if c.is_plain_string:
            nc = next(pre) if gpu else _take_plain_strings(c, idx, neg)
            if need_valid:
                if gpu:
                    src = c.valid
                    if src is None:
                        src = torch.ones(len(c), dtype=torch.bool, device=idx.device)
                        keepalive.append(src)
                    v = torch.empty(n, dtype=torch.bool, device=idx.device)
                    # validity gathered as a byte column; idx < 0 writes 0 = NULL
                    descs.append((_src_ptr(src), ptr(v), 1, 0, 0, src.numel()))
                else:
                    base = c.valid if c.valid is not None else torch.ones(len(c), dtype=torch.bool)
                    v = _cpu_take_tensor(base, idx, neg)
                nc.valid = v
            out.append(nc)
            continue
        if not gpu:
            data = _cpu_take_tensor(c.data, idx, neg)
            valid = None
            if need_valid:
                base = c.valid if c.valid is not None else torch.ones(len(c), dtype=torch.bool)
                valid = _cpu_take_tensor(base, idx, neg)
            out.append(Column(c.dtype, data, valid, dictionary=c.dictionary))
            continue
        data = torch.empty((n,) + tuple(c.data.shape[1:]), dtype=c.data.dtype, device=idx.device)
        esz = c.data.element_size() * (c.data.shape[1] if c.data.dim() == 2 else 1)
        valid = torch.empty(n, dtype=torch.bool, device=idx.device) if need_valid else None
        descs.append((_src_ptr(c.data), ptr(data), esz, _src_ptr(c.valid), ptr(valid), c.data.shape[0]))
        if not neg:
            _inherit(data, c.data, idx)
            if getattr(idx, "_igloo_incr", False) and getattr(c.data, "_igloo_distinct", False):
                data._igloo_distinct = True
        out.append(Column(c.dtype, data, valid, dictionary=c.dictionary))
    if gpu and descs and n:
        N = launch("gather_multi")
        N.gather_multi(ptr(idx), idx.dtype == torch.int64, n, descs, stream(idx))
    del keepalive
    return out


def gather_tensor(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``t[idx]`` along dim 0 (idx int32/int64, no negatives). GPU: the
    gather_multi kernel (int32 indices used as is, no int64 conversion pass)."""
    if not is_gpu(idx):
        return t.index_select(0, idx.long())
    t = t.contiguous()
    n = idx.numel()
    out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=idx.device)
    if n:
        esz = t.element_size() * (t.shape[1] if t.dim() == 2 else 1)
        launch("gather_multi").gather_multi(ptr(idx), idx.dtype == torch.int64, n,
                                            [(ptr(t), ptr(out), esz, 0, 0, t.shape[0])], stream(idx))
    _inherit(out, t, idx)
    return out


def take(col: Column, idx: torch.Tensor, neg: bool = False) -> Column:
    return take_many([col], idx, neg)[0]
