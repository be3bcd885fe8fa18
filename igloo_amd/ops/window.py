"""Window-function primitives (csrc/kernels/window.hip).

Rows arrive sorted by (partition, order) keys; ``ids`` are the sorted
partition (or peer-group) ids, so a segment is a run of equal ids. GPU
tensors run the hand-written gfx950 kernels; CPU tensors take the torch
reference path below (same results: the numerics oracle of the GPU tests).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._lib import is_gpu, launch, ptr, stream, to_host_int

# value sources (kernels.h WinVal)
V_I64, V_I32, V_F64, V_ONE, V_HEADIDX, V_HEAD2 = range(6)
# scan operators
SUM_I, SUM_F, MIN_I, MAX_I, MIN_F, MAX_F = range(6)
# ranking / index functions (kernels.h WinFn)
ROW_NUMBER, RANK, DENSE_RANK, PERCENT_RANK, CUME_DIST, NTILE = range(6)
LAG, FIRST, LAST, NTH = 10, 11, 12, 13
FRAME_KIND = {"unbounded_preceding": 0, "preceding": 1, "current": 2, "following": 3, "unbounded_following": 4}
UNIT = {"rows": 0, "range": 1, "groups": 2}

_I64MIN, _I64MAX = -2**63, 2**63 - 1


def _identity(op: int):
    return {SUM_I: 0, SUM_F: 0.0, MIN_I: _I64MAX, MAX_I: _I64MIN, MIN_F: float("inf"), MAX_F: float("-inf")}[op]


def seg_scan(ids: Optional[torch.Tensor], vals: Optional[torch.Tensor], vkind: int, op: int, n: int,
             valid: Optional[torch.Tensor] = None, ids2: Optional[torch.Tensor] = None, reverse: bool = False,
             err: Optional[torch.Tensor] = None, device=None) -> torch.Tensor:
    """Segmented inclusive scan in row order (``reverse``: from the end).
    Segments are runs of equal ``ids`` (None: one segment). Values: a column
    (``vals`` int64 / int32 / f64), 1 per row (V_ONE), the row index at heads
    of ``ids2`` (V_HEADIDX) or a 0/1 head flag of ``ids2`` (V_HEAD2). NULL
    rows (``valid`` False) contribute the operator's identity (0 for counts).
    Returns int64, or float64 for the f64 operators. ``err`` (int32 [1]):
    set when an int64 sum overflows."""
    ref = next((t for t in (ids, vals, ids2, valid) if t is not None), None)
    dev = ref.device if ref is not None else torch.device(device or "cpu")
    f64 = op in (SUM_F, MIN_F, MAX_F)
    if n == 0:
        return torch.zeros(0, dtype=torch.float64 if f64 else torch.int64, device=dev)
    if not dev.type == "cuda":
        return _seg_scan_cpu(ids, vals, vkind, op, n, valid, ids2, reverse)
    N = launch("win_seg_scan")
    tiles = N.win_scan_tiles(n)
    tflag = torch.empty(max(tiles, 1), dtype=torch.int32, device=dev)
    tval = torch.empty(max(tiles, 1), dtype=torch.int64, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    if vals is not None and vkind == V_F64:
        vals = vals.to(torch.float64).contiguous().view(torch.int64)
    elif vals is not None:
        vals = vals.contiguous()
    N.win_seg_scan(ptr(ids), ids is not None and ids.dtype == torch.int64, ptr(ids2),
                   ids2 is not None and ids2.dtype == torch.int64, ptr(vals), vkind,
                   ptr(valid.contiguous() if valid is not None else None), n, op, reverse, ptr(tflag), ptr(tval),
                   ptr(out), ptr(err), stream(out))
    return out.view(torch.float64) if f64 else out


def _heads(ids: Optional[torch.Tensor], order: torch.Tensor, n: int) -> torch.Tensor:
    h = torch.zeros(n, dtype=torch.bool)
    h[0] = True
    if ids is not None and n > 1:
        x = ids.to(torch.int64)[order]
        h[1:] = x[1:] != x[:-1]
    return h


def _seg_scan_cpu(ids, vals, vkind, op, n, valid, ids2, reverse) -> torch.Tensor:
    order = torch.arange(n - 1, -1, -1) if reverse else torch.arange(n)
    f64 = op in (SUM_F, MIN_F, MAX_F)
    ident = _identity(op)
    h = _heads(ids, order, n)
    if vkind in (V_I64, V_I32):
        v = vals.to(torch.int64)[order]
    elif vkind == V_F64:
        v = vals.to(torch.float64)[order]
    elif vkind == V_ONE:
        v = torch.ones(n, dtype=torch.int64)
    elif vkind == V_HEADIDX:
        v = torch.where(_heads(ids2, order, n), order, torch.full((n,), ident, dtype=torch.int64))
    else:
        v = _heads(ids2, order, n).to(torch.int64)
    if valid is not None:
        z = 0 if vkind in (V_ONE, V_HEAD2) else ident
        v = torch.where(valid[order], v, torch.full_like(v, z))
    if f64:
        v = v.to(torch.float64)
    # Hillis-Steele segmented scan: (f1,v1)+(f2,v2) = (f1|f2, f2 ? v2 : v1 op v2)
    f = h.clone()
    d = 1
    while d < n:
        a, b = v[:-d], v[d:]
        if op in (SUM_I, SUM_F):
            comb = a + b
        elif op in (MIN_I, MIN_F):
            comb = torch.minimum(a, b)
        else:
            comb = torch.maximum(a, b)
        nv = v.clone()
        nv[d:] = torch.where(f[d:], b, comb)
        nf = f.clone()
        nf[d:] = f[d:] | f[:-d]
        v, f = nv, nf
        d *= 2
    out = torch.empty_like(v)
    out[order] = v
    return out


def bounds(n: int, ss, se, ps, pe, unit: str, skind: str, soff, ekind: str, eoff, key=None, key_valid=None,
           desc: bool = False, gnum=None, gpos=None, ngroups: int = 0, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-row frame [lo, hi] (inclusive row indices; hi < lo = empty).
    ss/se: partition start/end per row (None: the whole input), ps/pe: peer
    group start/end, key: sorted ORDER BY key (int64 or f64) for RANGE
    offsets, gnum/gpos: global peer-group number per row / first row per
    group for GROUPS offsets."""
    ref = next((t for t in (ss, ps, key, gnum) if t is not None), None)
    dev = ref.device if ref is not None else torch.device(device or "cpu")
    key_f64 = key is not None and key.dtype.is_floating_point

    def _i(o):
        return 0 if o is None else int(o)

    def _f(o):
        return 0.0 if o is None else float(o)
    if dev.type == "cuda":
        lo = torch.empty(n, dtype=torch.int64, device=dev)
        hi = torch.empty(n, dtype=torch.int64, device=dev)
        if key is not None:
            key = key.to(torch.float64 if key_f64 else torch.int64).contiguous()
        launch("win_bounds").win_bounds(n, ptr(ss), ptr(se), ptr(ps), ptr(pe), UNIT[unit], FRAME_KIND[skind],
                                        _i(soff) if not key_f64 else 0, _f(soff), FRAME_KIND[ekind],
                                        _i(eoff) if not key_f64 else 0, _f(eoff), ptr(key), key_f64,
                                        ptr(key_valid), desc, ptr(gnum), ptr(gpos), ngroups, ptr(lo), ptr(hi),
                                        stream(lo))
        return lo, hi
    r = torch.arange(n, dtype=torch.int64)
    s0 = ss if ss is not None else torch.zeros(n, dtype=torch.int64)
    e0 = se if se is not None else torch.full((n,), n - 1, dtype=torch.int64)
    lo, hi = s0.clone(), e0.clone()
    sk, ek = FRAME_KIND[skind], FRAME_KIND[ekind]
    if sk == 2:
        lo = r.clone() if unit == "rows" else ps.clone()
    if ek == 2:
        hi = r.clone() if unit == "rows" else pe.clone()
    if unit == "rows":
        if sk == 1:
            lo = r - _i(soff)
        elif sk == 3:
            lo = r + _i(soff)
        if ek == 1:
            hi = r - _i(eoff)
        elif ek == 3:
            hi = r + _i(eoff)
    elif unit == "range" and (sk in (1, 3) or ek in (1, 3)):
        lo, hi = _range_cpu(n, s0, e0, ps, pe, sk, soff, ek, eoff, key, key_valid, desc, lo, hi)
    elif unit == "groups":
        g, g0, g1 = gnum, gnum[s0], gnum[e0]
        gend = torch.where(torch.arange(ngroups) + 1 < ngroups,
                           torch.cat([gpos[1:], gpos.new_tensor([n])]) - 1, torch.full((ngroups,), n - 1))
        if sk == 1:
            gg = g - _i(soff)
            lo = torch.where(gg < g0, s0, gpos[gg.clamp(min=0)])
        elif sk == 3:
            gg = g + _i(soff)
            lo = torch.where(gg > g1, e0 + 1, gpos[gg.clamp(max=ngroups - 1)])
        if ek == 1:
            gg = g - _i(eoff)
            hi = torch.where(gg < g0, s0 - 1, gend[gg.clamp(min=0)])
        elif ek == 3:
            gg = g + _i(eoff)
            hi = torch.where(gg > g1, e0, gend[gg.clamp(max=ngroups - 1)])
    return torch.maximum(lo, s0), torch.minimum(hi, e0)


def _search(key, lo, hi, t, desc, upper):
    """Vectorised binary search of every row's target inside [lo, hi]
    (the kernel's lower_idx / upper_idx)."""
    a, b = lo.clone(), hi + 1
    n = key.numel()
    for _ in range(64):
        act = a < b
        if not bool(act.any()):
            break
        m = a + ((b - a) >> 1)
        km = key[m.clamp(0, max(n - 1, 0))]
        if upper:
            go_right = (km >= t) if desc else (km <= t)
        else:
            go_right = (km > t) if desc else (km < t)
        a = torch.where(act & go_right, m + 1, a)
        b = torch.where(act & ~go_right, m, b)
    return a - 1 if upper else a


def _range_cpu(n, s0, e0, ps, pe, sk, soff, ek, eoff, key, key_valid, desc, lo, hi):
    f64 = key.dtype.is_floating_point
    k = key.to(torch.float64 if f64 else torch.int64)
    nb, ne = s0.clone(), e0.clone()
    if key_valid is not None:
        kv = key_valid
        nb = torch.where(~kv[s0], pe[s0] + 1, nb)
        ne = torch.where(~kv[e0], ps[e0] - 1, ne)

    def shift(forward, off):
        up = forward != desc
        o = float(off) if f64 else int(off)
        return k + o if up else k - o
    if sk == 1:
        lo = _search(k, nb, ne, shift(False, soff), desc, False)
    elif sk == 3:
        lo = _search(k, nb, ne, shift(True, soff), desc, False)
    if ek == 1:
        hi = _search(k, nb, ne, shift(False, eoff), desc, True)
    elif ek == 3:
        hi = _search(k, nb, ne, shift(True, eoff), desc, True)
    if key_valid is not None:
        nul = ~key_valid
        if sk != 0:
            lo = torch.where(nul, ps, lo)
        if ek != 4:
            hi = torch.where(nul, pe, hi)
    return lo, hi


def frame_sum(psum: Optional[torch.Tensor], pcnt: Optional[torch.Tensor], lo, hi, n: int):
    """Framed sum and count from inclusive global prefixes (sum: int64
    wrapping or f64)."""
    if n == 0 or not lo.is_cuda:
        empty = hi < lo
        li = (lo - 1).clamp(min=0)

        def diff(p):
            if p is None:
                return None
            z = torch.zeros((), dtype=p.dtype)
            before = torch.where(lo > 0, p[li] if n else p[:0], z)
            return torch.where(empty, z, p[hi.clamp(min=0)] - before) if n else p[:0]
        return diff(psum), diff(pcnt)
    f64 = psum is not None and psum.dtype == torch.float64
    so = torch.empty(n, dtype=torch.int64, device=lo.device) if psum is not None else None
    co = torch.empty(n, dtype=torch.int64, device=lo.device) if pcnt is not None else None
    launch("win_frame_sum").win_frame_sum(ptr(psum.view(torch.int64) if f64 else psum), f64, ptr(pcnt), ptr(lo),
                                          ptr(hi), n, ptr(so), ptr(co), stream(lo))
    return (so.view(torch.float64) if f64 else so), co


#: frames at most this wide loop over their rows; wider ones use a sparse table
LOOP_MAX_WIDTH = 32


def frame_minmax(vals: torch.Tensor, valid: Optional[torch.Tensor], lo, hi, n: int, is_max: bool):
    """min / max over each row's frame [lo, hi] -> (values, valid). Narrow
    frames: a loop over the frame; wider ones: a sparse table of
    ceil(log2(width)) levels (one pass each) and two reads per row, so a
    ``ROWS BETWEEN 100000 PRECEDING`` frame costs O(n log w), not O(n w)."""
    f64 = vals.dtype.is_floating_point
    if n == 0:
        return torch.zeros(0, dtype=torch.float64 if f64 else torch.int64, device=lo.device), \
            torch.zeros(0, dtype=torch.bool, device=lo.device)
    widest = to_host_int((hi - lo).max()) + 1
    v = vals.to(torch.float64 if f64 else torch.int64).contiguous()
    if lo.is_cuda and widest <= LOOP_MAX_WIDTH:
        out = torch.empty(n, dtype=torch.int64, device=lo.device)
        ov = torch.empty(n, dtype=torch.bool, device=lo.device)
        launch("win_frame_minmax").win_frame_minmax(ptr(v.view(torch.int64) if f64 else v), f64, is_max,
                                                    ptr(valid), ptr(lo), ptr(hi), n, ptr(out), ptr(ov), stream(out))
        return (out.view(torch.float64) if f64 else out), ov
    levels = max(1, widest.bit_length())
    pcnt = None
    if valid is not None:
        pcnt = torch.cumsum(valid.to(torch.int64), 0)
    if lo.is_cuda:
        table = torch.empty((levels, n), dtype=torch.int64, device=lo.device)
        out = torch.empty(n, dtype=torch.int64, device=lo.device)
        ov = torch.empty(n, dtype=torch.bool, device=lo.device)
        st = stream(out)
        N = launch("win_sparse")
        N.win_sparse_build(ptr(v.view(torch.int64) if f64 else v), f64, ptr(valid), n, is_max, levels, ptr(table), st)
        N.win_sparse_query(ptr(table), levels, n, ptr(lo.contiguous()), ptr(hi.contiguous()), ptr(pcnt), is_max,
                           f64, ptr(out), ptr(ov), st)
        del table
        return (out.view(torch.float64) if f64 else out), ov
    # host: the same sparse table with torch ops
    ident = float("-inf") if (is_max and f64) else float("inf") if f64 else (-(2**63) if is_max else 2**63 - 1)
    cur = v.clone()
    if valid is not None:
        cur = torch.where(valid, cur, torch.full_like(cur, ident))
    tabs = [cur]
    for k in range(1, levels):
        half = 1 << (k - 1)
        prev = tabs[-1]
        nxt = prev.clone()
        if half < n:
            nxt[:n - half] = torch.maximum(prev[:n - half], prev[half:]) if is_max else \
                torch.minimum(prev[:n - half], prev[half:])
        tabs.append(nxt)
    table = torch.stack(tabs)
    ok = hi >= lo
    w = (hi - lo + 1).clamp(min=1)
    k = torch.floor(torch.log2(w.to(torch.float64))).to(torch.int64).clamp(max=levels - 1)
    lo_c = lo.clamp(0, n - 1)
    hi2 = (hi - (1 << k) + 1).clamp(0, n - 1)
    a = table[k, lo_c]
    b = table[k, hi2]
    out = torch.maximum(a, b) if is_max else torch.minimum(a, b)
    if pcnt is not None:
        cnt = pcnt[hi.clamp(0, n - 1)] - torch.where(lo > 0, pcnt[(lo - 1).clamp(min=0)], torch.zeros_like(lo))
        ok = ok & (cnt > 0)
    out = torch.where(ok, out, torch.zeros_like(out))
    return out, ok


def rank(fn: int, arg: int, n: int, ss, se, ps, pe, dense, device) -> torch.Tensor:
    """Ranking functions (int64; percent_rank / cume_dist f64)."""
    f64 = fn in (PERCENT_RANK, CUME_DIST)
    if n and torch.device(device).type == "cuda":
        out = torch.empty(n, dtype=torch.int64, device=device)
        launch("win_rank").win_rank(fn, arg, n, ptr(ss), ptr(se), ptr(ps), ptr(pe), ptr(dense), ptr(out),
                                    stream(out))
        return out.view(torch.float64) if f64 else out
    r = torch.arange(n, dtype=torch.int64)
    s0 = ss if ss is not None else torch.zeros(n, dtype=torch.int64)
    e0 = se if se is not None else torch.full((n,), n - 1, dtype=torch.int64)
    size = e0 - s0 + 1
    p0 = ps if ps is not None else s0
    if fn == ROW_NUMBER:
        return r - s0 + 1
    if fn == RANK:
        return p0 - s0 + 1
    if fn == DENSE_RANK:
        return dense
    if fn == PERCENT_RANK:
        return torch.where(size > 1, (p0 - s0).double() / (size - 1).clamp(min=1).double(),
                           torch.zeros(n, dtype=torch.float64))
    if fn == CUME_DIST:
        p1 = pe if pe is not None else e0
        return (p1 - s0 + 1).double() / size.double()
    j = r - s0
    q = torch.div(size, arg, rounding_mode="floor")
    rem = size - q * arg
    big = rem * (q + 1)
    qs = q.clamp(min=1)
    return torch.where(q == 0, j + 1, torch.where(j < big, torch.div(j, q + 1, rounding_mode="floor") + 1,
                                                  torch.div(j - big, qs, rounding_mode="floor") + rem + 1))


def index(fn: int, arg: int, n: int, ss, se, lo, hi, device) -> torch.Tensor:
    """Source row of lag/lead (LAG with +-k), first/last/nth_value; -1 = none."""
    if n and torch.device(device).type == "cuda":
        out = torch.empty(n, dtype=torch.int64, device=device)
        launch("win_index").win_index(fn, arg, n, ptr(ss), ptr(se), ptr(lo), ptr(hi), ptr(out), stream(out))
        return out
    r = torch.arange(n, dtype=torch.int64)
    neg = torch.full((n,), -1, dtype=torch.int64)
    if fn == LAG:
        s0 = ss if ss is not None else torch.zeros(n, dtype=torch.int64)
        e0 = se if se is not None else torch.full((n,), n - 1, dtype=torch.int64)
        j = r - arg
        return torch.where((j >= s0) & (j <= e0), j, neg)
    ok = lo <= hi
    if fn == FIRST:
        return torch.where(ok, lo, neg)
    if fn == LAST:
        return torch.where(ok, hi, neg)
    j = lo + arg - 1
    return torch.where(ok & (j <= hi), j, neg)
