"""Sorting: multi-column argsort, top-k and secondary-index builds on the
hand-written radix sort (csrc/kernels/sort.hip).

ORDER BY keys are packed on the device into ONE order-preserving unsigned key
per row (``sort_key_pack``): each column contributes a field of
``bitlen(max - min)`` bits (DESC flips it inside its span, a nullable column
adds a NULL-order bit above it), so e.g. (l_returnflag, l_linestatus) packs
into 3 bits and sorts in one 8-bit pass. Column sets wider than 64 bits are
split into groups sorted least-significant group first (stable LSD). The
sort carries the row id as its value, so the result is a permutation.

``topk`` (ORDER BY ... LIMIT k) radix-selects first: histograms of the top
key digits (refined within the boundary bucket while it is large) find a
bound admitting k rows plus the boundary bucket's ties; only those candidates
are sorted. Ties resolve by row id exactly as the stable full sort does.

CPU tensors use torch's stable sort (reference implementation for tests).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence, Tuple

import torch

from ._lib import is_gpu, launch, ptr, stream, to_host_ints
from .select import mask_to_indices

#: ORDER BY column: (values, descending, nulls_first, validity or None)
SortKey = Tuple[torch.Tensor, bool, bool, Optional[torch.Tensor]]

_KIND = {torch.int8: (0, 1), torch.int16: (0, 2), torch.int32: (0, 4), torch.int64: (0, 8),
         torch.float64: (1, 8), torch.uint8: (2, 1), torch.bool: (2, 1), torch.float32: (3, 4)}
U64 = (1 << 64) - 1
#: integer key dtypes and their full value ranges (sort keys without a bound)
_FULL = {torch.int8: (-(1 << 7), (1 << 7) - 1), torch.int16: (-(1 << 15), (1 << 15) - 1),
         torch.int32: (-(1 << 31), (1 << 31) - 1), torch.int64: (-(1 << 63), (1 << 63) - 1),
         torch.uint8: (0, 255), torch.bool: (0, 1)}
#: inputs up to this many rows sort in one workgroup (sort.hip kRsTile)
SMALL_SORT = 4096


def _ordered_f64(x: float) -> int:
    if x == 0.0:
        x = 0.0
    b = struct.unpack("<Q", struct.pack("<d", x))[0]
    return (~b & U64) if b >> 63 else (b | (1 << 63))


def _ordered_f32(x: float) -> int:
    if x == 0.0:
        x = 0.0
    b = struct.unpack("<I", struct.pack("<f", x))[0]
    return (~b & 0xFFFFFFFF) if b >> 31 else (b | (1 << 31))


def _fields(keys: Sequence[SortKey]) -> List[tuple]:
    """Per column: (tensor, valid, lo, span, kind, width, bits, desc, nulls_first). One host sync for all bounds."""
    from .hashing import key_bound
    known = []
    for v, _desc, _nf, valid in keys:
        b = key_bound(v) if valid is None and v.numel() and is_gpu(v) and v.dtype in (torch.int32, torch.int64) \
            else None
        if b is None and v.numel():
            break
        known.extend(b if b is not None else (0, 0))
    else:
        # every key has a readback-free bound (resident origin, dictionary
        # codes, group ids): a wider field than the exact range, same order
        return _fields_from(keys, known)
    if all(v.numel() <= SMALL_SORT and is_gpu(v) and v.dtype in _FULL and (valid is None or v.dtype != torch.int64)
           for v, _desc, _nf, valid in keys):
        # a small sort (one workgroup) over integer keys: full-width fields
        # cost a few more digit passes inside one kernel, far less than the
        # host sync that would read the exact ranges (ORDER BY of a result)
        return _fields_from(keys, [x for v, _d, _n, _v in keys for x in _FULL[v.dtype]])
    stats = []
    for v, _desc, _nf, _valid in keys:
        if v.numel() == 0:
            stats.append(torch.zeros(2, dtype=torch.int64, device=v.device))
            continue
        x = v.to(torch.uint8) if v.dtype == torch.bool else v
        if is_gpu(x) and x.dtype in (torch.int32, torch.int64):
            # bounds from the hand-written two-stage reduction (util.hip): the
            # ATen aminmax zeroes its multi-block semaphores with a memset that
            # does not replay inside a HIP graph, so the query never graphed
            stats.append(_int_bounds(x))
            continue
        mn, mx = torch.aminmax(x)
        if x.dtype in (torch.float64, torch.float32):
            stats.append(torch.stack([mn.to(torch.float64), mx.to(torch.float64)]).view(torch.int64))
        else:
            stats.append(torch.stack([mn.to(torch.int64), mx.to(torch.int64)]))
    vals = to_host_ints(torch.cat(stats)) if stats else []
    return _fields_from(keys, vals)


def _fields_from(keys: Sequence[SortKey], vals: Sequence[int]) -> List[tuple]:
    out = []
    for i, (v, desc, nf, valid) in enumerate(keys):
        if v.dtype not in _KIND:
            raise TypeError(f"sort key dtype {v.dtype}")
        kind, width = _KIND[v.dtype]
        a, b = vals[2 * i], vals[2 * i + 1]
        if kind == 0:
            lo, hi = a + (1 << 63), b + (1 << 63)
        elif kind == 2:
            lo, hi = a, b
        else:
            fa, fb = struct.unpack("<2d", struct.pack("<2q", a, b))
            enc = _ordered_f64 if kind == 1 else _ordered_f32
            lo, hi = enc(fa), enc(fb)
        if v.numel() == 0:
            lo = hi = 0
        span = max(hi - lo, 0)
        bits = span.bit_length()
        t = v if v.dtype != torch.bool else v.view(torch.uint8)
        out.append((t.contiguous(), None if valid is None else valid.contiguous(), lo & U64, span, kind, width,
                    bits, int(desc), int(nf)))
    return out


def _int_bounds(x: torch.Tensor) -> torch.Tensor:
    """int64 [min, max] of an int32/int64 device column (no host sync)."""
    N = launch("column_stats")
    buf = torch.empty(N.STATS_SLOTS, dtype=torch.int64, device=x.device)
    x = x.contiguous()
    N.column_stats(ptr(x), x.dtype == torch.int64, 0, x.numel(), ptr(buf), stream(x))
    return buf[:2]


def _groups(fields: List[tuple]) -> List[List[tuple]]:
    """Split columns (most significant first) into runs of <= 64 key bits."""
    groups, cur, used = [], [], 0
    for f in fields:
        w = f[6] + (1 if f[1] is not None else 0)
        if cur and used + w > 64:
            groups.append(cur)
            cur, used = [], 0
        cur.append(f)
        used += w
    if cur:
        groups.append(cur)
    return groups


def _pack(group: List[tuple], n: int, perm: Optional[torch.Tensor], device) -> Tuple[torch.Tensor, int]:
    bits = sum(f[6] + (1 if f[1] is not None else 0) for f in group)
    out32 = bits <= 32
    keys = torch.empty(n, dtype=torch.int32 if out32 else torch.int64, device=device)
    cols = [(ptr(t), ptr(valid), lo, span, kind, width, b, desc, nf)
            for (t, valid, lo, span, kind, width, b, desc, nf) in group]
    launch("sort_key_pack").sort_key_pack(cols, ptr(perm), perm is not None and perm.dtype == torch.int64, n,
                                          ptr(keys), out32, stream(keys))
    return keys, bits


def sort_pairs(keys: torch.Tensor, vals: torch.Tensor, end_bit: int, begin_bit: int = 0,
               consume: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable sort of (key, value) pairs by key bits [begin_bit, end_bit);
    keys are int32/int64 tensors holding unsigned values. Returns new tensors
    (``consume``: the caller's contiguous, distinct inputs may serve as the
    sort's first buffers -- their contents are then undefined -- instead of
    being copied)."""
    n = keys.numel()
    if not is_gpu(keys):
        k = keys.to(torch.int64)
        if keys.dtype == torch.int32:
            k = k & 0xFFFFFFFF
        else:  # unsigned 64-bit order on a signed tensor: flip the sign bit
            k = k ^ torch.tensor(-(1 << 63), dtype=torch.int64)
        o = torch.sort(k, stable=True).indices
        return keys.index_select(0, o), vals.index_select(0, o)
    own = consume and keys.is_contiguous() and vals.is_contiguous() and keys.data_ptr() != vals.data_ptr()
    k0 = keys if own else keys.contiguous().clone()
    v0 = vals if own else vals.contiguous().clone()
    if n <= 1 or end_bit <= begin_bit:
        return k0, v0
    N = launch("radix_sort")
    if n <= SMALL_SORT:
        N.radix_sort_pairs(ptr(k0), 0, k0.dtype == torch.int64, ptr(v0), 0, v0.dtype == torch.int64, n, begin_bit,
                           end_bit, 0, stream(k0))
        return k0, v0
    k1 = torch.empty_like(k0)
    v1 = torch.empty_like(v0)
    ws = torch.empty(N.radix_sort_ws_bytes(n), dtype=torch.uint8, device=keys.device)
    which = N.radix_sort_pairs(ptr(k0), ptr(k1), k0.dtype == torch.int64, ptr(v0), ptr(v1),
                               v0.dtype == torch.int64, n, begin_bit, end_bit, ptr(ws), stream(k0))
    return (k1, v1) if which else (k0, v0)


def _row_ids(n: int, device) -> torch.Tensor:
    return torch.arange(n, dtype=torch.int32 if n < 2**31 - 1 else torch.int64, device=device)


def argsort(keys: Sequence[SortKey], n: int, device) -> torch.Tensor:
    """Stable lexicographic argsort over ORDER BY keys (int32/int64 permutation)."""
    device = torch.device(device)
    if n <= 1:
        return _row_ids(n, device)
    if device.type != "cuda":
        return _argsort_cpu(keys, n, device)
    groups = _groups(_fields(keys))
    perm = None
    for g in reversed(groups):          # least significant group first
        k, bits = _pack(g, n, perm, device)
        vals = perm if perm is not None else _row_ids(n, device)
        _, perm = sort_pairs(k, vals, bits)
    return perm


def topk(keys: Sequence[SortKey], n: int, k: int, device) -> torch.Tensor:
    """Row ids of the first ``k`` rows in ORDER BY order (same rows and order
    as ``argsort(...)[:k]``)."""
    device = torch.device(device)
    k = max(0, min(k, n))
    if device.type != "cuda" or n <= max(SMALL_SORT, 4 * k):
        return argsort(keys, n, device)[:k]
    fields = _fields(keys)
    groups = _groups(fields)
    lead, bits = _pack(groups[0], n, None, device)
    cand = _select_candidates(lead, bits, k)
    if cand is None:
        return argsort(keys, n, device)[:k]
    # sort only the candidates (their row ids carried as the permutation)
    m = cand.numel()
    perm = None
    for gi in range(len(groups) - 1, -1, -1):
        src = cand if perm is None else perm
        kk, b = _pack(groups[gi], m, src, device)
        _, perm = sort_pairs(kk, src, b)
    return perm[:k]


def topk_candidates(keys: Sequence[SortKey], n: int, k: int) -> Optional[torch.Tensor]:
    """Row ids (row order) of a superset of the first ``k`` rows under an
    ordering whose LEADING keys are ``keys`` (ties at the boundary kept), or
    None when it would not shrink the input. Lets the caller evaluate costly
    tie-breakers (string ranks) for a handful of rows only."""
    if n <= max(SMALL_SORT, 4 * k) or not keys or not is_gpu(keys[0][0]):
        return None
    groups = _groups(_fields(keys))
    lead, bits = _pack(groups[0], n, None, keys[0][0].device)
    return _select_candidates(lead, bits, max(k, 1))


def _select_candidates(keys: torch.Tensor, bits: int, k: int) -> Optional[torch.Tensor]:
    """Indices (in row order) of every row whose key is <= a digit-prefix bound
    admitting the k smallest keys (the boundary bucket's rows included); None
    when the bound would not shrink the input."""
    n = keys.numel()
    if bits == 0:
        return None
    N = launch("radix_select")
    k64 = keys.dtype == torch.int64
    st = stream(keys)
    limit = max(8 * k, 1 << 16)
    pshift, prefix = bits, 0        # rows in play: (key >> pshift) == prefix (all rows: keys < 2^bits)
    shift = max(bits - 8, 0)
    below = 0                       # rows known to rank before the bucket in play
    while True:
        hist = torch.empty(256, dtype=torch.int64, device=keys.device)   # fresh per pass: its readback may be replayed
        N.radix_digit_hist(ptr(keys), k64, n, shift, prefix, pshift, ptr(hist), st)
        counts = to_host_ints(hist)
        run, digit = below, 255
        for d, c in enumerate(counts):
            if run + c >= k:
                digit = d
                break
            run += c
        width = pshift - shift
        prefix = (prefix << width) | (digit & ((1 << width) - 1))
        pshift = shift
        below, in_bucket = run, counts[digit]
        if below + in_bucket <= limit or shift == 0:
            break
        shift = max(shift - 8, 0)
    if below + in_bucket >= n:
        return None
    bound = (((prefix + 1) << pshift) - 1) & U64
    mask = torch.empty(n, dtype=torch.bool, device=keys.device)
    N.radix_le_mask(ptr(keys), k64, n, bound, ptr(mask), st)
    return mask_to_indices(mask)


def perm_sort_int(keys: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(keys sorted, int32/int64 row permutation) of a non-null int32/int64
    column — the secondary index of a resident key column. Non-negative keys
    sort on their raw low bits (ceil(bitlen(max) / 8) passes)."""
    n = keys.numel()
    if n == 0 or not is_gpu(keys):
        sk, perm = torch.sort(keys, stable=True)
        return sk, perm.to(torch.int32 if n < 2**31 - 1 else torch.int64)
    mn, mx = to_host_ints(torch.stack(list(torch.aminmax(keys))).to(torch.int64))
    rows = _row_ids(n, keys.device)
    if mn >= 0:
        return sort_pairs(keys, rows, max(int(mx).bit_length(), 1))
    perm = argsort([(keys, False, False, None)], n, keys.device)
    return keys.index_select(0, perm.long()), perm


def _argsort_cpu(keys: Sequence[SortKey], n: int, device) -> torch.Tensor:
    perm = torch.arange(n, dtype=torch.int64, device=device)
    for vals, desc, nulls_first, valid in reversed(list(keys)):
        v = vals.index_select(0, perm)
        if v.dtype == torch.bool:
            v = v.to(torch.int8)
        if valid is not None:   # NULLs tie with each other (as on the GPU)
            v = torch.where(valid.index_select(0, perm), v, torch.zeros_like(v))
        o = torch.sort(v, stable=True, descending=desc).indices
        perm = perm.index_select(0, o)
        if valid is not None:
            vv = valid.index_select(0, perm)
            o2 = torch.sort(vv.to(torch.int8), stable=True, descending=not nulls_first).indices
            perm = perm.index_select(0, o2)
    return perm
