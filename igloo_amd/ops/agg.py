"""Grouped aggregation (csrc/kernels/agg.hip).

``grouped_aggregate`` updates up to 8 aggregate states per launch from one
pass over the group ids. Integer SUMs are exact 128-bit; the result comes
back as int64 when every group fits, else as an [g, 2] (lo, hi) tensor.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch

from ..utils import switches as _sw
from ._lib import is_gpu, launch, native, ptr, stream, to_host_ints

OPS = {"sum_int": 0, "sum_f64": 1, "count": 2, "min_int": 3, "max_int": 4, "min_f64": 5, "max_f64": 6,
       "and_int": 7, "or_int": 8, "xor_int": 9}
_INT_OPS = ("sum_int", "min_int", "max_int", "and_int", "or_int", "xor_int")
I64_MAX = 2**63 - 1
I64_MIN = -(2**63)

Spec = Tuple[str, Optional[torch.Tensor], Optional[torch.Tensor]]  # (op, values, valid)


def _ordered_to_f64(x: torch.Tensor) -> torch.Tensor:
    mask = (x >> 63) & 0x7FFFFFFFFFFFFFFF
    return (x ^ mask).view(torch.float64)


def _wide_flags(pairs) -> torch.Tensor:
    """int32 [len(pairs)]: 1 where some (lo, hi) sum of the pair does not fit
    int64 (one hand-written pass per pair, no torch reduction)."""
    dev = pairs[0][0].device
    flags = torch.empty(len(pairs), dtype=torch.int32, device=dev)
    N = launch("wide_fits")
    for i, (lo, hi) in enumerate(pairs):
        lo, hi = lo.contiguous(), hi.contiguous()
        N.wide_fits(ptr(lo), ptr(hi), lo.numel(), ptr(flags) + 4 * i, stream(lo))
    return flags


def _wide_to_result(lo: torch.Tensor, hi: torch.Tensor) -> torch.Tensor:
    if lo.is_cuda:
        fits = not to_host_ints(_wide_flags([(lo, hi)]))[0]
    else:
        fits = bool((hi == (lo >> 63)).all().item())
    if fits:
        return lo
    return torch.stack([lo, hi], dim=1)


def grouped_aggregate(gid: Optional[torch.Tensor], ngroups: int, specs: Sequence[Spec], n: int,
                      device, sorted_gids: bool = False) -> List[torch.Tensor]:
    """``sorted_gids``: group ids are non-decreasing (clustered keys) — the GPU
    then folds runs in registers instead of issuing one atomic per row."""
    device = torch.device(device)
    if device.type != "cpu":
        return _gpu(gid, ngroups, specs, n, device, sorted_gids)
    return _cpu(gid, ngroups, specs, n)


def _sum_fits(vals: Optional[torch.Tensor], n: int) -> bool:
    """Every partial and total SUM of these ``n`` values fits in int64, by a
    bound known without a readback (ops/hashing.py key_bound: the range of
    the resident column they were gathered from)."""
    if vals is None or vals.dim() != 1:
        return False
    from .hashing import key_bound
    b = key_bound(vals)
    return b is not None and n * max(abs(b[0]), abs(b[1])) < 2**62


def _narrow_sums(specs, n) -> set:
    """Indices of the integer SUM specs that accumulate in one int64 word (no
    carry word, half the atomics, no "fits" pass afterwards): int32 values,
    whose exact total over fewer than 2^31 rows provably fits. (int64 values
    would need a bounds pass and a host sync to decide: measured no gain,
    profiles/r3_ab_narrow_sums.txt, so they keep the 128-bit state.)"""
    if n == 0 or n >= 2**31:
        return set()
    return {i for i, (op, vals, _valid) in enumerate(specs)
            if op == "sum_int" and vals is not None and vals.dtype == torch.int32}


def _gpu(gid, ngroups, specs, n, device, sorted_gids=False) -> List[torch.Tensor]:
    N = native()
    g = max(ngroups, 1)
    outs, descs, posts = [], [], []
    narrow = _narrow_sums(specs, n)
    # every zero-initialised state of the call (sums, their carry words,
    # counts) in ONE zeroed buffer: one fill kernel instead of one per state
    # (slots padded to 512 bytes, the alignment of a fresh allocation)
    nz = sum((2 if op == "sum_int" and si not in narrow else 1) if op in ("sum_int", "sum_f64", "count") else 0
             for si, (op, _v, _m) in enumerate(specs))
    slot = -(-g // 64) * 64
    zbuf = torch.zeros(nz * slot, dtype=torch.int64, device=device) if nz else None
    zi = 0

    def zeros(dt=torch.int64):
        nonlocal zi
        z = zbuf[zi * slot: zi * slot + g]
        zi += 1
        return z.view(dt) if dt != torch.int64 else z
    for si, (op, vals, valid) in enumerate(specs):
        code = OPS[op]
        dst2 = None
        if op in ("sum_int", "sum_f64", "count"):
            dst = zeros(torch.float64 if op == "sum_f64" else torch.int64)
            if op == "sum_int" and si not in narrow:
                dst2 = zeros()
        elif op.startswith("min"):
            dst = torch.full((g,), I64_MAX, dtype=torch.int64, device=device)
        elif op in ("and_int", "or_int", "xor_int"):
            dst = torch.full((g,), -1 if op == "and_int" else 0, dtype=torch.int64, device=device)
        else:
            dst = torch.full((g,), I64_MIN, dtype=torch.int64, device=device)
        src64 = 1
        if vals is not None:
            assert vals.numel() == n and vals.is_contiguous()
            if op in _INT_OPS:
                assert vals.dtype in (torch.int32, torch.int64), vals.dtype
                src64 = 1 if vals.dtype == torch.int64 else 0
            else:
                assert vals.dtype == torch.float64 or op == "count"
        descs.append((code, src64, ptr(vals), ptr(valid), ptr(dst), ptr(dst2)))
        posts.append((op, dst, dst2))
    if n > 0:
        s = stream(gid if gid is not None else posts[0][1])
        for i in range(0, len(descs), 8):
            chunk = descs[i:i + 8]
            if gid is not None and not sorted_gids and _partitioned_ok(n, ngroups, len(chunk)):
                _agg_partitioned(gid, n, ngroups, chunk, specs[i:i + 8], s)
                continue
            launch("agg_update")
            N.agg_update(ptr(gid), n, ngroups if gid is not None else 1, chunk, s, bool(sorted_gids))
    # one host sync for every 128-bit integer SUM's "fits in int64" check
    # (none for a SUM whose input has a readback-free bound proving it fits)
    known = {si for si, (op, vals, _v) in enumerate(specs) if op == "sum_int" and posts[si][2] is not None
             and _sum_fits(vals, n)}
    wide = [(dst, dst2) for si, (op, dst, dst2) in enumerate(posts)
            if op == "sum_int" and dst2 is not None and si not in known]
    fits = [1 - f for f in to_host_ints(_wide_flags(wide))] if wide else []
    fit_iter = iter(fits)
    for si, (op, dst, dst2) in enumerate(posts):
        if op == "sum_int":
            ok = dst2 is None or si in known or next(fit_iter)
            outs.append(dst if ok else torch.stack([dst, dst2], dim=1))
        elif op in ("min_f64", "max_f64"):
            # empty groups keep the int64 sentinel: report +/-inf like the CPU path
            sentinel = I64_MAX if op == "min_f64" else I64_MIN
            inf = float("inf") if op == "min_f64" else float("-inf")
            outs.append(torch.where(dst == sentinel, torch.full_like(dst, 0).double() + inf, _ordered_to_f64(dst)))
        else:
            outs.append(dst)
    return outs


#: radix-partitioned aggregation (csrc/kernels/agg.hip agg_partitioned) for
#: unclustered group ids past the LDS kernel's group count: from this many rows,
#: at least AGG_PART_MIN_RATIO rows per group and AGG_PART_MIN_BUCKETS buckets.
#: Few buckets are shared by several LDS workgroups each (slices merged with
#: atomics): TPC-H Q16's 27,840 groups make 7 buckets -- one workgroup per
#: bucket ran 0.5 ms slower than the atomics. IGLOO_DEBUG=no_agg_part: off
AGG_PARTITIONED = not _sw.debug("no_agg_part")
AGG_PART_MIN_ROWS = 1 << 21
AGG_PART_MIN_RATIO = 2
AGG_PART_MIN_BUCKETS = 1 if not _sw.debug("agg_part_min128") else 128


def _partitioned_ok(n: int, ngroups: int, nagg: int) -> bool:
    if not (AGG_PARTITIONED and AGG_PART_MIN_ROWS <= n < 2**31 - 1 and ngroups < 2**31 - 1
            and n >= AGG_PART_MIN_RATIO * ngroups):
        return False
    N = native()
    return ngroups > N.agg_lds_max_groups(nagg) and N.agg_part_buckets(ngroups, nagg) >= AGG_PART_MIN_BUCKETS


def _agg_partitioned(gid: torch.Tensor, n: int, ngroups: int, descs, specs, s) -> None:
    """Rows bucketed by their high group-id bits, each bucket aggregated in
    LDS by one workgroup: no global atomics (one memory-side request per row
    and aggregate otherwise). No host synchronisation."""
    from .select import exclusive_scan
    N = launch("agg_partitioned")
    dev = gid.device
    gid = gid.contiguous()
    nbk, nblk = N.agg_part_buckets(ngroups, len(descs)), N.agg_part_blocks()
    cnt = torch.empty(nbk * nblk, dtype=torch.int32, device=dev)
    N.agg_partitioned(ptr(gid), n, ngroups, descs, 0, ptr(cnt), 0, 0, 0, [0] * len(descs), s)
    off, total = exclusive_scan(cnt, host_total=False)
    pg = torch.empty(n, dtype=torch.int16, device=dev)
    bufs = [None if (op == "count" and valid is None) else torch.empty(n, dtype=torch.int64, device=dev)
            for op, _vals, valid in specs]
    vp = [ptr(b) for b in bufs]
    N.agg_partitioned(ptr(gid), n, ngroups, descs, 1, 0, ptr(off), 0, ptr(pg), vp, s)
    N.agg_partitioned(ptr(gid), n, ngroups, descs, 2, 0, ptr(off), ptr(total), ptr(pg), vp, s)


def _cpu(gid, ngroups, specs, n) -> List[torch.Tensor]:
    g = max(ngroups, 1)
    if gid is None:
        gi = torch.zeros(n, dtype=torch.int64)
    else:
        gi = gid.to(torch.int64)
    outs = []
    for op, vals, valid in specs:
        idx = gi
        v = vals
        if valid is not None:
            sel = valid
            idx = gi[sel]
            v = vals[sel] if vals is not None else None
        if op == "count":
            outs.append(torch.bincount(idx, minlength=g)[:g].to(torch.int64) if idx.numel() else torch.zeros(g, dtype=torch.int64))
        elif op == "sum_f64":
            outs.append(torch.zeros(g, dtype=torch.float64).index_add_(0, idx, v.to(torch.float64)))
        elif op == "sum_int":
            v64 = v.to(torch.int64)
            hi32 = v64 >> 32
            lo32 = v64 & 0xFFFFFFFF
            hs = torch.zeros(g, dtype=torch.int64).index_add_(0, idx, hi32)
            ls = torch.zeros(g, dtype=torch.int64).index_add_(0, idx, lo32)
            approx = hs.to(torch.float64) * 4294967296.0 + ls.to(torch.float64)
            if bool((approx.abs() < 2.0**62).all().item()):
                outs.append((hs << 32) + ls)
            else:
                tot = [int(h) * 4294967296 + int(l) for h, l in zip(hs.tolist(), ls.tolist())]
                lo = torch.tensor([((t + 2**64) % 2**64) - (2**64 if ((t + 2**64) % 2**64) >= 2**63 else 0) for t in tot], dtype=torch.int64)
                hi = torch.tensor([t >> 64 for t in tot], dtype=torch.int64)
                outs.append(_wide_to_result(lo, hi))
        elif op in ("min_int", "max_int"):
            init = I64_MAX if op == "min_int" else I64_MIN
            base = torch.full((g,), init, dtype=torch.int64)
            outs.append(base.scatter_reduce(0, idx, v.to(torch.int64), reduce="amin" if op == "min_int" else "amax"))
        elif op in ("min_f64", "max_f64"):
            init = float("inf") if op == "min_f64" else float("-inf")
            base = torch.full((g,), init, dtype=torch.float64)
            outs.append(base.scatter_reduce(0, idx, v.to(torch.float64), reduce="amin" if op == "min_f64" else "amax"))
        elif op in ("and_int", "or_int", "xor_int"):
            import numpy as np
            ufn = {"and_int": np.bitwise_and, "or_int": np.bitwise_or, "xor_int": np.bitwise_xor}[op]
            res = np.full(g, -1 if op == "and_int" else 0, dtype=np.int64)
            if idx.numel():
                order = torch.argsort(idx, stable=True)
                gi_s = idx[order].numpy()
                vs = v.to(torch.int64)[order].numpy()
                starts = np.flatnonzero(np.r_[True, gi_s[1:] != gi_s[:-1]])
                res[gi_s[starts]] = ufn.reduceat(vs, starts)
            outs.append(torch.from_numpy(res))
        else:
            raise ValueError(op)
    return outs


def wide_to_python(t: torch.Tensor) -> List[int]:
    """[g] int64 or [g, 2] (lo, hi) -> Python ints."""
    t = t.cpu()
    if t.dim() == 1:
        return [int(x) for x in t.tolist()]
    out = []
    for lo, hi in t.tolist():
        out.append((hi << 64) + (lo & 0xFFFFFFFFFFFFFFFF))
    return out


def key_histogram(keys: torch.Tensor, kmin: int, span: int, valid: Optional[torch.Tensor] = None,
                  sparse: bool = False) -> torch.Tensor:
    """int64 counts[span]: rows per key value kmin + i (NULL / out-of-domain keys skipped).
    GPU: 32-bit atomics straight from the key column (csrc/kernels/agg.hip).
    ``sparse``: few rows are valid -- always the direct atomic kernel (the
    radix-partitioned one pays its fixed passes for the many)."""
    if keys.device.type == "cpu" or keys.numel() >= 2**31:   # (int32 counters)
        k = keys.to(torch.int64) - kmin
        ok = (k >= 0) & (k < span)
        if valid is not None:
            ok &= valid
        return torch.bincount(k[ok], minlength=span)[:span]
    assert keys.dtype in (torch.int32, torch.int64) and span < 2**31
    keys = keys.contiguous()
    n = keys.numel()
    # (int32 scatter positions: n < 2^31 is guaranteed by the bincount branch above)
    if HIST_PARTITIONED and not sparse and (1 << 22) <= n < 2**31 - 1 and (1 << 16) <= span <= (1 << 27):
        return _key_histogram_partitioned(keys, kmin, span, valid)
    counts = torch.zeros(span, dtype=torch.int32, device=keys.device)
    launch("key_histogram").key_histogram(ptr(keys), keys.dtype == torch.int64,
                                          ptr(valid.contiguous() if valid is not None else None), keys.numel(), kmin,
                                          span, ptr(counts), stream(keys))
    return counts.to(torch.int64)


HIST_PARTITIONED = True


def _key_histogram_partitioned(keys: torch.Tensor, kmin: int, span: int, valid: Optional[torch.Tensor]):
    """Radix-partitioned COUNT per key (csrc/kernels/agg.hip): bucket counts,
    scan, 16-bit scatter, one LDS histogram per 16384-key bucket."""
    from .select import exclusive_scan
    N = launch("key_histogram_partitioned")
    st = stream(keys)
    dev = keys.device
    n = keys.numel()
    k64 = keys.dtype == torch.int64
    vp = ptr(valid.contiguous() if valid is not None else None)
    nbk, nblk = N.key_histogram_buckets(span), N.key_histogram_blocks()
    cnt = torch.empty(nbk * nblk, dtype=torch.int32, device=dev)
    N.key_histogram_partitioned(ptr(keys), k64, vp, n, kmin, span, 0, ptr(cnt), 0, 0, 0, 0, st)
    off, total = exclusive_scan(cnt)
    part = torch.empty(max(total, 1), dtype=torch.int16, device=dev)
    counts = torch.empty(span, dtype=torch.int32, device=dev)
    N.key_histogram_partitioned(ptr(keys), k64, vp, n, kmin, span, 1, 0, ptr(off), total, ptr(part), 0, st)
    N.key_histogram_partitioned(ptr(keys), k64, vp, n, kmin, span, 2, 0, ptr(off), total, ptr(part), ptr(counts), st)
    return counts.to(torch.int64)


HAVING_OPS = {"=": 0, "<>": 1, "<": 2, "<=": 3, ">": 4, ">=": 5}


def sorted_having(keys: torch.Tensor, specs: Sequence[Spec], hidx: int, hop: str, hconst) -> Optional[Tuple[
        torch.Tensor, List[torch.Tensor]]]:
    """GROUP BY sorted ``keys`` HAVING specs[hidx] <hop> hconst in one pass
    (csrc/kernels/agg.hip sorted_having): (run start rows of the passing
    groups in row order, per-spec results for them), or None when a run is
    longer than the kernel follows or too many groups pass (the caller takes
    the general path). ``hconst``: int in the aggregate's raw units, or float
    for f64 aggregates."""
    from .sort import argsort
    n = keys.numel()
    dev = keys.device
    cap = n // 64 + 4096
    descs, posts = [], []
    for op, vals, valid in specs:
        dst = torch.empty(cap, dtype=torch.float64 if op == "sum_f64" else torch.int64, device=dev)
        dst2 = torch.empty(cap, dtype=torch.int64, device=dev) if op == "sum_int" else None
        src64 = 1
        if vals is not None:
            assert vals.numel() == n and vals.is_contiguous()
            if op in _INT_OPS:
                # int16 / int8 (codes 2 / 3): a NULL-free SUM for the streaming kernel only
                src64 = {torch.int64: 1, torch.int32: 0, torch.int16: 2, torch.int8: 3}[vals.dtype]
                assert src64 < 2 or (op == "sum_int" and valid is None), "narrow values: NULL-free SUM only"
        descs.append((OPS[op], src64, ptr(vals), ptr(valid), ptr(dst), ptr(dst2)))
        posts.append((op, dst, dst2))
    c = int(hconst) if not isinstance(hconst, float) else 0
    lo = ((c + 2**64) % 2**64) - (2**64 if ((c + 2**64) % 2**64) >= 2**63 else 0)
    hi = c >> 64
    if not (I64_MIN <= hi <= I64_MAX):
        return None
    rep = torch.empty(cap, dtype=torch.int64, device=dev)
    counter = torch.zeros(2, dtype=torch.int64, device=dev)
    launch("sorted_having").sorted_having(ptr(keys.contiguous()), keys.dtype == torch.int64, n, descs, hidx,
                                          HAVING_OPS[hop], lo, hi, float(hconst), ptr(rep), cap, ptr(counter),
                                          stream(keys))
    m, overflow = to_host_ints(counter)
    if overflow or m > cap:
        return None
    perm = argsort([(rep[:m], False, False, None)], m, dev) if m > 1 else torch.arange(m, device=dev)
    rep = rep[:m].index_select(0, perm.long())
    outs = []
    wide = [(dst[:m].index_select(0, perm.long()), dst2[:m].index_select(0, perm.long()))
            for op, dst, dst2 in posts if op == "sum_int"]
    fits = iter([1 - f for f in to_host_ints(_wide_flags(wide))] if wide and m else [1] * len(wide))
    witer = iter(wide)
    for op, dst, dst2 in posts:
        if op == "sum_int":
            lo_, hi_ = next(witer)
            outs.append(lo_ if next(fits) else torch.stack([lo_, hi_], dim=1))
            continue
        d = dst[:m].index_select(0, perm.long())
        if op in ("min_f64", "max_f64"):
            sentinel = I64_MAX if op == "min_f64" else I64_MIN
            inf = float("inf") if op == "min_f64" else float("-inf")
            d = torch.where(d == sentinel, torch.full_like(d, 0).double() + inf, _ordered_to_f64(d))
        outs.append(d)
    return rep, outs
