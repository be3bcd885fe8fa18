"""Hash-join tables and GROUP BY encoding (csrc/kernels/hashtable.hip).

``JoinTable`` builds once on the (smaller) build side and supports the probe
shapes the join operator needs: full pair expansion (inner / outer), first
match (unique build keys, semi/anti), and build-side "matched" flags (right /
full outer). ``group_ids`` maps int64 group keys to dense group ids.

CPU tensors use a sort + searchsorted reference implementation.
"""
from __future__ import annotations

from ..utils import switches as _sw
import contextvars
import os
from typing import List, Optional, Sequence, Tuple

import torch

from .gather import origin as _origin
from ._lib import capturing, check_not_capturing, is_gpu, launch, native, ptr, stream, to_host_f64s, to_host_int, to_host_ints, unlogged
from .select import exclusive_scan, mask_to_indices

EMPTY_KEY = -(2**63)
INT32_MAX = 2**31 - 1
BLOOM_MAX_KEYS = 4 << 20   # build sides up to this size get a Bloom filter
BLOOM_MIN_RATIO = 4        # ... used when probe rows >= ratio x build rows
EXACT_BITMAP = True
EXACT_BITMAP_MAX_SPAN = 1 << 25   # direct tables up to this key span use an exact bitmap instead
#: join build keys whose [min, max] span is at most this use the direct-mapped
#: table (one random read per probe) whatever the build size: 2^26 slots is a
#: 256 MB head array, small next to 288 GB of HBM
DIRECT_JOIN_MAX_SPAN = 1 << 26

#: bytes one join table may take under an engine device budget (set around a
#: query's execution by engine.py); None = unbounded. A direct-mapped table is
#: sized by the key span, not the build rows: a grace partition or a streamed
#: semi-join build side keeps the whole span of its keys
TABLE_BYTES_LIMIT: "contextvars.ContextVar[Optional[int]]" = contextvars.ContextVar("igloo_table_bytes", default=None)
#: first-match probes that only select rows use the two-pass hit-bit kernels
PROBE_SELECT = True


def _next_pow2(x: int) -> int:
    p = 1
    while p < x:
        p <<= 1
    return p


def column_stats(keys: torch.Tensor, valid: Optional[torch.Tensor] = None) -> Tuple[Optional[Tuple[int, int]], bool]:
    """((min, max) of the non-NULL keys or None, non-decreasing?) — one pass of
    csrc/kernels/util.hip and one host sync on the GPU. Remembered on resident
    key columns (no validity)."""
    if valid is None:
        hit = getattr(keys, "_igloo_stats", None)
        if hit is not None:
            return hit
    n = keys.numel()
    if not is_gpu(keys) or keys.dtype not in (torch.int32, torch.int64):
        k = keys if valid is None else keys[valid]
        if k.numel() == 0:
            return None, True
        mn, mx = torch.aminmax(k)
        srt = True if k.numel() < 2 else bool((k[1:] >= k[:-1]).all().item())
        return (int(mn.item()), int(mx.item())), srt
    N = launch("column_stats")
    buf = torch.empty(N.STATS_SLOTS, dtype=torch.int64, device=keys.device)   # result + per-block partials
    N.column_stats(ptr(keys.contiguous()), keys.dtype == torch.int64,
                   ptr(valid.contiguous() if valid is not None else None), n, ptr(buf), stream(keys))
    out = buf[:3]
    if valid is None and getattr(keys, "_igloo_resident", False):
        with unlogged():      # remembered below: a one-time build (ops/_lib.py unlogged)
            mn, mx, bad = to_host_ints(out)
    else:
        mn, mx, bad = to_host_ints(out)
    res = ((mn, mx) if mn <= mx else None), (bad == 0 and valid is None)
    if valid is None:
        # remembered on any key tensor (like is_sorted's flag): a sortedness
        # check followed by a range lookup of the same keys (group_ids_ex ->
        # group_ids, inner_pairs -> JoinTable) reads the stats back once
        try:
            keys._igloo_stats = res
            if getattr(keys, "_igloo_resident", False):
                keys._igloo_sorted = res[1]
        except (AttributeError, RuntimeError):
            pass
    return res


def key_range(keys: torch.Tensor, valid: Optional[torch.Tensor] = None) -> Optional[Tuple[int, int]]:
    return column_stats(keys, valid)[0]


#: below this many keys a readback-free bound that rules out the direct table
#: is trusted (hash table, no range readback); above it the exact range is read,
#: since a filtered subset may still fit a direct table (far cheaper at size)
BOUND_TRUST_ROWS = 1 << 20


#: IGLOO_DEBUG=key_tags (tests set CHECK_KEY_TAGS directly): verify every
#: readback-free key fact (key_unique tags, key_bound intervals) against the
#: data it describes, one readback each
CHECK_KEY_TAGS = _sw.debug("key_tags")


def _check_bound(keys: torch.Tensor, b: Tuple[int, int]) -> Tuple[int, int]:
    if CHECK_KEY_TAGS and keys.numel() and not capturing():
        lo, hi = to_host_ints(torch.stack([keys.min().to(torch.int64), keys.max().to(torch.int64)]))
        if lo < b[0] or hi > b[1]:
            raise AssertionError(f"key_bound {b} does not hold the keys' range [{lo}, {hi}]")
    return b


def key_bound(keys: torch.Tensor) -> Optional[Tuple[int, int]]:
    """An interval holding every key, known without a readback in steady
    state: the (remembered) range of the resident column the keys were
    gathered from, or a bound its producer attached (``_igloo_bound``:
    dictionary codes lie in [0, dictionary size)). Looser than ``key_range``
    for a filtered subset; callers use it where a bound suffices
    (direct-mapped table spans, bit widths, overflow-free sums)."""
    b = getattr(keys, "_igloo_bound", None)
    if b is not None:
        return _check_bound(keys, b)
    o = _origin(keys)
    if o is None or o.dtype != keys.dtype or o.dim() != 1:
        return None
    st = getattr(o, "_igloo_stats", None)
    if st is None:
        if capturing():
            return None
        st = column_stats(o)
    return _check_bound(keys, st[0]) if st[0] is not None else None


#: unsorted resident key columns up to this many rows get a one-time
#: uniqueness check (sorted ones: one adjacent-difference pass at any size)
UNIQUE_CHECK_MAX_ROWS = 1 << 27


def _check_unique(keys: torch.Tensor, why: str) -> bool:
    """IGLOO_DEBUG=key_tags: a tag-derived uniqueness must hold on the data."""
    if CHECK_KEY_TAGS and keys.numel() > 1 and not capturing():
        n = keys.numel()
        u = torch.unique(keys.to(torch.int64)).numel()
        if u != n:
            raise AssertionError(f"key_unique() trusted {why} on {n} keys with {n - u} duplicates")
    return True


def key_unique(keys: torch.Tensor) -> bool:
    """True only when the keys are known distinct with no readback in steady
    state: a single GROUP BY key (``_igloo_distinct``, kept through filters
    that select rows in order, ops/gather.py take_many), distinct rows (a resident column, or a filtered scan's rows of one,
    in row order) of a resident column whose values are unique (checked once
    and remembered on it)."""
    if getattr(keys, "_igloo_distinct", False):
        return _check_unique(keys, "a distinct tag")
    if getattr(keys, "_igloo_resident", False):
        o = keys
    else:
        base = getattr(keys, "_igloo_base", None)
        if base is None or base[0].data.dtype != keys.dtype or not getattr(base[0].data, "_igloo_resident", False):
            return False
        o = base[0].data
    u = getattr(o, "_igloo_unique", None)
    if u is None:
        if capturing() or not is_gpu(o) or o.dim() != 1:
            return False
        if TABLE_BYTES_LIMIT.get() is not None or (o.numel() > UNIQUE_CHECK_MAX_ROWS and not is_sorted(o)):
            # under a device budget, or an unsorted column too large for a
            # one-time group-by pass: not known unique (the build's own
            # duplicate check decides)
            return False
        with unlogged():     # one-time check of a resident column (ops/_lib.py unlogged)
            n = o.numel()
            if n < 2:
                u = True
            elif column_stats(o)[1]:
                u = to_host_int((o[1:] == o[:-1]).any().to(torch.int64)) == 0
            else:
                u = group_ids(o)[1] == n
        try:
            o._igloo_unique = u
        except (AttributeError, RuntimeError):
            return False
    return u and _check_unique(keys, "the resident base column's uniqueness" if o is not keys else
                               "a resident column's uniqueness")


def _keys_ok(k: torch.Tensor) -> torch.Tensor:
    assert k.dim() == 1 and k.dtype in (torch.int32, torch.int64), f"join keys must be int32/int64, got {k.dtype}"
    return k.contiguous()


class JoinTable:
    """Hash table over build-side keys (int32/int64; NULL keys never match)."""

    def __init__(self, keys: torch.Tensor, valid: Optional[torch.Tensor] = None, defer_unique: bool = False):
        """``defer_unique``: the build's duplicate count is read back only when
        ``unique`` is first asked -- or together with the first
        ``probe_select``'s hit total (one readback for both)."""
        keys = _keys_ok(keys)
        self.n = n = keys.numel()
        self._dups = None
        self.device = keys.device
        self.gpu = is_gpu(keys)
        self.valid = valid
        rng = None
        if valid is None and self.gpu:
            # a resident-derived bound that already selects the direct table
            # (the exact range could only narrow it): no range readback
            bnd = key_bound(keys)
            if bnd is not None and (self._direct_for(bnd[1] - bnd[0] + 1, n) or n < BOUND_TRUST_ROWS):
                rng = bnd
        if rng is None:
            rng = key_range(keys, valid)
        self.empty = rng is None
        if self.empty:
            self.unique = True
            return
        self.kmin, kmax = rng
        span = kmax - self.kmin + 1
        self.direct = self._direct_for(span, n)
        if not self.gpu:
            k = keys if valid is None else torch.where(valid, keys, torch.full_like(keys, kmax + 1) if kmax < 2**62 else keys)
            sk, order = torch.sort(k.to(torch.int64), stable=True)
            if valid is not None:
                nv = int(valid.sum().item())
                sk, order = sk[:nv], order[:nv]
            self.sorted_keys, self.order = sk, order
            self.unique = bool((sk[1:] != sk[:-1]).all().item()) if sk.numel() > 1 else True
            return
        known_unique = valid is None and key_unique(keys)
        N = launch("join_build")
        self.cap = span if self.direct else _next_pow2(2 * n)
        # Bloom filter for selective probes: ~8 bits per key, at most 4 MB (L2-resident)
        self.bits, self.bmask = None, 0
        if self.direct and EXACT_BITMAP and span <= EXACT_BITMAP_MAX_SPAN:
            # exact membership bitmap over the key span (<= 4 MB, L2-resident):
            # no false positives (csrc/kernels/hashtable.hip kExactBits)
            self.bits = torch.zeros((span + 31) // 32, dtype=torch.int32, device=self.device)
            self.bmask = 1 << 63
        elif n <= BLOOM_MAX_KEYS:
            nbits = min(max(_next_pow2(8 * n), 1 << 15), 1 << 25)
            self.bits = torch.zeros(nbits // 32, dtype=torch.int32, device=self.device)
            self.bmask = nbits - 1
        # row ids: int32 below 2^31 build rows, int64 above
        self.rid = torch.int32 if n < INT32_MAX else torch.int64
        self.rid64 = self.rid == torch.int64
        self.thead = torch.full((self.cap,), -1, dtype=self.rid, device=self.device)
        self.tkeys = (torch.empty(1, dtype=torch.int64, device=self.device) if self.direct
                      else torch.full((self.cap,), EMPTY_KEY, dtype=torch.int64, device=self.device))
        dups = torch.zeros(1, dtype=torch.int64, device=self.device)
        k64 = keys.dtype == torch.int64
        st = stream(keys)
        N.join_build(ptr(keys), k64, ptr(valid), n, ptr(self.tkeys), ptr(self.thead), self.rid64, self.cap,
                     self.kmin, self.direct, ptr(dups), ptr(self.bits), self.bmask, st)
        if known_unique and CHECK_KEY_TAGS and not capturing():
            # debug / test mode: the tag-derived uniqueness must match the build's own duplicate count
            if to_host_int(dups) != 0:
                raise AssertionError("key_unique() trusted a key tag on keys that hold duplicates")
        self.cstart = self.crows = None
        self._csr_src = (keys, valid)
        if known_unique:
            self._unique = True
        elif defer_unique:
            self._unique, self._dups = None, dups
        else:
            self._set_unique(to_host_int(dups) == 0)

    @property
    def unique(self) -> bool:
        if self._unique is None:
            self._set_unique(to_host_int(self._dups) == 0)
        return self._unique

    @unique.setter
    def unique(self, v: bool) -> None:
        self._unique = v

    def _set_unique(self, u: bool) -> None:
        """Record the build's uniqueness; duplicate keys get CSR runs (count ->
        exclusive scan -> scatter), so a multi-match probe reads one
        contiguous run of build rows."""
        self._unique, self._dups = u, None
        if not u:
            keys, valid = self._csr_src
            k64 = keys.dtype == torch.int64
            st = stream(keys)
            n = self.n
            cnt = torch.zeros(self.cap + 1, dtype=self.rid, device=self.device)
            launch("join_csr_count").join_csr_count(ptr(keys), k64, ptr(valid), n, ptr(self.tkeys), ptr(cnt),
                                                    self.rid64, self.cap, self.kmin, self.direct, st)
            self.cstart = torch.zeros(self.cap + 1, dtype=self.rid, device=self.device)
            torch.cumsum(cnt[:-1], 0, dtype=self.rid, out=self.cstart[1:])
            self.crows = torch.empty(n, dtype=self.rid, device=self.device)
            launch("join_csr_scatter").join_csr_scatter(ptr(keys), k64, ptr(valid), n, ptr(self.tkeys), ptr(cnt),
                                                        ptr(self.cstart), ptr(self.crows), self.rid64, self.cap,
                                                        self.kmin, self.direct, st)

    @staticmethod
    def _direct_for(span: int, n: int) -> bool:
        lim = TABLE_BYTES_LIMIT.get()
        # (head + CSR start/count arrays: up to 3 int32 words per slot)
        wide_ok = span <= DIRECT_JOIN_MAX_SPAN and (lim is None or 12 * span <= lim)
        return span < 2**31 - 1 and (span <= 4 * n + 4096 or wide_ok)

    # ----------------------------------------------------------------- probes
    def probe_first(self, pkeys: torch.Tensor, pvalid: Optional[torch.Tensor] = None,
                    build_matched: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One matching build row per probe row (-1 if none). Exact for unique builds;
        with duplicates it returns an arbitrary match (enough for semi/anti joins)."""
        self.unique      # a deferred duplicate count is read now (CSR runs built if any)
        pkeys = _keys_ok(pkeys)
        m = pkeys.numel()
        if self.empty or m == 0:
            return torch.full((m,), -1, dtype=torch.int32, device=pkeys.device)
        if not self.gpu:
            cnt, lo = self._cpu_ranges(pkeys, pvalid)
            first = torch.where(cnt > 0, self.order.index_select(0, lo.clamp(max=max(self.order.numel() - 1, 0))),
                                torch.full_like(lo, -1)).to(torch.int32)
            if build_matched is not None:
                self._cpu_mark(cnt, lo, build_matched)
            return first
        first = torch.empty(m, dtype=self.rid, device=pkeys.device)
        N = launch("join_probe")
        bits, bmask = self._bloom(m)
        N.join_probe(ptr(pkeys), pkeys.dtype == torch.int64, ptr(pvalid), m, ptr(self.tkeys), ptr(self.thead),
                     ptr(self.cstart), ptr(self.crows), self.rid64, self.cap, self.kmin, self.direct, 0, ptr(first),
                     ptr(build_matched), bits, bmask, stream(pkeys))
        return first

    def probe_select(self, pkeys: torch.Tensor, pvalid: Optional[torch.Tensor] = None, negate: bool = False,
                     want_build: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Probe rows with a match (``negate``: without one), in row order, and
        for matches their (first) build row — what ``probe_first`` + compaction
        give, in two passes that never write a per-row result (GPU)."""
        pkeys = _keys_ok(pkeys)
        m = pkeys.numel()
        dev = pkeys.device
        if not self.gpu or self.empty or m == 0 or not PROBE_SELECT:
            first = self.probe_first(pkeys, pvalid)      # resolves a deferred ``unique``
            if not self.unique and want_build and not negate:
                return None     # duplicate build keys: the caller takes the multi-match probe (as the GPU path)
            sel = mask_to_indices(first < 0 if negate else first >= 0)
            return sel, (first.index_select(0, sel.long()) if want_build and not negate else None)
        N = launch("probe_hits")
        st = stream(pkeys)
        k64 = pkeys.dtype == torch.int64
        tiles = N.probe_hit_tiles(m)
        words = torch.empty(tiles * 128, dtype=torch.int64, device=dev)
        tcount = torch.empty(tiles, dtype=torch.int64, device=dev)
        bits, bmask = self._bloom(m)
        N.probe_hits(ptr(pkeys), k64, ptr(pvalid), m, ptr(self.tkeys), ptr(self.thead), self.rid64, self.cap,
                     self.kmin, self.direct, bits, bmask, negate, ptr(words), ptr(tcount), st)
        if self._unique is None:
            # deferred duplicate count: read back with the hit total (one sync);
            # duplicate build keys leave the pairs to the multi-match probe
            toff, tdev = exclusive_scan(tcount, host_total=False)
            dups, total = to_host_ints(torch.cat([self._dups.reshape(-1)[:1], tdev.reshape(-1)[:1]]))
            self._set_unique(dups == 0)
            if dups and want_build and not negate:
                return None
        else:
            toff, total = exclusive_scan(tcount)
        it = torch.int32 if m < INT32_MAX else torch.int64
        pidx = torch.empty(total, dtype=it, device=dev)
        bidx = torch.empty(total, dtype=self.rid, device=dev) if want_build and not negate else None
        if total:
            N.probe_write(ptr(pkeys), k64, ptr(pvalid), m, ptr(self.tkeys), ptr(self.thead), self.rid64, self.cap,
                          self.kmin, self.direct, ptr(words), ptr(toff), ptr(pidx), it == torch.int64, ptr(bidx),
                          pidx.numel(), st)
        pidx._igloo_incr = True      # hit rows in row order
        return pidx, bidx

    def probe_pairs(self, pkeys: torch.Tensor, pvalid: Optional[torch.Tensor] = None,
                    build_matched: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """All (probe_row, build_row) matches, grouped by probe row.
        Returns (probe_idx int32, build_idx (int32 below 2^31 build rows, else int64),
        counts int32 per probe row)."""
        self.unique      # a deferred duplicate count is read now (CSR runs built if any)
        pkeys = _keys_ok(pkeys)
        m = pkeys.numel()
        dev = pkeys.device
        if self.empty or m == 0:
            z = torch.zeros(0, dtype=torch.int32, device=dev)
            return z, z, torch.zeros(m, dtype=torch.int32, device=dev)
        if not self.gpu:
            cnt, lo = self._cpu_ranges(pkeys, pvalid)
            if build_matched is not None:
                self._cpu_mark(cnt, lo, build_matched)
            total = int(cnt.sum().item())
            pidx = torch.repeat_interleave(torch.arange(m), cnt)
            starts = torch.cumsum(cnt, 0) - cnt
            within = torch.arange(total) - starts.index_select(0, pidx)
            bpos = lo.index_select(0, pidx) + within
            bidx = self.order.index_select(0, bpos)
            return pidx.to(torch.int32), bidx.to(torch.int32), cnt.to(torch.int32)
        if m >= INT32_MAX:
            raise ValueError(f"probe_pairs: {m} probe rows exceed int32 probe ids; split the probe side")
        N = launch("join_probe")
        s = stream(pkeys)
        counts = torch.empty(m, dtype=torch.int32, device=dev)
        k64 = pkeys.dtype == torch.int64
        bits, bmask = self._bloom(m)
        N.join_probe(ptr(pkeys), k64, ptr(pvalid), m, ptr(self.tkeys), ptr(self.thead), ptr(self.cstart),
                     ptr(self.crows), self.rid64, self.cap, self.kmin, self.direct, ptr(counts), 0,
                     ptr(build_matched), bits, bmask, s)
        offsets, total = exclusive_scan(counts)
        pidx = torch.empty(total, dtype=torch.int32, device=dev)
        bidx = torch.empty(total, dtype=self.rid, device=dev)
        if total:
            launch("join_expand")
            N.join_expand(ptr(pkeys), k64, ptr(pvalid), m, ptr(self.tkeys), ptr(self.thead), ptr(self.cstart),
                          ptr(self.crows), self.rid64, self.cap, self.kmin, self.direct, ptr(offsets), ptr(pidx),
                          ptr(bidx), bits, bmask, pidx.numel(), s)
        return pidx, bidx, counts

    def _bloom(self, m: int) -> Tuple[int, int]:
        """Use the Bloom filter only when the probe side is much larger than the
        build side (then most probes are expected to miss)."""
        if self.bits is not None and m >= BLOOM_MIN_RATIO * self.n:
            return ptr(self.bits), self.bmask
        return 0, 0

    # ------------------------------------------------------------ cpu helpers
    def _cpu_ranges(self, pkeys, pvalid):
        pk = pkeys.to(torch.int64)
        lo = torch.searchsorted(self.sorted_keys, pk, right=False)
        hi = torch.searchsorted(self.sorted_keys, pk, right=True)
        cnt = hi - lo
        if pvalid is not None:
            cnt = torch.where(pvalid, cnt, torch.zeros_like(cnt))
        return cnt, lo

    def _cpu_mark(self, cnt, lo, build_matched):
        total = int(cnt.sum().item())
        if total == 0:
            return
        pidx = torch.repeat_interleave(torch.arange(cnt.numel()), cnt)
        starts = torch.cumsum(cnt, 0) - cnt
        bpos = lo.index_select(0, pidx) + torch.arange(total) - starts.index_select(0, pidx)
        build_matched.index_fill_(0, self.order.index_select(0, bpos).long(), True)


#: inputs at least this large are checked for sorted (clustered) keys first
SORTED_CHECK_ROWS = 1 << 20

def is_sorted(keys: torch.Tensor) -> bool:
    """Non-decreasing check (one pass; remembered on the tensor object, so the
    resident key columns of a table are checked once)."""
    hit = getattr(keys, "_igloo_sorted", None)
    if hit is not None:
        if hit and CHECK_KEY_TAGS and not capturing() and not getattr(keys, "_igloo_resident", False) \
                and keys.numel() > 1 and keys.is_cuda:
            # test mode: a sortedness tag inferred through gathers must hold
            if to_host_int((keys[1:] < keys[:-1]).any().to(torch.int64)):
                raise AssertionError("an inferred sorted tag does not hold")
        return hit
    base = getattr(keys, "_igloo_base", None)
    if base is not None and base[0].data.dtype == keys.dtype and is_sorted(base[0].data):
        # a filtered scan's rows of a sorted source column, in row order
        # (exec/scan.py _tag_base): sorted without another pass (the
        # source's flag is computed once and remembered on it)
        return True
    n = keys.numel()
    r = True if n < 2 else column_stats(keys)[1]
    try:
        keys._igloo_sorted = r
    except (AttributeError, RuntimeError):
        pass
    return r


DENSE_INDEX = True
DENSE_INDEX_MIN_QUERIES = 1 << 20   # below this a binary search per query is cheaper than building
DENSE_INDEX_MAX_SPAN_RATIO = 4      # table entries per indexed row (orders: 1 of 4 key values used)


def dense_index(big: torch.Tensor, build: bool = True, queries: Optional[int] = None):
    """Lower-bound table of a sorted key column (csrc/kernels/ranges.hip):
    ``(kmin, kmax, first)`` with first[k - kmin] = first row whose key >= k,
    or None when the key span is too sparse. Remembered on the tensor object
    (resident table columns build it once)."""
    hit = getattr(big, "_igloo_dense", None)
    # (the sorted keys of a resident column's secondary index live as long as
    # the column: their table is built once too -- Q9's 1.1M green parts
    # searched 600M l_partkey keys by bisection, 0.93 ms per query)
    resident = getattr(big, "_igloo_resident", False) or getattr(big, "_igloo_index_keys", False)
    if hit or (hit is False and (queries is None or resident)):
        return hit or None
    if resident:
        # built once and kept with the resident column: every later lookup
        # reuses it, so only its size matters, not this call's lookup count
        # (lineitem.l_orderkey at SF100: 2.4 GB of int32 for 600M rows)
        if queries is None or queries < DENSE_RESIDENT_MIN_QUERIES:
            return None
        with unlogged():
            return _dense_index_build(big, None, resident=True)
    if not build:
        return None
    rng = getattr(big, "_igloo_range", None)
    if hit is False and rng is not None and rng[1] - rng[0] + 1 > _dense_limit(big.numel(), queries):
        return None           # still too sparse for this many lookups: nothing to build
    return _dense_index_build(big, queries)    # an intermediate: built (and read back) every execution


#: resident columns: lookups per call that justify building the table once,
#: and the largest table (entries) worth its HBM when the keys are sparser
#: than DENSE_INDEX_MAX_SPAN_RATIO (a hash-partitioned rank's slice of a fact
#: table keeps the whole key span)
DENSE_RESIDENT_MIN_QUERIES = 4096
DENSE_RESIDENT_MAX_ENTRIES = 1 << 30


def _dense_limit(nb: int, queries: Optional[int], resident: bool = False) -> int:
    """Largest key span worth a table: small next to both the indexed rows and
    the lookups it serves (resident columns: next to the rows, or 4 GiB)."""
    if resident:
        return max(DENSE_INDEX_MAX_SPAN_RATIO * nb, DENSE_RESIDENT_MAX_ENTRIES) + 4096
    return DENSE_INDEX_MAX_SPAN_RATIO * min(nb, queries if queries is not None else nb) + 4096


def _dense_index_build(big: torch.Tensor, queries: Optional[int], resident: bool = False):
    nb = big.numel()
    idx = False
    if nb:
        rng = getattr(big, "_igloo_range", None)
        if rng is None:
            rng = tuple(to_host_ints(torch.stack([big[0].to(torch.int64), big[-1].to(torch.int64)])))
            try:
                big._igloo_range = rng
            except (AttributeError, RuntimeError):
                pass
        kmin, kmax = rng
        span = kmax - kmin + 1
        if span <= _dense_limit(nb, queries, resident):
            it = torch.int64 if nb >= INT32_MAX else torch.int32
            first = torch.empty(span + 1, dtype=it, device=big.device)
            gap = torch.zeros(1, dtype=torch.int32, device=big.device)
            N = launch("dense_index_build")
            st = stream(big)
            N.dense_index_build(ptr(big), big.dtype == torch.int64, nb, kmin, kmax, ptr(first),
                                it == torch.int64, ptr(gap), st)
            if to_host_int(gap):
                # long key gaps: rebuild over a -1 fill, then search the entries left at -1
                first.fill_(-1)
                N.dense_index_build(ptr(big), big.dtype == torch.int64, nb, kmin, kmax, ptr(first),
                                    it == torch.int64, ptr(gap), st)
                N.dense_index_build(ptr(big), big.dtype == torch.int64, nb, kmin, kmax, ptr(first),
                                    it == torch.int64, 0, st)
            idx = (kmin, kmax, first)
    try:
        big._igloo_dense = idx
    except (AttributeError, RuntimeError):
        pass
    return idx or None


def sorted_ranges(big: torch.Tensor, q: torch.Tensor, qvalid: Optional[torch.Tensor] = None
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """For each probe key q[i]: (lo, cnt) with big[lo : lo+cnt] == q[i] (big non-decreasing).
    GPU: one fused search kernel (csrc/kernels/ranges.hip)."""
    big = _keys_ok(big)
    q = q.to(big.dtype).contiguous()
    nq = q.numel()
    if not is_gpu(big):
        lo = torch.searchsorted(big, q)
        cnt = torch.searchsorted(big, q, right=True) - lo
        if qvalid is not None:
            cnt = torch.where(qvalid, cnt, torch.zeros_like(cnt))
        return lo, cnt
    lo = torch.empty(nq, dtype=torch.int64, device=big.device)
    cnt = torch.empty(nq, dtype=torch.int64, device=big.device)
    idx = dense_index(big, build=nq >= DENSE_INDEX_MIN_QUERIES, queries=nq) if DENSE_INDEX else None
    if idx:
        kmin, kmax, first = idx
        launch("dense_ranges").dense_ranges(ptr(first), first.dtype == torch.int64, kmin, kmax, ptr(q),
                                            q.dtype == torch.int64,
                                            ptr(qvalid.contiguous() if qvalid is not None else None), nq, ptr(lo),
                                            ptr(cnt), stream(big))
        return lo, cnt
    fence = search_fence(big) if SEARCH_FENCE else None
    launch("sorted_ranges").sorted_ranges(ptr(big), big.dtype == torch.int64, big.numel(), ptr(q),
                                          ptr(qvalid.contiguous() if qvalid is not None else None), nq, ptr(lo),
                                          ptr(cnt), ptr(fence), 0 if fence is None else fence.numel(), stream(big))
    return lo, cnt


def unique_lookup(big: torch.Tensor, q: torch.Tensor, qvalid: Optional[torch.Tensor] = None
                  ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """``sorted_ranges`` into DISTINCT sorted keys (``key_unique(big)``):
    (hit bool mask, int32 row in ``big``; 0 on a miss) per probe key. None
    when ``big`` has 2^31 rows or more (the caller takes ``sorted_ranges``).
    GPU: one kernel writing 5 bytes per probe row (csrc/kernels/ranges.hip
    unique_lookup) through the dense index when the column has one."""
    big = _keys_ok(big)
    nb = big.numel()
    if nb >= 2**31 - 1:
        return None
    q = q.to(big.dtype).contiguous()
    nq = q.numel()
    if not is_gpu(big):
        lo = torch.searchsorted(big, q)
        hit = lo < nb
        if nb:
            hit &= big[lo.clamp(max=nb - 1)] == q
        if qvalid is not None:
            hit &= qvalid
        return hit, torch.where(hit, lo, torch.zeros_like(lo)).to(torch.int32)
    hit = torch.empty(nq, dtype=torch.bool, device=big.device)
    pos = torch.empty(nq, dtype=torch.int32, device=big.device)
    qv = ptr(qvalid.contiguous()) if qvalid is not None else 0
    idx = dense_index(big, build=nq >= DENSE_INDEX_MIN_QUERIES, queries=nq) if DENSE_INDEX else None
    N = launch("unique_lookup")
    if idx:
        kmin, kmax, first = idx
        N.unique_lookup(0, big.dtype == torch.int64, nb, ptr(first), first.dtype == torch.int64, kmin, kmax, ptr(q),
                        qv, nq, ptr(hit), ptr(pos), 0, 0, stream(big))
    else:
        fence = search_fence(big) if SEARCH_FENCE else None
        N.unique_lookup(ptr(big), big.dtype == torch.int64, nb, 0, False, 0, 0, ptr(q), qv, nq, ptr(hit), ptr(pos),
                        ptr(fence), 0 if fence is None else fence.numel(), stream(big))
    return hit, pos


SEARCH_FENCE = True
SEARCH_FENCE_MIN_ROWS = 1 << 22


def search_fence(big: torch.Tensor) -> Optional[torch.Tensor]:
    """Every 256th key of a large sorted RESIDENT key column (1/256 of its
    bytes, kept with it like the other derived structures): binary searches
    first narrow to one 256-row window through it (L2/MALL-resident), then
    touch only that window of the column (csrc/kernels/ranges.hip)."""
    if big.numel() < SEARCH_FENCE_MIN_ROWS or not getattr(big, "_igloo_resident", False):
        return None
    hit = getattr(big, "_igloo_fence", None)
    if hit is None:
        check_not_capturing("search fence of a resident column")
        hit = big[::native().SEARCH_FENCE].contiguous()
        try:
            big._igloo_fence = hit
        except (AttributeError, RuntimeError):
            return None
    return hit


def perm_index(keys: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Secondary index of an unsorted resident key column: (keys in sorted
    order, int32 row permutation), built once per column tensor (the stable
    radix sort of ops/sort.py) and kept with it like the other derived
    structures (charged to the column in the HBM cache budget) —
    a join with a much smaller side then reads only the matching ranges
    instead of probing every row of the column."""
    hit = getattr(keys, "_igloo_perm", None)
    if hit is not None:
        return hit
    from .sort import perm_sort_int
    with unlogged():
        out = perm_sort_int(keys)
    try:
        out[0]._igloo_sorted = True
        out[0]._igloo_index_keys = True
        keys._igloo_perm = out
    except (AttributeError, RuntimeError):
        pass
    return out


def expand_ranges(lo: torch.Tensor, cnt: torch.Tensor, big_n: int, scanned=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All pairs (s, lo[s] + k), k < cnt[s], grouped by s (int32 when they fit).
    ``scanned``: the caller's ``exclusive_scan(cnt)`` result, reused."""
    ns = lo.numel()
    dev = lo.device
    off, total = scanned if scanned is not None else exclusive_scan(cnt)
    it = torch.int32 if max(total, big_n, ns) < INT32_MAX else torch.int64
    if not is_gpu(lo):
        sidx = torch.repeat_interleave(torch.arange(ns, dtype=it), cnt, output_size=total)
        bidx = (lo.index_select(0, sidx.long()) - off.index_select(0, sidx.long())
                + torch.arange(total, dtype=torch.int64)).to(it)
        return sidx, bidx
    sidx = torch.empty(total, dtype=it, device=dev)
    bidx = torch.empty(total, dtype=it, device=dev)
    if total:
        launch("expand_ranges").expand_ranges(ptr(off), ptr(lo.contiguous()), ns, total, ptr(sidx), ptr(bidx),
                                              it == torch.int64, stream(lo))
    return sidx, bidx


def sorted_match_pairs(big1: torch.Tensor, big2: torch.Tensor, small1: torch.Tensor, small2: torch.Tensor,
                       identity_ok: bool = False) -> Tuple[Optional[torch.Tensor], torch.Tensor]:
    """(small row, big row) pairs with big1 == small1 and big2 == small2, big1
    non-decreasing (ranges on the first key, then the second key checked inside
    each range on the device). Grouped by small row. ``identity_ok``: when
    every small row has exactly one match (Q9's lineitem into partsupp's
    (partkey, suppkey) key) the small side comes back as None and the count
    pass's first matches are the big rows: no scan, no write pass."""
    lo, cnt = sorted_ranges(big1, small1)
    ns = small1.numel()
    big2 = _keys_ok(big2)
    small2 = small2.to(big2.dtype).contiguous()
    if not is_gpu(big1):
        s, b = expand_ranges(lo, cnt, big1.numel())
        keep = big2.index_select(0, b.long()) == small2.index_select(0, s.long())
        return s[keep], b[keep]
    N = launch("sorted_match")
    st = stream(big1)
    counts = torch.empty(max(ns, 1), dtype=torch.int32, device=big1.device)
    k64 = big2.dtype == torch.int64
    first = torch.empty(ns, dtype=torch.int32, device=big1.device) \
        if identity_ok and ns and max(big1.numel(), ns) < INT32_MAX else None
    N.sorted_match(ptr(big2), ptr(small2), k64, ptr(lo), ptr(cnt), ns, ptr(counts), 0, 0, 0, False, 0, ptr(first), st)
    if first is not None:
        c = counts[:ns]
        total, odd = to_host_ints(torch.stack([c.sum(), (c != 1).sum()]))
        if odd == 0:
            return None, first
        off, _ = exclusive_scan(c, host_total=False)
    else:
        off, total = exclusive_scan(counts[:ns])
    it = torch.int32 if max(total, big1.numel(), ns) < INT32_MAX else torch.int64
    sidx = torch.empty(total, dtype=it, device=big1.device)
    bidx = torch.empty(total, dtype=it, device=big1.device)
    if total:
        N.sorted_match(ptr(big2), ptr(small2), k64, ptr(lo), ptr(cnt), ns, 0, ptr(off), ptr(sidx), ptr(bidx),
                       it == torch.int64, total, 0, st)
    return sidx, bidx


def masked_expand(lo: torch.Tensor, cnt: torch.Tensor, mask: torch.Tensor, big_n: int
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """``expand_ranges`` keeping only the big rows set in ``mask`` (bool[big_n]):
    the pairs of a sorted join whose big side is a filtered table probed in
    place -- its own sorted key column under the filter mask, not a compacted
    copy (exec/joins.py inner_pairs). Grouped by small row."""
    ns = lo.numel()
    if not is_gpu(lo):
        s, b = expand_ranges(lo, cnt, big_n)
        keep = mask.index_select(0, b.long())
        return s[keep], b[keep]
    N = launch("sorted_masked")
    st = stream(lo)
    mk = mask.contiguous().view(torch.uint8)
    counts = torch.empty(max(ns, 1), dtype=torch.int32, device=lo.device)
    N.sorted_masked(ptr(mk), ptr(lo), ptr(cnt), ns, ptr(counts), 0, 0, 0, False, 0, st)
    off, total = exclusive_scan(counts[:ns])
    it = torch.int32 if max(total, big_n, ns) < INT32_MAX else torch.int64
    sidx = torch.empty(total, dtype=it, device=lo.device)
    bidx = torch.empty(total, dtype=it, device=lo.device)
    if total:
        N.sorted_masked(ptr(mk), ptr(lo), ptr(cnt), ns, 0, ptr(off), ptr(sidx), ptr(bidx), it == torch.int64, total,
                        st)
    return sidx, bidx


EXISTS_OPS = {"=": 0, "<>": 1, "<": 2, "<=": 3, ">": 4, ">=": 5, "any": 6}


def sorted_exists(big2: Optional[torch.Tensor], small2: Optional[torch.Tensor], lo: torch.Tensor, cnt: torch.Tensor,
                  op: str, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bool[ns]: some row k of small row i's range (lo, cnt) has big2[k] OP
    small2[i] (op "any": any row; big2 / small2 unused). ``mask``: only the
    big rows set in it count (a filtered big side searched in place)."""
    ns = lo.numel()
    if op == "any":
        big2 = small2 = None
        dt = torch.int32
    else:
        dt = torch.int64 if torch.int64 in (big2.dtype, small2.dtype) else torch.int32
        big2, small2 = big2.to(dt).contiguous(), small2.to(dt).contiguous()
    if not is_gpu(lo):
        nb = mask.numel() if mask is not None else big2.numel()
        s, b = expand_ranges(lo, cnt, nb)
        if op == "any":
            ok = torch.ones(s.numel(), dtype=torch.bool)
        else:
            bv, sv = big2.index_select(0, b.long()), small2.index_select(0, s.long())
            ok = {"=": bv == sv, "<>": bv != sv, "<": bv < sv, "<=": bv <= sv, ">": bv > sv, ">=": bv >= sv}[op]
        if mask is not None:
            ok = ok & mask.index_select(0, b.long())
        hit = torch.zeros(ns, dtype=torch.bool)
        hit.index_fill_(0, s.long()[ok], True)
        return hit
    hit = torch.empty(ns, dtype=torch.bool, device=lo.device)
    mk = mask.contiguous().view(torch.uint8) if mask is not None else None
    launch("sorted_exists").sorted_exists(ptr(big2), ptr(small2), dt == torch.int64, ptr(lo), ptr(cnt), ns,
                                          EXISTS_OPS[op], ptr(mk), ptr(hit), stream(lo))
    return hit


def group_ids_ex(keys: torch.Tensor) -> Tuple[torch.Tensor, int, torch.Tensor, bool]:
    """``group_ids`` plus whether the ids are non-decreasing. Clustered keys
    (lineitem by l_orderkey, any output that follows a sorted probe side) get
    run ids from a boundary compaction instead of a hash table."""
    keys = _keys_ok(keys)
    n = keys.numel()
    if n >= SORTED_CHECK_ROWS and is_gpu(keys):
        if is_sorted(keys):
            bound = torch.empty(n, dtype=torch.bool, device=keys.device)
            launch("run_bounds").run_bounds(ptr(keys), keys.dtype == torch.int64, n, ptr(bound), stream(keys))
            starts = mask_to_indices(bound)
            g = starts.numel()
            gid = torch.empty(n, dtype=torch.int32, device=keys.device)
            launch("fill_runs").fill_runs(ptr(starts), starts.dtype == torch.int64, g, n, ptr(gid), stream(keys))
            gid._igloo_bound = (0, max(g - 1, 0))
            return gid, g, starts.to(torch.int32), True
    gid, g, rep = group_ids(keys)
    return gid, g, rep, False


def group_ids(keys: torch.Tensor) -> Tuple[torch.Tensor, int, torch.Tensor]:
    """Dense group ids for int keys (no NULLs: callers map NULL to a reserved key).

    Returns (gid int32 [n], number of groups, representative row per group int32)."""
    keys = _keys_ok(keys)
    n = keys.numel()
    dev = keys.device
    if n == 0:
        z = torch.zeros(0, dtype=torch.int32, device=dev)
        return z, 0, z
    if not is_gpu(keys):
        uniq, inv = torch.unique(keys, sorted=True, return_inverse=True)
        g = uniq.numel()
        rep = torch.full((g,), n, dtype=torch.int64).scatter_reduce(0, inv, torch.arange(n), reduce="amin")
        return inv.to(torch.int32), g, rep.to(torch.int32)
    bnd = key_bound(keys)
    if bnd is not None and (bnd[1] - bnd[0] + 1 <= 2 * n + 65536 or n < BOUND_TRUST_ROWS):
        kmin, kmax = bnd         # a readback-free bound decides: no range readback
    elif getattr(keys, "_igloo_hashed", False) and n > 1:
        kmin, kmax = 0, 2**62    # 64-bit hashes: the hash table, no range readback
    else:
        kmin, kmax = key_range(keys)
    span = kmax - kmin + 1
    direct = span <= 2 * n + 65536 and span < 2**31 - 1
    cap = span if direct else _next_pow2(2 * n)
    N = launch("groupby")
    s = stream(keys)
    k64 = keys.dtype == torch.int64
    trow = torch.full((cap,), INT32_MAX, dtype=torch.int32, device=dev)
    tkeys = (torch.empty(1, dtype=torch.int64, device=dev) if direct
             else torch.full((cap,), EMPTY_KEY, dtype=torch.int64, device=dev))
    N.groupby_build(ptr(keys), k64, n, ptr(tkeys), ptr(trow), cap, kmin, direct, s)
    occ = torch.empty(cap, dtype=torch.bool, device=dev)
    gid_of_slot = torch.empty(cap, dtype=torch.int32, device=dev)
    N.groupby_occupied(ptr(trow), cap, ptr(occ), ptr(gid_of_slot), s)
    slots = mask_to_indices(occ)
    g = slots.numel()
    rep = torch.empty(g, dtype=torch.int32, device=dev)
    N.groupby_assign(ptr(slots), slots.dtype == torch.int64, g, cap, ptr(trow), ptr(gid_of_slot), ptr(rep), s)
    gid = torch.empty(n, dtype=torch.int32, device=dev)
    N.groupby_lookup(ptr(keys), k64, n, ptr(tkeys), ptr(gid_of_slot), cap, kmin, direct, ptr(gid), s)
    if not direct and g > 1:
        # hashed slots depend on the order in which threads inserted colliding
        # keys, so slot-order ids differ between runs; renumber the groups by
        # their first row (the direct path is already in key order). Stable ids
        # keep every later readback that depends on them (packed-key ranges,
        # group order) identical across executions, which replayed readbacks
        # and query graphs rely on.
        from .gather import gather_tensor
        first = rep.clamp(max=n - 1).long()        # in bounds even under a mismatched replay
        mark = torch.zeros(n, dtype=torch.bool, device=dev)
        mark.index_fill_(0, first, True)
        order = mask_to_indices(mark, total=g)     # g marks: no count readback
        newpos = torch.zeros(n, dtype=torch.int32, device=dev)
        newpos.index_copy_(0, order.long(), torch.arange(order.numel(), dtype=torch.int32, device=dev))
        remap = newpos.index_select(0, first)
        gid = gather_tensor(remap, gid)
        rep = order.to(torch.int32)
    gid._igloo_bound = (0, max(g - 1, 0))     # readback-free bound for packing / regrouping
    return gid, g, rep


def first_rows_mask(keys: torch.Tensor) -> torch.Tensor:
    """bool[n]: True on the first row of every distinct key (the rows
    COUNT/SUM(DISTINCT) keep). GPU: the group-by table's build pass (which
    keeps each group's smallest row) and one pass over its slots -- no group
    ids, no group count readback, no renumbering."""
    keys = _keys_ok(keys)
    n = keys.numel()
    dev = keys.device
    if n == 0 or not is_gpu(keys):
        mark = torch.zeros(n, dtype=torch.bool, device=dev)
        if n:
            _, _, rep = group_ids(keys)
            mark[rep.long()] = True
        return mark
    bnd = key_bound(keys)
    if bnd is not None and (bnd[1] - bnd[0] + 1 <= 2 * n + 65536 or n < BOUND_TRUST_ROWS):
        kmin, kmax = bnd
    elif getattr(keys, "_igloo_hashed", False) and n > 1:
        kmin, kmax = 0, 2**62
    else:
        kmin, kmax = key_range(keys)
    span = kmax - kmin + 1
    direct = span <= 2 * n + 65536 and span < 2**31 - 1
    cap = span if direct else _next_pow2(2 * n)
    s = stream(keys)
    trow = torch.full((cap,), INT32_MAX, dtype=torch.int32, device=dev)
    tkeys = (torch.empty(1, dtype=torch.int64, device=dev) if direct
             else torch.full((cap,), EMPTY_KEY, dtype=torch.int64, device=dev))
    launch("groupby").groupby_build(ptr(keys), keys.dtype == torch.int64, n, ptr(tkeys), ptr(trow), cap, kmin,
                                    direct, s)
    mark = torch.zeros(n, dtype=torch.bool, device=dev)
    launch("mark_slot_rows").mark_slot_rows(ptr(trow), cap, n, ptr(mark), s)
    return mark


HLL_BITS = 12
HLL_M = 1 << HLL_BITS


def hll_sketch(keys: torch.Tensor, valid: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """HyperLogLog registers (uint8 [4096]) of the key column (GPU only; None on CPU).
    Sketches of several ranks merge by element-wise max."""
    src = keys
    if valid is None:
        hit = getattr(src, "_igloo_hll", None)
        if hit is not None:   # resident table columns are sketched once (like is_sorted)
            return hit
    if valid is None and getattr(src, "_igloo_resident", False):
        check_not_capturing("sketch of a resident column")   # kept on the column: a one-time build
    keys = _keys_ok(keys)
    n = keys.numel()
    if not is_gpu(keys):
        return None
    regs = torch.zeros(HLL_M, dtype=torch.uint8, device=keys.device)
    if n == 0:
        return regs
    N = launch("hll_sketch")
    ws = torch.empty(N.hll_blocks(n) * HLL_M, dtype=torch.uint8, device=keys.device)
    N.hll_sketch(ptr(keys), keys.dtype == torch.int64, ptr(valid), n, ptr(ws), ptr(regs), stream(keys))
    if valid is None:
        try:
            src._igloo_hll = regs
        except (AttributeError, RuntimeError):
            pass
    return regs


def hll_terms(regs: torch.Tensor) -> torch.Tensor:
    """Per sketch (rows of ``regs``) the float64 pair (sum 2^-r, zero
    registers) the estimate is computed from, on the device."""
    r = regs.to(torch.float64)
    return torch.stack([torch.pow(2.0, -r).sum(-1), (regs == 0).sum(-1).to(torch.float64)], -1)


def hll_estimate(regs: torch.Tensor) -> float:
    """Cardinality estimate from HLL registers (bias-corrected; linear counting
    for small cardinalities). Relative error ~1.04/sqrt(4096) = 1.6%."""
    z, zeros = to_host_f64s(hll_terms(regs))
    return hll_from_terms(z, int(zeros))


def hll_from_terms(z: float, zeros: int) -> float:
    m = float(HLL_M)
    alpha = 0.7213 / (1.0 + 1.079 / m)
    e = alpha * m * m / z
    if e <= 2.5 * m and zeros > 0:
        import math
        e = m * math.log(m / zeros)
    return e


def ndv(keys: torch.Tensor, valid: Optional[torch.Tensor] = None) -> int:
    """Distinct count: HLL estimate on GPU, exact on CPU."""
    if keys.numel() == 0:
        return 0
    if is_gpu(keys):
        return max(1, int(round(hll_estimate(hll_sketch(keys, valid)))))
    k = keys if valid is None else keys[valid]
    return int(torch.unique(k).numel())


def pack_keys(cols: Sequence[torch.Tensor]) -> torch.Tensor:
    """Combine several integer key columns into ONE int64 key per row that is
    equal iff all inputs are equal. Bit-packs when the value ranges fit in 63
    bits, otherwise re-encodes pairwise through ``group_ids``."""
    assert cols
    if len(cols) == 1:
        c = cols[0]
        return c if c.dtype in (torch.int32, torch.int64) else c.to(torch.int64)
    ranges = _bounded_ranges(cols)
    bits = [max(1, int(hi - lo).bit_length()) for lo, hi in ranges]
    if sum(bits) <= 62:
        return _pack_bits(cols, ranges, bits)
    # pairwise dense re-encoding keeps every intermediate code < n
    acc = cols[0].to(torch.int64)
    for c in cols[1:]:
        g1, n1, _ = group_ids(acc)
        g2, n2, _ = group_ids(c.to(torch.int64) if c.dtype != torch.int64 else c)
        acc = g1.to(torch.int64) * max(n2, 1) + g2.to(torch.int64)
    return acc


def pack_keys_pair(left: Sequence[torch.Tensor], right: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Pack multi-column join keys of both sides with ONE shared encoding."""
    if len(left) == 1:
        return left[0], right[0]
    nl = left[0].numel()
    if is_gpu(left[0]) and len(left) <= MAX_PACK_BITS:
        # one shared bit layout from both sides' ranges: each side packed in
        # place, no concatenated copies
        both = _bounded_ranges(list(left) + list(right))      # at most one readback for both sides
        rl, rr = both[:len(left)], both[len(left):]
        if right[0].numel() == 0:
            ranges = rl
        elif nl == 0:
            ranges = rr
        else:
            ranges = [(min(a[0], b[0]), max(a[1], b[1])) for a, b in zip(rl, rr)]
        bits = [max(1, int(hi - lo).bit_length()) for lo, hi in ranges]
        if sum(bits) <= 62:
            return _pack_bits(list(left), ranges, bits), _pack_bits(list(right), ranges, bits)
    both = [torch.cat([a.to(torch.int64), b.to(torch.int64)]) for a, b in zip(left, right)]
    packed = pack_keys(both)
    return packed[:nl], packed[nl:]


#: columns one pack_bits launch combines (csrc/kernels/kernels.h kMaxPackBits)
MAX_PACK_BITS = 8


def key_ranges(cols: Sequence[torch.Tensor]) -> List[Tuple[int, int]]:
    """(min, max) of each integer key column ((0, 0) for an empty one; an
    all-NULL-free column assumed), with ONE readback for all of them on the
    GPU (resident columns answer from their remembered stats)."""
    out: List[Optional[Tuple[int, int]]] = [None] * len(cols)
    todo = []
    for i, c in enumerate(cols):
        if c.numel() == 0:
            out[i] = (0, 0)
            continue
        hit = getattr(c, "_igloo_stats", None)
        if hit is not None and hit[0] is not None:
            out[i] = hit[0]
        elif is_gpu(c) and c.dtype in (torch.int32, torch.int64) and c.dim() == 1:
            todo.append(i)
        else:
            r = key_range(c)
            out[i] = r if r is not None else (0, 0)
    if todo:
        N = launch("column_stats")
        bufs = []
        for i in todo:
            c = cols[i].contiguous()
            buf = torch.empty(N.STATS_SLOTS, dtype=torch.int64, device=c.device)
            N.column_stats(ptr(c), c.dtype == torch.int64, 0, c.numel(), ptr(buf), stream(c))
            bufs.append(buf[:2])
        vals = to_host_ints(torch.cat(bufs))
        for j, i in enumerate(todo):
            lo, hi = vals[2 * j], vals[2 * j + 1]
            out[i] = (lo, hi) if lo <= hi else (0, 0)
    return out  # type: ignore[return-value]


def _bounded_ranges(cols: Sequence[torch.Tensor]) -> List[Tuple[int, int]]:
    """Per column an interval holding all its values: the readback-free
    bound where one is known (``key_bound``), else the exact range (read
    back together for all such columns). Packing needs no more than that."""
    out: List[Optional[Tuple[int, int]]] = [None] * len(cols)
    todo = []
    for i, c in enumerate(cols):
        b = key_bound(c) if is_gpu(c) and c.numel() else None
        if b is not None:
            out[i] = b
        else:
            todo.append(i)
    if todo:
        for i, r in zip(todo, key_ranges([cols[i] for i in todo])):
            out[i] = r
    return out  # type: ignore[return-value]


def _pack_bits(cols: Sequence[torch.Tensor], ranges, bits) -> torch.Tensor:
    n = cols[0].numel()
    if not is_gpu(cols[0]) or len(cols) > MAX_PACK_BITS or any(c.dtype not in (torch.int32, torch.int64)
                                                                for c in cols):
        out = None
        for c, (lo, _), b in zip(cols, ranges, bits):
            v = c.to(torch.int64) - lo
            out = v if out is None else (out << b) | v
        return out
    cs = [c.contiguous() for c in cols]
    out = torch.empty(n, dtype=torch.int64, device=cs[0].device)
    shifts = [0] + list(bits[1:])      # acc = (acc << bits[c]) | (v - lo) for every column after the first
    launch("pack_bits").pack_bits([ptr(c) for c in cs], [c.dtype == torch.int64 for c in cs],
                                  [int(lo) for lo, _ in ranges], shifts, n, ptr(out), stream(out))
    return out
