"""Stream compaction and prefix sums (csrc/kernels/select.hip, scan.hip)."""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from ._lib import idx_dtype, is_gpu, launch, ptr, stream, to_host_int, to_host_ints


#: masks of more tiles than select.hip's one-workgroup count (kSmallTiles = 8)
#: take per-tile counts from the kernel that wrote them
_SMALL_TILES = 8


def fused_counts_ok(n: int) -> bool:
    return -(-n // 8192) > _SMALL_TILES


def attach_tile_counts(mask: torch.Tensor, tc: torch.Tensor) -> None:
    """``tc`` [tiles + 1] holds the per-tile set-row counts of ``mask`` as
    written with it (exec/fused_jit.py tiled mask kernel): the next count of
    this mask scans them instead of re-reading the mask. Tied to the mask's
    version counter, so an in-place change of the mask drops them."""
    mask._igloo_tc = (tc, mask._version)


def _select_count(N, mask: torch.Tensor, n: int, tiles: int, s) -> torch.Tensor:
    """ws [tiles + 1] int64: exclusive per-tile offsets of the set rows of
    ``mask`` and their total (select.hip select_count) -- from the tile counts
    the mask's kernel wrote when it has them (consumed: scanned in place)."""
    pre = getattr(mask, "_igloo_tc", None)
    if pre is not None:
        mask._igloo_tc = None
        ws, ver = pre
        if ver == mask._version and ws.numel() == tiles + 1 and tiles > _SMALL_TILES:
            N.select_scan_counts(ptr(ws), tiles, ptr(ws) + 8 * tiles, s)
            return ws
    ws = torch.empty(tiles + 1, dtype=torch.int64, device=mask.device)
    N.select_count(ptr(mask), n, ptr(ws), ptr(ws) + 8 * tiles, s)
    return ws


def mask_to_indices(mask: torch.Tensor, total: Optional[int] = None) -> torch.Tensor:
    """Ordered indices of the True entries of a bool mask (int32 when they fit).
    ``total``: the caller knows how many are set (no count readback)."""
    assert mask.dtype == torch.bool and mask.dim() == 1
    n = mask.numel()
    it = idx_dtype(n)
    if not is_gpu(mask):
        out = torch.nonzero(mask).flatten().to(it)
        out._igloo_incr = True
        return out
    mask = mask.contiguous()
    N = launch("select")
    tiles = N.select_num_tiles(n)
    s = stream(mask)
    ws = _select_count(N, mask, n, tiles, s)
    if total is None:
        total = to_host_int(ws[tiles:])
    out = torch.empty(total, dtype=it, device=mask.device)
    if total:
        N.select_write(ptr(mask), n, ptr(ws), ptr(out), it == torch.int64, total, s)
    out._igloo_incr = True       # strictly increasing: gathers by it keep distinct rows distinct
    return out


class MaskRows:
    """The set rows of a bool mask as a count now and an index vector on
    first use: the count pass and its readback run at once, the index write
    (select_write: 4 bytes per surviving row) only when something reads
    ``idx`` -- a join probing the masked table in place never does
    (exec/joins.py _in_place_side)."""

    __slots__ = ("mask", "_total", "_ws", "_idx", "_tiles")

    def __init__(self, mask: torch.Tensor, defer: bool = False):
        """``defer``: the count's readback waits until ``total`` is read (or
        ``resolve`` reads several at once: a multi-way join's filtered inputs
        are counted with one readback)."""
        assert mask.dtype == torch.bool and mask.dim() == 1
        self.mask = mask.contiguous()
        self._idx = None
        self._ws = None
        self._total = None
        if not is_gpu(mask):
            self._idx = mask_to_indices(self.mask)
            self._total = self._idx.numel()
            return
        n = mask.numel()
        N = launch("select")
        self._tiles = tiles = N.select_num_tiles(n)
        self._ws = _select_count(N, self.mask, n, tiles, stream(mask))
        if not defer:
            self._total = to_host_int(self._ws[tiles:])

    @property
    def total(self) -> int:
        if self._total is None:
            self._total = to_host_int(self._ws[self._tiles:])
        return self._total

    @staticmethod
    def resolve(rows: Sequence["MaskRows"]) -> None:
        """Read the pending counts of ``rows`` back together (one sync)."""
        pend = [r for r in rows if r._total is None]
        if len(pend) > 1:
            for r, v in zip(pend, to_host_ints(torch.cat([r._ws[r._tiles:] for r in pend]))):
                r._total = v

    @property
    def idx(self) -> torch.Tensor:
        if self._idx is None:
            n = self.mask.numel()
            out = torch.empty(self.total, dtype=idx_dtype(n), device=self.mask.device)
            if self.total:
                launch("select").select_write(ptr(self.mask), n, ptr(self._ws), ptr(out), out.dtype == torch.int64,
                                              self.total, stream(self.mask))
            out._igloo_incr = True
            self._idx, self._ws = out, None
        return self._idx


def count_true(mask: torch.Tensor) -> int:
    """Number of True entries of a bool mask (one count pass, one readback)."""
    assert mask.dtype == torch.bool and mask.dim() == 1
    n = mask.numel()
    if not is_gpu(mask):
        return int(mask.sum().item())
    mask = mask.contiguous()
    N = launch("select")
    tiles = N.select_num_tiles(n)
    ws = _select_count(N, mask, n, tiles, stream(mask))
    return to_host_int(ws[tiles:])


def exclusive_scan(counts: torch.Tensor, host_total: bool = True):
    """int32/int64 counts -> (int64 exclusive offsets, total). ``host_total``
    False: the total stays a 1-element device tensor (no readback)."""
    assert counts.dim() == 1 and counts.dtype in (torch.int32, torch.int64)
    n = counts.numel()
    if not is_gpu(counts):
        c = counts.to(torch.int64)
        inc = torch.cumsum(c, 0)
        total = int(inc[-1].item()) if n else 0
        return inc - c, (total if host_total else torch.tensor([total], dtype=torch.int64))
    counts = counts.contiguous()
    N = launch("exclusive_scan")
    tiles = N.scan_workspace_tiles(n)
    ws = torch.empty(tiles + 1, dtype=torch.int64, device=counts.device)
    out = torch.empty(n, dtype=torch.int64, device=counts.device)
    N.exclusive_scan(ptr(counts), counts.dtype == torch.int64, n, ptr(out), ptr(ws), ptr(ws) + 8 * tiles, stream(counts))
    return out, (to_host_int(ws[tiles:]) if host_total else ws[tiles:])


def offsets_from_lengths(lengths: torch.Tensor, host_total: bool = True):
    """Arrow offsets [n+1] from per-row lengths (``host_total`` False: no
    readback; the total comes back as a device tensor, the offsets' last
    element). GPU: the scan writes the offsets and the total in place."""
    n = lengths.numel()
    if not is_gpu(lengths):
        ex, total = exclusive_scan(lengths, host_total)
        off = torch.empty(n + 1, dtype=torch.int64)
        off[:-1] = ex
        off[-1] = int(total) if host_total else int(total[0])
        return off, (total if host_total else off[-1:])
    lengths = lengths.contiguous()
    N = launch("exclusive_scan")
    tiles = N.scan_workspace_tiles(n)
    ws = torch.empty(tiles, dtype=torch.int64, device=lengths.device)
    off = torch.empty(n + 1, dtype=torch.int64, device=lengths.device)
    N.exclusive_scan(ptr(lengths), lengths.dtype == torch.int64, n, ptr(off), ptr(ws), ptr(off) + 8 * n,
                     stream(lengths))
    return off, (to_host_int(off[n:]) if host_total else off[n:])


#: columns per fused compaction launch (csrc/kernels/kernels.h kMaxCompactCols)
COMPACT_MAX_COLS = 12


def compact_columns(mask: torch.Tensor, cols, total: Optional[int] = None, want_idx: bool = True):
    """Rows where ``mask`` is True of every column in ``cols`` -> (row indices
    or None, compacted columns). On the GPU the fixed-width columns (numbers,
    dates, dictionary codes, 128-bit decimals, with their validity) are
    compacted in ONE fused pass per 12 columns (select.hip tile_compact): the
    mask's surviving offsets are staged per tile in LDS and every column is
    copied through them, with no index vector between the mask and the
    gathers. Plain string columns go through the indices."""
    from ..columnar import Column
    from .gather import _inherit, take_many
    assert mask.dtype == torch.bool and mask.dim() == 1
    n = mask.numel()
    if not is_gpu(mask):
        idx = mask_to_indices(mask, total)
        return idx, take_many(list(cols), idx)
    mask = mask.contiguous()
    N = launch("select_compact")
    tiles = N.select_num_tiles(n)
    s = stream(mask)
    ws = _select_count(N, mask, n, tiles, s)
    if total is None:
        total = to_host_int(ws[tiles:])
    it = idx_dtype(n)
    plain = [c for c in cols if c.is_plain_string]
    idx = torch.empty(total, dtype=it, device=mask.device) if (want_idx or plain) else None
    outs = {}
    descs = []
    for k, c in enumerate(cols):
        if c.is_plain_string:
            continue
        d = c.data.contiguous()
        out = torch.empty((total,) + tuple(d.shape[1:]), dtype=d.dtype, device=mask.device)
        esz = d.element_size() * (d.shape[1] if d.dim() == 2 else 1)
        dv = torch.empty(total, dtype=torch.bool, device=mask.device) if c.valid is not None else None
        descs.append((ptr(d), ptr(out), esz, ptr(c.valid.contiguous() if c.valid is not None else None), ptr(dv)))
        _inherit(out, c.data)
        if getattr(c.data, "_igloo_distinct", False):
            out._igloo_distinct = True        # rows kept in order: still distinct
        outs[k] = Column(c.dtype, out, dv, dictionary=c.dictionary)
    if n and (descs or idx is not None):
        first = True
        for a in range(0, max(len(descs), 1), COMPACT_MAX_COLS):
            N.select_compact(ptr(mask), n, ptr(ws), descs[a:a + COMPACT_MAX_COLS],
                             ptr(idx) if first and idx is not None else 0, it == torch.int64, total, s)
            first = False
    if idx is not None:
        idx._igloo_incr = True
    if plain:
        for k, c in zip([k for k, c in enumerate(cols) if c.is_plain_string], take_many(plain, idx)):
            outs[k] = c
    return idx, [outs[k] for k in range(len(cols))]
