"""Stream compaction and prefix sums (csrc/kernels/select.hip, scan.hip)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._lib import idx_dtype, is_gpu, launch, ptr, stream, to_host_int


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
    ws = torch.empty(tiles + 1, dtype=torch.int64, device=mask.device)
    s = stream(mask)
    N.select_count(ptr(mask), n, ptr(ws), ptr(ws) + 8 * tiles, s)
    if total is None:
        total = to_host_int(ws[tiles:])
    out = torch.empty(total, dtype=it, device=mask.device)
    if total:
        N.select_write(ptr(mask), n, ptr(ws), ptr(out), it == torch.int64, total, s)
    out._igloo_incr = True       # strictly increasing: gathers by it keep distinct rows distinct
    return out


def count_true(mask: torch.Tensor) -> int:
    """Number of True entries of a bool mask (one count pass, one readback)."""
    assert mask.dtype == torch.bool and mask.dim() == 1
    n = mask.numel()
    if not is_gpu(mask):
        return int(mask.sum().item())
    mask = mask.contiguous()
    N = launch("select")
    tiles = N.select_num_tiles(n)
    ws = torch.empty(tiles + 1, dtype=torch.int64, device=mask.device)
    N.select_count(ptr(mask), n, ptr(ws), ptr(ws) + 8 * tiles, stream(mask))
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
