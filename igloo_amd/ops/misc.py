"""Partitioning, date parts and sorting (csrc/kernels/partition.hip)."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import idx_dtype, is_gpu, launch, ptr, stream, to_host_ints

DATE_FIELDS = {"year": 0, "month": 1, "day": 2, "quarter": 3, "dow": 4, "doy": 5}


# ------------------------------------------------------------------ partition
def _mix64_np(k: np.ndarray) -> np.ndarray:
    k = k.astype(np.uint64)
    with np.errstate(over="ignore"):
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xFF51AFD7ED558CCD)
        k ^= k >> np.uint64(33)
        k *= np.uint64(0xC4CEB9FE1A85EC53)
        k ^= k >> np.uint64(33)
    return k


def partition_ids(keys: torch.Tensor, nparts: int) -> torch.Tensor:
    """Destination partition of each row: mix64(key) % nparts (same on CPU and GPU)."""
    n = keys.numel()
    if not is_gpu(keys):
        h = _mix64_np(keys.cpu().numpy().astype(np.int64).view(np.uint64))
        return torch.from_numpy((h % np.uint64(nparts)).astype(np.int32))
    out = torch.empty(n, dtype=torch.int32, device=keys.device)
    launch("partition_ids").partition_ids(ptr(keys), keys.dtype == torch.int64, n, nparts, ptr(out), stream(out))
    return out


def hash_partition(keys: torch.Tensor, nparts: int) -> Tuple[torch.Tensor, List[int]]:
    """Stable permutation grouping rows by destination + rows per destination."""
    keys = keys.contiguous()
    n = keys.numel()
    if nparts == 1:
        return torch.arange(n, dtype=idx_dtype(n), device=keys.device), [n]
    if not is_gpu(keys):
        pid = partition_ids(keys, nparts).to(torch.int64)
        perm = torch.sort(pid, stable=True).indices.to(idx_dtype(n))
        counts = torch.bincount(pid, minlength=nparts).tolist()
        return perm, counts
    N = launch("partition")
    blocks = N.partition_run_blocks(n)
    ws = torch.empty(nparts * blocks + 1, dtype=torch.int64, device=keys.device)
    it = idx_dtype(n)
    perm = torch.empty(n, dtype=it, device=keys.device)
    N.partition_run(ptr(keys), keys.dtype == torch.int64, n, nparts, ptr(ws), ptr(ws) + 8 * nparts * blocks,
                    ptr(perm), it == torch.int64, stream(keys))
    starts = to_host_ints(ws[: nparts * blocks].view(nparts, blocks)[:, 0])
    counts = [(starts[p + 1] if p + 1 < nparts else n) - starts[p] for p in range(nparts)]
    return perm, counts


# ------------------------------------------------------------------ date parts
def date_part(days: torch.Tensor, field: str) -> torch.Tensor:
    f = DATE_FIELDS[field]
    n = days.numel()
    if not is_gpu(days):
        d = days.cpu().numpy().astype("int64").astype("datetime64[D]")
        if field == "year":
            r = d.astype("datetime64[Y]").astype(np.int64) + 1970
        elif field == "month":
            r = d.astype("datetime64[M]").astype(np.int64) % 12 + 1
        elif field == "day":
            r = (d - d.astype("datetime64[M]")).astype(np.int64) + 1
        elif field == "quarter":
            r = (d.astype("datetime64[M]").astype(np.int64) % 12) // 3 + 1
        elif field == "dow":
            r = (days.cpu().numpy().astype(np.int64) % 7 + 7 + 4) % 7
        else:
            r = (d - d.astype("datetime64[Y]")).astype(np.int64) + 1
        return torch.from_numpy(r.astype(np.int32))
    days = days.contiguous().to(torch.int32)
    out = torch.empty(n, dtype=torch.int32, device=days.device)
    launch("date_part").date_part(ptr(days), n, f, ptr(out), stream(out))
    return out


# ---------------------------------------------------------------------- sorting
def argsort_keys(keys: Sequence[Tuple[torch.Tensor, bool, bool, Optional[torch.Tensor]]], n: int,
                 device) -> torch.Tensor:
    """Lexicographic stable argsort. keys: (values, descending, nulls_first, valid).
    GPU: packed keys + the radix sort of ops/sort.py; values must be numeric
    (strings are turned into order-preserving ranks by the caller)."""
    from .sort import argsort
    return argsort(keys, n, device)
