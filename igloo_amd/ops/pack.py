"""Row packing of several columns into one byte matrix (csrc/kernels/pack.hip),
so an exchange moves every fixed-width column (values, validity bytes,
string lengths, dictionary codes) with ONE collective."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from ._lib import is_gpu, launch, ptr, stream

Layout = Tuple[int, List[Tuple[int, int, int]]]   # (row bytes, [(tensor index, width, offset)])


def _width(t: torch.Tensor) -> int:
    return t.element_size() * (t.shape[1] if t.dim() == 2 else 1)


def layout(tensors: Sequence[torch.Tensor]) -> Layout:
    """Fields widest first (natural alignment), rows padded to 8 bytes."""
    order = sorted(range(len(tensors)), key=lambda i: -_width(tensors[i]))
    fields, off = [], 0
    for i in order:
        w = _width(tensors[i])
        fields.append((i, w, off))
        off += w
    return (off + 7) // 8 * 8, fields


def pack_rows(tensors: Sequence[torch.Tensor], perm: Optional[torch.Tensor], n: int,
              lay: Optional[Layout] = None) -> Tuple[torch.Tensor, Layout]:
    """uint8 [n, row_bytes]: row i holds every tensor's value at perm[i] (or i)."""
    lay = lay or layout(tensors)
    rb, fields = lay
    dev = tensors[0].device if tensors else torch.device("cpu")
    out = torch.empty((n, rb), dtype=torch.uint8, device=dev)
    if n == 0 or not fields:
        return out, lay
    if not is_gpu(out):
        idx = perm.long() if perm is not None else None
        for i, w, off in fields:
            t = tensors[i].contiguous()
            if idx is not None:
                t = t.index_select(0, idx)
            out[:, off:off + w] = t.reshape(n, -1).view(torch.uint8).reshape(n, w)
        return out, lay
    srcs = [tensors[i].contiguous() for i, _, _ in fields]
    cols = [(ptr(s), 0, w, off) for s, (_, w, off) in zip(srcs, fields)]
    launch("pack_rows").pack_rows(cols, rb, ptr(perm), perm is not None and perm.dtype == torch.int64, n, ptr(out),
                                  stream(out))
    return out, lay


def unpack_rows(packed: torch.Tensor, lay: Layout, like: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Split a packed [n, row_bytes] matrix back into tensors shaped/typed like ``like``."""
    rb, fields = lay
    n = packed.shape[0]
    outs: List[Optional[torch.Tensor]] = [None] * len(like)
    for i, _, _ in fields:
        t = like[i]
        outs[i] = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=packed.device)
    if n == 0 or not fields:
        return outs
    if not is_gpu(packed):
        for i, w, off in fields:
            outs[i].reshape(n, -1).view(torch.uint8).reshape(n, w).copy_(packed[:, off:off + w])
        return outs
    cols = [(0, ptr(outs[i]), w, off) for i, w, off in fields]
    launch("unpack_rows").unpack_rows(cols, rb, ptr(packed.contiguous()), n, stream(packed))
    return outs
