"""HBM accounting for resident columns and the structures derived from them.

Resident table columns carry derived structures built on first use and kept
with the column tensor like an index (attributes set by the operators):

* ``_igloo_narrow``  narrow integer copy read by the fused scans (exec/fused.py);
* ``_igloo_perm``    secondary index: sorted keys + row permutation (ops/hashing.py);
* ``_igloo_dense``   dense lower-bound range index of a sorted key column;
* ``_igloo_hll``     HyperLogLog registers (4 KB);
* ``_igloo_fence``   every 256th key of a sorted column (binary-search fence);
* ``_igloo_packed``  row-packed copies of column sets for sparse gathers
  (ops/packed_gather.py), kept on the set's first column.

The cache tier (cache/tiered.py) charges them to the column that owns them,
so the HBM budget covers what the table really holds, and evicting a column
drops its derived structures with it.
"""
from __future__ import annotations

from typing import Iterable

import torch

DERIVED_ATTRS = ("_igloo_narrow", "_igloo_perm", "_igloo_dense", "_igloo_hll", "_igloo_fence", "_igloo_packed")


def _tensor_bytes(x) -> int:
    if isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, (tuple, list)):
        return sum(_tensor_bytes(v) for v in x)
    return 0


def derived_nbytes(t: torch.Tensor) -> int:
    """Bytes held by the derived structures attached to ``t``."""
    n = 0
    for a in DERIVED_ATTRS:
        v = getattr(t, a, None)
        if v is None or v is t or v is False:
            continue
        n += _tensor_bytes(v)
        if a == "_igloo_perm" and isinstance(v, tuple) and v and isinstance(v[0], torch.Tensor):
            n += derived_nbytes(v[0])     # the index keys' own dense table
    return n


def column_nbytes(col) -> int:
    """Bytes of a Column including the derived structures of its data tensor."""
    return col.nbytes + derived_nbytes(col.data)


def batch_nbytes(cols: Iterable) -> int:
    return sum(column_nbytes(c) for c in cols)


def drop_derived(t: torch.Tensor) -> None:
    for a in DERIVED_ATTRS:
        if hasattr(t, a):
            try:
                delattr(t, a)
            except (AttributeError, RuntimeError):
                pass


def device_capacity(device) -> int:
    """Total memory of ``device`` in bytes (0 for the CPU)."""
    device = torch.device(device)
    if device.type != "cuda":
        return 0
    try:
        return torch.cuda.get_device_properties(device).total_memory
    except (RuntimeError, AssertionError):
        return 0
