"""Loader for the native extension and launch helpers.

On a GPU tensor every op in ``igloo_amd.ops`` runs a hand-written gfx950
kernel from ``_native``; if the extension is missing the op raises
``DeviceError`` instead of silently falling back. CPU tensors take a
torch/pyarrow reference path (used by the CPU test-suite and as the numerics
oracle for the GPU tests).
"""
from __future__ import annotations

import collections
import os

import torch

from ..utils.errors import DeviceError

_native = None
_native_err = None
# per-kernel launch counters: tests assert the native path actually ran
KERNEL_CALLS: "collections.Counter[str]" = collections.Counter()


def native():
    global _native, _native_err
    if _native is None:
        if _native_err is not None:
            raise DeviceError(_native_err)
        try:
            from .. import _native as n  # noqa: F401  (torch already imported: shares its HIP runtime)
            _native = n
        except ImportError as e:  # pragma: no cover - exercised only on broken installs
            _native_err = f"igloo native extension not built/loadable: {e}. Run `python -m igloo_amd._build`."
            raise DeviceError(_native_err) from e
    return _native


def have_native() -> bool:
    try:
        native()
        return True
    except DeviceError:
        return False


def is_gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def launch(name: str):
    """Record a native launch (cheap counter) and return the native module."""
    KERNEL_CALLS[name] += 1
    return native()


def idx_dtype(n: int) -> torch.dtype:
    return torch.int32 if n < 2**31 - 1 else torch.int64


SYNC_CHECK = os.environ.get("IGLOO_SYNC_CHECK", "0") not in ("", "0")
