"""roctx ranges for rocprofv3 timelines (``IGLOO_DEBUG=roctx``).

Every physical operator's execution, every EXPLAIN-ANALYZE phase span and
every query become named ranges in the marker trace
(``rocprofv3 --marker-trace --kernel-trace``), so kernels line up with the
operator that launched them. Loaded through ctypes from ROCm's libroctx64;
with the variable unset (the default) the hooks are a constant-False check.
"""
from __future__ import annotations

from ..utils import switches as _sw
import ctypes
import os

ENABLED = _sw.debug("roctx")
_lib = None


def _load():
    global _lib, ENABLED
    if _lib is None:
        # the rocprofiler-sdk roctx first: rocprofv3 --marker-trace records its ranges
        for name in ("/opt/rocm/lib/librocprofiler-sdk-roctx.so", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except (OSError, AttributeError):
                continue
        if _lib is None:
            ENABLED = False
    return _lib


def push(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxRangePushA(name.encode()[:200])


def pop() -> None:
    if ENABLED and _lib is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxMarkA(name.encode()[:200])


class Range:
    """``with trace.Range("query Q1"): ...``"""

    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        push(self.name)
        return self

    def __exit__(self, *exc):
        pop()
        return False
