"""Loader for the native extension and launch helpers.

On a GPU tensor every op in ``igloo_amd.ops`` runs a hand-written gfx950
kernel from ``_native``; if the extension is missing the op raises
``DeviceError`` instead of silently falling back. CPU tensors take a
torch/pyarrow reference path (used by the CPU test-suite and as the numerics
oracle for the GPU tests).
"""
from __future__ import annotations

from ..utils import switches as _sw
import collections
import os
import sys
import threading

import torch

from ..utils import faults as _faults
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


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream(t: torch.Tensor) -> int:
    """Handle of the current HIP stream of ``t``'s device (inside a capture:
    the capture stream). The raw-handle query skips building a Stream
    object per launch (~5 us each, ~1000 launches per fresh query suite)."""
    d = t.device.index
    if _raw_stream is not None and d is not None:
        return _raw_stream(d)
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def launch(name: str):
    """Record a native launch (cheap counter) and return the native module."""
    KERNEL_CALLS[name] += 1
    if _faults.ACTIVE:
        _faults.check("kernel_error", name)
    return native()


def idx_dtype(n: int) -> torch.dtype:
    return torch.int32 if n < 2**31 - 1 else torch.int64


SYNC_CHECK = _sw.debug("sync_check")


# ------------------------------------------------------------------ host readback
_SENTINEL = -0x5A5A5A5A5A5A5A5B
_pinned = threading.local()
# polled pinned readback: ~48 us less per sync in isolation (scripts/sync_bench.py) but no gain on the
# SF100 suite (A/B 0.228 vs 0.226 s), so off by default
FAST_READBACK = False


def _pinned_buf(n: int) -> torch.Tensor:
    buf = getattr(_pinned, "buf", None)
    if buf is None or buf.numel() < n:
        buf = torch.empty(max(n, 64), dtype=torch.int64, pin_memory=True)
        _pinned.buf = buf
    return buf


def _distributed() -> bool:
    d = torch.distributed
    return d.is_available() and d.is_initialized()


class CaptureAbort(RuntimeError):
    """Raised while a query is being captured into a HIP graph
    (exec/graphs.py) at anything a graph cannot replay: a real host readback,
    a one-time build of a derived structure, a generated-kernel load, a spill
    to host memory. Raised before any HIP call, so the capture ends cleanly
    and the query runs eagerly."""


_capture = threading.local()


def capturing() -> bool:
    """This thread is capturing a query graph."""
    return getattr(_capture, "on", False)


def set_capturing(on: bool) -> None:
    _capture.on = on


#: host steps a GPU query took (name -> count): work that left the device
#: (exec/expr_eval.py, ops/strings.py); EXPLAIN ANALYZE lists them and the GPU
#: tests assert the TPC-H / reference-compat queries take none
HOST_STEPS: "collections.Counter[str]" = collections.Counter()


def note_host_step(what: str) -> None:
    HOST_STEPS[what] += 1


def device_ints(values, device, dtype=torch.int64) -> torch.Tensor:
    """Host ints -> a device tensor without a synchronizing copy: staged in
    pinned memory and copied stream-ordered; under graph capture (where the
    runtime refuses host-to-device copies) written by a kernel whose
    arguments carry the values."""
    if torch.device(device).type != "cuda":
        return torch.tensor(values, dtype=dtype, device=device)
    if getattr(_capture, "on", False):
        # inside a graph capture: the values travel as kernel arguments
        vals = [int(v) for v in values]
        out = torch.empty(len(vals), dtype=torch.int64, device=device)
        if vals:
            launch("const_ints").const_ints(out.data_ptr(), vals, torch.cuda.current_stream(out.device).cuda_stream)
        return out if dtype == torch.int64 else out.to(dtype)
    h = torch.tensor(values, dtype=dtype).pin_memory()
    return h.to(device, non_blocking=True)


def capture_hold(obj) -> None:
    """Keep ``obj`` (a device buffer a captured kernel reads, e.g. a cached
    pattern constant) alive as long as the graph being captured."""
    if getattr(_capture, "on", False):
        keep = getattr(_capture, "keep", None)
        if keep is None:
            keep = _capture.keep = []
        keep.append(obj)


def capture_keepalive() -> list:
    """Host buffers the current capture's graph reads (cleared per capture)."""
    keep = getattr(_capture, "keep", None) or []
    _capture.keep = []
    return keep


def check_not_capturing(what: str) -> None:
    if getattr(_capture, "on", False):
        raise CaptureAbort(what)


class Speculation:
    """Host readbacks of one query execution, recorded or replayed.

    A query's host-side control flow (output sizes, key ranges, strategy
    choices) depends only on the plan and the data, and every such value
    reaches the host through ``to_host_ints``. ``record`` keeps each value
    with its call site; ``replay`` hands the recorded value back at once (no
    device sync: the host keeps launching while the GPU works) and queues a
    device-side copy of the real value; ``validate`` compares all of them with
    one sync at the end of the query. A call-site mismatch ends speculation
    for the rest of the query (real readbacks from there on) and the query's
    recording is
    re-recorded; any value mismatch re-executes the query. engine.py keys
    recordings on the plan, the catalog version and the cache generation, and
    trusts one only after two executions produced the same call sequence;
    values that differed between those two (non-deterministic intermediates,
    e.g. hash-assigned ids) are marked volatile (``None``) and always read back.
    """

    __slots__ = ("mode", "log", "pos", "actual", "expected", "diverged", "checked", "fresh")

    def __init__(self, mode: str, log: list = None):
        self.mode = mode
        self.log = log if log is not None else []
        self.pos = 0
        self.actual: list = []
        self.expected: list = []
        self.diverged = False
        self.checked = 0
        self.fresh: list = []   # replay: this run's own (site, values) sequence
    @property
    def complete(self) -> bool:
        """The replay followed the recorded call sequence to its end."""
        return not self.diverged and self.pos == len(self.log)

    def expected_values(self) -> list:
        """Every non-volatile value of the recorded log, in call order: what a
        complete replay hands out (and what the device must confirm)."""
        out = []
        for _site, vals in self.log:
            if vals is not None:
                out.extend(vals)
        return out

    def device_mismatches(self, expected_dev: torch.Tensor) -> torch.Tensor:
        """Device int64 scalar: how many replayed values differ from the device
        (stream-ordered, no sync; used inside a graph capture)."""
        if not self.actual:
            return torch.zeros((), dtype=torch.int64, device=expected_dev.device)
        act = torch.cat(self.actual)
        if act.numel() != expected_dev.numel():
            raise CaptureAbort("replayed value count differs from the recording")
        self.actual = [act]      # kept: a mismatch report reads the device values back
        return (act != expected_dev).sum()

    def mismatch_sites(self, act: list) -> list:
        """(file:line, replayed, device) of every replayed value that differs."""
        out, pos = [], 0
        for site, vals in self.log:
            if vals is None:
                continue
            got = act[pos:pos + len(vals)]
            if got != list(vals):
                code, line = site[0]
                out.append((f"{code.co_filename.split('igloo_amd/')[-1]}:{line}", list(vals)[:4], got[:4]))
            pos += len(vals)
        return out

    def validate(self) -> bool:
        """True when every replayed value equals the device value (one sync).
        Values handed out before a divergence were replayed at matching call
        sites; after it, readbacks were real - so a diverged run is still
        correct when this holds (its recording just needs refreshing)."""
        if self.mode != "replay":
            return True
        if not self.actual:
            return True
        dev = self.actual[0].device
        act = torch.cat(self.actual)
        exp = torch.tensor(self.expected, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        self.checked = act.numel()
        ok = bool((act == exp).all().item())
        if not ok and _sw.debug("spec"):
            a, pos = act.tolist(), 0
            for (site, vals) in self.log[:self.pos]:
                if vals is None:
                    continue
                got = a[pos:pos + len(vals)]
                if got != list(vals):
                    code, line = site[0]
                    print(f"[speculation] {code.co_filename}:{line} ({code.co_name}) replayed {list(vals)[:8]} "
                          f"device {got[:8]}", flush=True)
                pos += len(vals)
        return ok


_spec = threading.local()


def set_speculation(s: "Speculation | None") -> None:
    _spec.cur = s


class unlogged:
    """Readbacks inside are real and stay out of the speculation log: used
    around the one-time builds of derived structures remembered on resident
    columns (stats, sortedness, indexes, sketches, narrow copies), so the
    first execution of a query records the same readback sequence as the
    later ones that find those structures cached."""

    __slots__ = ("prev",)

    def __enter__(self):
        check_not_capturing("one-time build of a derived structure")
        self.prev = getattr(_spec, "cur", None)
        _spec.cur = None
        return self

    def __exit__(self, *exc):
        _spec.cur = self.prev
        return False


def _site() -> tuple:
    f = sys._getframe(2)
    if f.f_code is to_host_int.__code__ or f.f_code is to_host_f64s.__code__:
        f = f.f_back
    return (f.f_code, f.f_lineno)


def to_host_ints(t: torch.Tensor) -> list:
    sp = getattr(_spec, "cur", None)
    if sp is None or not t.is_cuda:
        return _to_host_ints(t)
    site = (_site(), t.numel())
    if sp.mode == "record":
        v = _to_host_ints(t)
        sp.log.append((site, v))
        return v
    if not sp.diverged and sp.pos < len(sp.log) and sp.log[sp.pos][0] == site:
        v = sp.log[sp.pos][1]
        sp.pos += 1
        if v is None:                  # volatile site: differs between runs, always read for real
            v = _to_host_ints(t)
            sp.fresh.append((site, v))
            return v
        # a reference, not a copy: the tensor stays alive (its memory is not
        # reused) and readback sources are not written again after being read
        # (a copy per value was ~700 D2D copy launches per SF100 suite); a
        # source that were overwritten would fail validation, never pass it
        a = t.reshape(-1)
        sp.actual.append(a if a.dtype == torch.int64 else a.to(torch.int64))
        sp.expected.extend(v)
        sp.fresh.append((site, v))
        return list(v)
    sp.diverged = True
    v = _to_host_ints(t)
    sp.fresh.append((site, v))
    return v


#: blocking device -> host readbacks so far (engine.py reports them per query)
READBACKS = [0]


def _to_host_ints(t: torch.Tensor) -> list:
    """Small int device tensor -> Python ints with one stream-ordered copy into
    pinned memory that the host polls, instead of ``.item()`` / ``.tolist()``
    (a blocking D2H copy + stream synchronize: ~66 us per call on MI355X vs
    ~18 us polled; a query issues ~25 data-dependent sizes). Values are exact:
    the poll ends on a changed sentinel or an idle stream, whichever first."""
    if t.is_cuda:
        check_not_capturing("host readback")
        READBACKS[0] += 1
    # single-process only: a 2-rank run sharing one GPU hung in its first query
    # with polled readbacks (cause not isolated), so SPMD ranks keep .tolist()
    if not t.is_cuda or not FAST_READBACK or _distributed():
        return [int(v) for v in t.reshape(-1).tolist()]
    n = t.numel()
    if n == 0:
        return []
    buf = _pinned_buf(n)
    view = buf.numpy()
    view[:n] = _SENTINEL
    src = t.reshape(-1).to(torch.int64)
    buf[:n].copy_(src, non_blocking=True)
    st = torch.cuda.current_stream(t.device)
    spins = 0
    pending = (lambda: view[0] == _SENTINEL) if n == 1 else (lambda: bool((view[:n] == _SENTINEL).any()))
    while pending():
        spins += 1
        if spins % 256 == 0 and st.query():
            break
    return [int(v) for v in view[:n]]


def to_host_int(t: torch.Tensor) -> int:
    return to_host_ints(t)[0]


def to_host_f64s(t: torch.Tensor) -> list:
    """Small float device tensor -> Python floats (bit-exact, via to_host_ints)."""
    import numpy as np
    bits = to_host_ints(t.reshape(-1).to(torch.float64).view(torch.int64))
    return np.array(bits, dtype=np.int64).view(np.float64).tolist()
