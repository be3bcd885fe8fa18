"""Fault injection for failure-detection / recovery tests.

The reference has no fault injection at all: worker liveness is a heartbeat
the coordinator never checks (crates/worker/src/main.rs:29-41,
crates/coordinator/src/service.rs:37-50) and any fragment error fails the
whole query (crates/coordinator/src/distributed_executor.rs:80-83). Here the
recovery paths (heartbeat eviction, query retry on another worker group,
typed device / comm errors) are exercised by faults named in ``IGLOO_FAULT``
(or the ``fault`` config key, or :func:`inject` in tests):

    IGLOO_FAULT="drop_heartbeat;kernel_error@join_probe:1;comm_timeout@all_to_all_v"

Each entry is ``kind[@target][:count]``; without ``:count`` it fires every
time. Kinds and the hook that consumes them:

* ``drop_heartbeat[@worker-id-prefix]`` — the worker skips heartbeats, so the
  coordinator's reaper evicts it (service/worker.py);
* ``fail_query[@sql-substring]`` — a worker group fails the query with a
  DeviceError (Flight "unavailable"), so the coordinator marks it dead and
  retries on another group (service/worker.py, service/coordinator.py);
* ``kill_worker`` — the worker process exits (status 17) at its next query;
* ``kernel_error@<native op>`` — ``ops._lib.launch(<op>)`` raises DeviceError
  before launching (a simulated GPU fault, surfaced like a real one);
* ``comm_timeout[@<collective>]`` — a Communicator collective raises CommError
  (parallel/comm.py).
"""
from __future__ import annotations

import os
import threading
from contextlib import contextmanager
from dataclasses import dataclass
from typing import List, Optional

KINDS = ("drop_heartbeat", "fail_query", "kill_worker", "kernel_error", "comm_timeout")


@dataclass
class Fault:
    kind: str
    target: Optional[str] = None
    remaining: Optional[int] = None   # None = unlimited
    fired: int = 0

    def matches(self, kind: str, target: Optional[str]) -> bool:
        if self.kind != kind or self.remaining == 0:
            return False
        if self.target is None:
            return True
        if target is None:
            return False
        if kind == "fail_query":
            return self.target in target
        if kind == "drop_heartbeat":
            return target.startswith(self.target)
        return self.target == target


def parse(spec: Optional[str]) -> List[Fault]:
    out = []
    for item in (spec or "").replace(",", ";").split(";"):
        item = item.strip()
        if not item:
            continue
        count = None
        head = item
        if ":" in item.rsplit("@", 1)[-1]:
            head, c = item.rsplit(":", 1)
            count = int(c)
            if count < 0:
                raise ValueError(f"IGLOO_FAULT: negative count in {item!r}")
        kind, _, target = head.partition("@")
        kind = kind.strip()
        if kind not in KINDS:
            raise ValueError(f"IGLOO_FAULT: unknown fault kind {kind!r} (one of {', '.join(KINDS)})")
        out.append(Fault(kind, target.strip() or None, count))
    return out


_lock = threading.Lock()
_faults: List[Fault] = parse(os.environ.get("IGLOO_FAULT"))
ACTIVE = bool(_faults)   # read by hot paths: one attribute test when no fault is configured


def configure(spec: Optional[str]) -> List[Fault]:
    """Replace the active fault set (None/"" clears it)."""
    global _faults, ACTIVE
    with _lock:
        _faults = parse(spec)
        ACTIVE = bool(_faults)
        return list(_faults)


def active() -> List[Fault]:
    with _lock:
        return list(_faults)


def fire(kind: str, target: Optional[str] = None) -> bool:
    """True when a configured fault of ``kind`` (and target) should fire now;
    consumes one of its counts."""
    if not ACTIVE:
        return False
    with _lock:
        for f in _faults:
            if f.matches(kind, target):
                f.fired += 1
                if f.remaining is not None:
                    f.remaining -= 1
                return True
    return False


def check(kind: str, target: Optional[str] = None):
    """Raise the error a real failure of this kind surfaces as."""
    if not fire(kind, target):
        return
    from .errors import CommError, DeviceError
    what = f"{kind}@{target}" if target else kind
    if kind in ("kernel_error", "fail_query"):
        raise DeviceError(f"injected fault {what}: kernel launch failed")
    if kind == "comm_timeout":
        raise CommError(f"injected fault {what}: collective timed out")
    if kind == "kill_worker":
        os._exit(17)
    raise AssertionError(kind)


@contextmanager
def inject(spec: str):
    """Test helper: activate ``spec`` for the duration of the block."""
    prev = ";".join(f"{f.kind}{'@' + f.target if f.target else ''}"
                    f"{'' if f.remaining is None else ':' + str(f.remaining)}" for f in active())
    configure(spec)
    try:
        yield
    finally:
        configure(prev)
