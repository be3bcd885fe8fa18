"""Change data capture: table versions, change events, cache invalidation.

Parity: the reference's CDC crate is empty (reference crates/cdc/src/lib.rs:9
"TODO: Implement CDC logic") while its README promises "transparent caching
layer with automatic cache invalidation via CDC" (README.md:42).

Model: every registered table has a monotonically increasing version
(watermark). Versions advance either by *pushed* change events
(``apply_event`` — e.g. from a Postgres logical-replication consumer) or by
*polling* a version probe (Iceberg current-snapshot-id, file mtimes, a
Postgres ``max(xmin)`` / ``max(updated_at)`` query). When a table's version
changes, every cache entry under that table's prefix is invalidated and
subscribers are notified. ``CachedTable`` wraps any source so scans are
served from the HBM tier until the source changes.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..catalog import TableSource
from ..columnar import Batch
from ..utils.log import get_logger
from .tiered import TieredCache

log = get_logger("cdc")


@dataclass
class ChangeEvent:
    table: str
    op: str                 # insert | update | delete | truncate | snapshot
    version: Any = None     # source position (LSN, snapshot id, ...)
    rows: Optional[list] = None
    ts: float = field(default_factory=time.time)


class CdcManager:
    def __init__(self, cache: Optional[TieredCache] = None):
        self.cache = cache
        self._lock = threading.RLock()
        self._versions: Dict[str, Any] = {}
        self._probes: Dict[str, Callable[[], Any]] = {}
        self._subs: List[Callable[[ChangeEvent], None]] = []
        self.events: List[ChangeEvent] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ---------------------------------------------------------- registration
    def track(self, table: str, probe: Optional[Callable[[], Any]] = None, version: Any = 0):
        with self._lock:
            self._versions[table] = probe() if probe is not None else version
            if probe is not None:
                self._probes[table] = probe

    def version(self, table: str) -> Any:
        with self._lock:
            return self._versions.get(table)

    def subscribe(self, fn: Callable[[ChangeEvent], None]):
        self._subs.append(fn)

    # -------------------------------------------------------------- changes
    def apply_event(self, ev: ChangeEvent):
        with self._lock:
            cur = self._versions.get(ev.table, 0)
            nv = ev.version if ev.version is not None else (cur + 1 if isinstance(cur, int) else time.time())
            self._versions[ev.table] = nv
            self.events.append(ev)
        self._invalidate(ev.table)
        for s in self._subs:
            s(ev)

    def poll(self) -> List[str]:
        """Re-run every version probe; returns tables whose version changed."""
        changed = []
        for t, probe in list(self._probes.items()):
            try:
                v = probe()
            except Exception as e:  # noqa: BLE001 - a failing probe must not kill the poller
                log.warning("cdc probe for %s failed: %s", t, e)
                continue
            if v != self._versions.get(t):
                self.apply_event(ChangeEvent(t, "snapshot", v))
                changed.append(t)
        return changed

    def start(self, interval_s: float = 5.0):
        if self._thread is not None:
            return

        def loop():
            while not self._stop.wait(interval_s):
                self.poll()
        self._thread = threading.Thread(target=loop, daemon=True, name="igloo-cdc")
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def _invalidate(self, table: str):
        if self.cache is not None:
            n = self.cache.invalidate(f"{table}/")
            log.info("cdc: %s changed, invalidated %d cache entries", table, n)


class CachedTable(TableSource):
    """Serve scans of ``source`` from the HBM cache tier, keyed by the CDC version."""

    def __init__(self, name: str, source: TableSource, cache: TieredCache, cdc: Optional[CdcManager] = None):
        self.name = name
        self.source = source
        self.cache = cache
        self.cdc = cdc
        self.partitioned_by = getattr(source, "partitioned_by", None)
        self.replicated = getattr(source, "replicated", False)
        if cdc is not None and cdc.version(name) is None:
            probe = (lambda s=source: getattr(s, "version", None)) if hasattr(source, "version") else None
            cdc.track(name, probe)

    def schema(self):
        return self.source.schema()

    def num_rows(self):
        return self.source.num_rows()

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        ver = self.cdc.version(self.name) if self.cdc is not None else None
        rank = ctx.comm.rank if ctx is not None and ctx.comm is not None else 0
        out, n, missing = {}, None, []
        for c in columns:
            hit = self.cache.get(f"{self.name}/{rank}/{c}", ver)
            if hit is None:
                missing.append(c)
            else:
                out[c] = hit.columns[c]
                n = hit.num_rows
        if missing:
            b = self.source.scan(missing, ctx)
            for c in missing:
                self.cache.put(f"{self.name}/{rank}/{c}", Batch({c: b.columns[c]}, b.num_rows), ver)
                out[c] = b.columns[c]
            n = b.num_rows
        return Batch({c: out[c] for c in columns}, n if n is not None else 0)
