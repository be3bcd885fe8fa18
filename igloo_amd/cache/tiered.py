"""Tiered result/column cache: HBM -> host memory -> disk (Arrow IPC).

Parity: reference crates/cache/src/lib.rs — ``Cache`` is an async
RwLock<HashMap<String, Vec<RecordBatch>>> whose ``get`` clones on hit (info! hit
/ warn! miss) and ``put`` overwrites, with no eviction and an unused
``CacheConfig { capacity }`` (:12-56); ``InMemoryCache`` is a String->String map
whose ``get`` errors with "Key not found" (:59-87).

Here the same API is backed by three byte-capped LRU tiers sized for an
MI355X (default HBM tier 64 GiB of the 288 GB): device-resident Batches are
demoted to host memory (Arrow) and then spilled to Arrow IPC files, and
promoted back on hit. Entries carry a version (table snapshot / CDC
watermark) so stale entries are never returned.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import threading
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple, Union

import pyarrow as pa
import pyarrow.ipc as ipc
import torch

from ..columnar import Batch, Column
from ..utils.errors import IglooError
from ..utils.log import get_logger
from ..utils.memory import batch_nbytes

log = get_logger("cache")
GiB = 1 << 30


@dataclass
class CacheConfig:
    capacity: Optional[int] = None          # reference field: max entries (None = unbounded)
    hbm_bytes: int = 64 * GiB
    host_bytes: int = 32 * GiB
    disk_path: Optional[str] = None         # None = no disk tier
    disk_bytes: int = 1 << 40
    device: str = "cpu"


Value = Union[List[pa.RecordBatch], pa.Table, Batch]


def _nbytes(v) -> int:
    if isinstance(v, Batch):
        # device columns are charged with their derived structures (narrow
        # copies, secondary / range indexes) — utils/memory.py
        return batch_nbytes(v.columns.values())
    if isinstance(v, pa.Table):
        return v.nbytes
    if isinstance(v, list):
        return sum(b.nbytes for b in v)
    return 0


def _to_table(v) -> pa.Table:
    if isinstance(v, pa.Table):
        return v
    if isinstance(v, Batch):
        return v.to_arrow()
    if isinstance(v, list):
        return pa.Table.from_batches(v) if v else pa.table({})
    raise TypeError(type(v))


class TieredCache:
    def __init__(self, config: Optional[CacheConfig] = None):
        self.config = config or CacheConfig()
        self._lock = threading.RLock()
        self._hbm: "OrderedDict[str, Tuple[Any, Any, int]]" = OrderedDict()   # key -> (value, version, bytes)
        self._host: "OrderedDict[str, Tuple[pa.Table, Any, int, str]]" = OrderedDict()  # kind: batch|batches|table
        self._disk: "OrderedDict[str, Tuple[str, Any, int, str]]" = OrderedDict()
        self.stats = {"hits": 0, "misses": 0, "evictions": 0, "spills": 0, "promotions": 0}
        #: bumped whenever cached data changes identity (replace / drop / evict /
        #: re-materialise from a lower tier; adding a new key does not);
        #: engine.py keys replayed query readbacks on it
        self.generation = 0
        self._dir = None
        if self.config.disk_path:
            os.makedirs(self.config.disk_path, exist_ok=True)
            self._dir = self.config.disk_path

    # ---------------------------------------------------------------- sizes
    def _used(self, tier) -> int:
        if tier is self._hbm:
            # derived structures attach to resident columns after ``put``:
            # re-measure device entries every time
            return sum(_nbytes(e[0]) for e in tier.values())
        return sum(e[2] for e in tier.values())

    def enforce(self) -> None:
        """Re-apply the byte budgets (after queries grew derived structures)."""
        with self._lock:
            self._enforce()

    @property
    def hbm_used(self) -> int:
        return self._used(self._hbm)

    @property
    def host_used(self) -> int:
        return self._used(self._host)

    def __len__(self):
        return len(self._hbm) + len(self._host) + len(self._disk)

    def __contains__(self, key):
        return key in self._hbm or key in self._host or key in self._disk

    # ---------------------------------------------------------------- API
    def put(self, key: str, value: Value, version: Any = None) -> None:
        with self._lock:
            if key in self:
                self._drop(key)   # replaced data: _drop bumps the generation
            nb = _nbytes(value)
            if isinstance(value, Batch):
                self._hbm[key] = (value, version, nb)
            else:
                kind = "batches" if isinstance(value, list) else "table"
                self._host[key] = (_to_table(value), version, nb, kind)
            self._enforce()

    def get(self, key: str, version: Any = None) -> Optional[Value]:
        with self._lock:
            for tier in (self._hbm, self._host, self._disk):
                if key in tier:
                    e = tier[key]
                    if version is not None and e[1] != version:
                        self._drop(key)
                        break
                    tier.move_to_end(key)
                    self.stats["hits"] += 1
                    log.info("cache hit %s", key)
                    return self._materialise(key, tier, e)
            self.stats["misses"] += 1
            log.info("cache miss %s", key)
            return None

    def touch(self, keys) -> None:
        """Mark HBM entries as just used (a query graph replay reads them
        without going through ``get``)."""
        with self._lock:
            for k in keys:
                if k in self._hbm:
                    self._hbm.move_to_end(k)

    def invalidate(self, prefix: str = "") -> int:
        with self._lock:
            keys = [k for k in list(self._hbm) + list(self._host) + list(self._disk) if k.startswith(prefix)]
            for k in keys:
                self._drop(k)
            return len(keys)

    def clear(self):
        self.invalidate("")

    # ------------------------------------------------------------ internals
    def _materialise(self, key, tier, e):
        if tier is self._hbm:
            return e[0]
        self.generation += 1     # a fresh copy of the data (new device tensors)
        if tier is self._host:
            t, ver, nb, kind = e
        else:
            path, ver, nb, kind = e
            with ipc.open_file(path) as r:
                t = r.read_all()
            del self._disk[key]
            try:
                os.remove(path)
            except OSError:
                pass
            self._host[key] = (t, ver, nb, kind)
            self.stats["promotions"] += 1
            self._enforce()
        if kind == "batches":
            return t.to_batches()
        if kind == "batch":
            return Batch.from_arrow(t, device=self.config.device)
        return t

    def _drop(self, key):
        self.generation += 1
        self._hbm.pop(key, None)
        self._host.pop(key, None)
        e = self._disk.pop(key, None)
        if e is not None:
            try:
                os.remove(e[0])
            except OSError:
                pass

    def _enforce(self):
        cfg = self.config
        while self._hbm and self._used(self._hbm) > cfg.hbm_bytes:
            k, (v, ver, nb) = self._hbm.popitem(last=False)
            t = v.to_arrow()
            self._host[k] = (t, ver, t.nbytes, "batch")
            self.stats["evictions"] += 1
            log.info("cache: demoted %s from HBM to host (%d bytes)", k, nb)
        while self._host and self._used(self._host) > cfg.host_bytes:
            k, (t, ver, nb, kind) = self._host.popitem(last=False)
            if self._dir:
                path = os.path.join(self._dir, f"{abs(hash(k))}.arrow")
                with ipc.new_file(path, t.schema) as w:
                    w.write_table(t)
                self._disk[k] = (path, ver, nb, kind)
                self.stats["spills"] += 1
            else:
                self.stats["evictions"] += 1
        while self._disk and self._used(self._disk) > cfg.disk_bytes:
            k = next(iter(self._disk))
            self._drop(k)
            self.stats["evictions"] += 1
        if cfg.capacity is not None:
            while len(self) > cfg.capacity:
                k = next(iter(self._hbm or self._host or self._disk))
                self._drop(k)
                self.stats["evictions"] += 1


class Cache(TieredCache):
    """Reference-compatible name: ``Cache::new(CacheConfig)``, ``get``, ``put``."""

    @staticmethod
    def new(config: Optional[CacheConfig] = None) -> "Cache":
        return Cache(config)


class InMemoryCache:
    """String key/value store (reference cache/src/lib.rs:59-87)."""

    def __init__(self):
        self._d: Dict[str, str] = {}
        self._lock = threading.Lock()

    def set(self, key: str, value: str) -> None:
        with self._lock:
            self._d[key] = value

    def get(self, key: str) -> str:
        with self._lock:
            if key not in self._d:
                raise IglooError("Key not found")
            return self._d[key]
