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

from ..catalog import TableSource, _mark_resident
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
        self._last_poll: Dict[str, float] = {}
        self._subs: List[Callable[[ChangeEvent], None]] = []
        self.events: List[ChangeEvent] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ---------------------------------------------------------- registration
    def track(self, table: str, probe: Optional[Callable[[], Any]] = None, version: Any = 0):
        """Start tracking ``table`` (re-registering a name resets it and drops
        its cache entries)."""
        with self._lock:
            known = table in self._versions
            self._versions[table] = probe() if probe is not None else version
            self._probes.pop(table, None)
            if probe is not None:
                self._probes[table] = probe
                self._last_poll[table] = time.monotonic()
        if known:
            self._invalidate(table)

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

    def maybe_poll(self, table: str, min_interval_s: float = 1.0) -> bool:
        """Poll one table's version probe unless it ran within ``min_interval_s``;
        True when the version changed (its cache entries are then invalid)."""
        probe = self._probes.get(table)
        if probe is None:
            return False
        now = time.monotonic()
        with self._lock:
            if now - self._last_poll.get(table, -1e18) < min_interval_s:
                return False
            self._last_poll[table] = now
        try:
            v = probe()
        except Exception as e:  # noqa: BLE001 - a failing probe keeps the cached data
            log.warning("cdc probe for %s failed: %s", table, e)
            return False
        if v != self._versions.get(table):
            self.apply_event(ChangeEvent(table, "snapshot", v))
            return True
        return False

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


def _slice(c, a: int, b: int):
    """Rows [a, b) of a resident column as views (string bytes re-based; the
    byte bounds come through the replayable readback path)."""
    from ..columnar import Column
    from ..ops._lib import to_host_ints
    valid = None if c.valid is None else c.valid[a:b]
    if c.offsets is not None:
        off = c.offsets[a:b + 1]
        lo, hi = to_host_ints(off[[0, -1]]) if b > a else (0, 0)
        return Column(c.dtype, c.data[lo:hi], valid, offsets=off - lo)
    return Column(c.dtype, c.data[a:b], valid, dictionary=c.dictionary)


class CachedTable(TableSource):
    """Serve scans of ``source`` from the cache tier, keyed by the CDC version.

    Every external source the engine registers (Parquet, Iceberg, CSV,
    Postgres, MySQL) is wrapped in one: the first scan of a column reads it
    from the source (GPU Parquet / CSV decode, wire protocols) into HBM and
    later scans hand out the resident column. The column's version comes from
    the table's CDC probe (file set + mtimes, Iceberg snapshot id, Postgres
    ``version_sql``), polled at most every ``poll_interval_s``; a new version
    invalidates the table's entries. HBM / host / disk byte budgets are the
    TieredCache's (config ``cache_hbm_gb`` / ``cache_host_gb`` / ``cache_dir``).
    """

    cacheable = False

    def __init__(self, name: str, source: TableSource, cache: TieredCache, cdc: Optional[CdcManager] = None,
                 poll_interval_s: Optional[float] = None):
        self.name = name
        self.source = source
        self.cache = cache
        self.cdc = cdc
        # bounded staleness: file-system probes (stat of every file) run at most
        # once a second; database probes (``version_sql``) on every scan
        self.poll_interval_s = poll_interval_s if poll_interval_s is not None else \
            getattr(source, "cdc_poll_s", 1.0)
        self.partitioned_by = getattr(source, "partitioned_by", None)
        self.replicated = getattr(source, "replicated", False)
        self.cluster_key = getattr(source, "cluster_key", None)
        self.hits = self.misses = 0
        #: row-group statistics pruning on the cached path (see ``_prune_rows``)
        self.last_prune_stats: dict = {}
        self._ranges_cache: dict = {}
        self._prune_memo: dict = {}
        if cdc is not None:
            probe = (lambda s=source: getattr(s, "version", None)) if hasattr(type(source), "version") else None
            cdc.track(name, probe)

    def __getattr__(self, item):
        # connector-specific attributes (last_gpu_stats, files, ...) of the wrapped source
        if item == "source":
            raise AttributeError(item)
        return getattr(self.source, item)

    @property
    def prunes(self) -> bool:
        """Scans take pushed filters when the source keeps row-group statistics."""
        return bool(getattr(self.source, "prunes", False)) and hasattr(self.source, "prune")

    def schema(self):
        return self.source.schema()

    def num_rows(self):
        return self.source.num_rows()

    def _key(self, c: str, ctx) -> str:
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        dev = str(ctx.device) if ctx is not None else "cpu"
        return f"{self.name}/{rank}of{world}/{dev}/{c}"

    def poll(self) -> bool:
        """Run this table's CDC probe (rate-limited by ``poll_interval_s``);
        True when the source changed (its cache entries are then dropped and
        the cache generation moves). engine.py calls it before replaying a
        query graph, which never reaches ``scan``."""
        if self.cdc is None:
            return False
        return self.cdc.maybe_poll(self.name, self.poll_interval_s)

    def cdc_version(self):
        return self.cdc.version(self.name) if self.cdc is not None else None

    def _prune_rows(self, ctx, filters):
        """Rows of the resident columns that the source's row-group statistics
        cannot rule out: None (all rows), a (start, stop) slice, or a device
        index vector. Resident columns concatenate this rank's row groups in
        ``my_row_groups`` order, so a kept row group is a row range of them."""
        src = self.source
        groups = src.my_row_groups(ctx)
        # the statistics walk is host work over every row group's footer
        # entries: memoised per filter set and source version
        mkey = (repr(filters), getattr(src, "_stat_version", None), len(groups),
                ctx.comm.rank if ctx is not None and ctx.comm is not None else 0)
        keep = self._prune_memo.get(mkey)
        if keep is None:
            keep = src.prune(groups, filters)
            if len(self._prune_memo) > 256:
                self._prune_memo.clear()
            self._prune_memo[mkey] = keep
        self.last_prune_stats = {"row_groups": len(groups), "row_groups_read": len(keep),
                                 "row_groups_pruned": len(groups) - len(keep)}
        if len(keep) == len(groups):
            return None
        kept = set(keep)
        ranges, pos = [], 0
        nrows = src.group_rows() if hasattr(src, "group_rows") else None
        for fi, rg in groups:
            n = nrows[(fi, rg)] if nrows is not None else src._meta[fi].row_group(rg).num_rows
            if (fi, rg) in kept:
                if ranges and ranges[-1][1] == pos:
                    ranges[-1] = (ranges[-1][0], pos + n)
                else:
                    ranges.append((pos, pos + n))
            pos += n
        if not ranges:
            return (0, 0)
        if len(ranges) == 1:
            return ranges[0]
        if 2 * sum(b - a for a, b in ranges) > pos:
            # most rows survive in several runs: gathering every scanned column
            # costs more than letting the filter kernel read them all (and the
            # resident columns keep their derived structures: sortedness,
            # indexes)
            self.last_prune_stats["gathered"] = False
            return None
        key = (tuple(ranges), str(ctx.device) if ctx is not None else "cpu")
        idx = self._ranges_cache.get(key)
        if idx is None:
            import torch
            from ..ops._lib import device_ints
            lens = [b - a for a, b in ranges]
            starts = device_ints([a for a, _ in ranges], ctx.device)
            rep = torch.repeat_interleave(starts, device_ints(lens, ctx.device), output_size=sum(lens))
            first = device_ints([0] + list(__import__("itertools").accumulate(lens))[:-1], ctx.device)
            pos_in = torch.arange(sum(lens), device=ctx.device) - torch.repeat_interleave(
                first, device_ints(lens, ctx.device), output_size=sum(lens))
            idx = rep + pos_in
            if len(self._ranges_cache) > 64:
                self._ranges_cache.clear()
            self._ranges_cache[key] = idx
        return idx

    def scan(self, columns: Sequence[str], ctx, filters=None) -> Batch:
        b = self._scan_all(columns, ctx)
        if not filters or not self.prunes:
            self.last_prune_stats = {}
            return b
        rows = self._prune_rows(ctx, filters)
        if rows is None:
            return b
        if isinstance(rows, tuple):
            a, z = rows
            return Batch({c: _slice(col, a, z) for c, col in b.columns.items()}, z - a)
        from ..ops.gather import take_many
        keys = list(b.columns)
        return Batch(dict(zip(keys, take_many([b.columns[k] for k in keys], rows))), int(rows.numel()))

    def scan_morsels(self, columns: Sequence[str], ctx, filters=None, max_rows: int = 1 << 20):
        """Morsels straight from the source (exec/morsel.py): a streamed scan
        exists to keep the table out of device memory, so it bypasses the
        cache tier."""
        if self.cdc is not None:
            self.cdc.maybe_poll(self.name, self.poll_interval_s)
        yield from self.source.scan_morsels(columns, ctx, filters, max_rows)

    @property
    def can_stream(self) -> bool:
        return bool(getattr(self.source, "can_stream", False))

    def _scan_all(self, columns: Sequence[str], ctx) -> Batch:
        ver = None
        if self.cdc is not None:
            self.cdc.maybe_poll(self.name, self.poll_interval_s)
            ver = self.cdc.version(self.name)
        out, n, missing = {}, None, []
        keys = getattr(ctx, "cache_keys", None)
        for c in columns:
            if keys is not None:
                keys.append(self._key(c, ctx))
            hit = self.cache.get(self._key(c, ctx), ver)
            if hit is None:
                missing.append(c)
            else:
                out[c] = hit.columns[c]
                n = hit.num_rows
        if missing:
            self.misses += len(missing)
            from ..ops._lib import unlogged
            with unlogged():     # a cache fill, not part of the query's repeatable readbacks
                b = self.source.scan(missing, ctx)
            for c in missing:
                col = b.columns[c]
                _mark_resident(col)
                self.cache.put(self._key(c, ctx), Batch({c: col}, b.num_rows), ver)
                out[c] = col
            n = b.num_rows
        self.hits += len(columns) - len(missing)
        if n is None:
            n = self.source.num_rows() or 0
        return Batch({c: out[c] for c in columns}, n)

    def evict(self) -> int:
        return self.cache.invalidate(f"{self.name}/")
