"""Query graphs: a repeated query over unchanged data runs as one HIP graph.

Once a query's host readbacks replay completely from a trusted recording
(engine.py ``_execute_speculative``, ops/_lib.py ``Speculation``), its host
control flow no longer depends on the device: every kernel, memset and copy it
enqueues is fixed by the plan and the data. The next execution then runs the
operators once more under stream capture instead of eagerly. The HIP graph it
records is the whole query (scans, joins, aggregation, sort, and the device-side
check of every replayed value), and every later execution is one
``hipGraphLaunch`` plus one stream sync. That removes the Python operator
dispatch (2-6 ms per query at SF100, ``profiles/r2_roctx_per_query_idle_sf100.txt``)
and the per-launch overhead from the critical path.

Every replay still runs every kernel over the resident columns. Nothing is cached
but the launch sequence. What keeps a graph valid:

* the key. Graphs live in the speculation state, which is keyed on the SQL text,
  the catalog version and the cache generation (a table change, eviction or
  refill drops them), and each graph also records the generated-kernel set it
  was captured with (ops/jit.py ``generation``). A kernel that finishes
  compiling makes the next execution re-capture.
* the device check. The replayed sizes and ranges are compared with the device
  values inside the graph (one int64 mismatch count read after each replay). On
  a mismatch the graph is dropped and the query re-executes eagerly with real
  readbacks.
* the first replay. Right after capture, the graph's result digest
  (utils/digest.py) must equal the previous eager execution's. Otherwise the
  query is marked never to be captured again.
* capture refusal. Anything a graph cannot replay raises
  ``CaptureAbort`` before any HIP call (ops/_lib.py): a real readback, a
  one-time derived-structure build, a generated-kernel load, a host spill. The
  query then stays eager.

Memory: each graph owns a private pool (its whole working set stays reserved
between replays). The capture measures the pool's bytes and the engine charges
them, together with the cache tier's resident columns, against its HBM budget
(engine.py ``enforce_graph_budget``): past it, the least recently replayed
graphs are dropped and their pools freed. ``SHARED_POOL = True`` shares
one pool between all graphs of an engine instead.

CDC: a replay never reaches ``CachedTable.scan``, so the engine polls the CDC
probes of the query's tables before every replay (same rate limit); a changed
source moves the cache generation and so the key, and the stale graph is
dropped.

The reference has no GPU execution and so nothing comparable; its engine
rebuilds DataFusion physical plans per query (reference
crates/engine/src/lib.rs:112-140). This is the HIP-graph half of SURVEY §5.7's
"HIP streams and graphs instead of a tracing compiler".
"""
from __future__ import annotations

from ..utils import switches as _sw
import gc
import logging
import os
import traceback
from typing import Optional

import torch

from ..ops import _lib
from ..ops import jit as _jit

log = logging.getLogger("igloo.graphs")

GRAPHS = os.environ.get("IGLOO_GRAPHS", "1") == "1"
#: one memory pool for all graphs of an engine (0: a private pool per graph)
SHARED_POOL = False

_streams: dict = {}
STATS = {"captured": 0, "replays": 0, "aborted": 0, "failed": 0, "mismatch": 0}
LAST_ERROR: list = []    # why the last captures did not produce a graph (debugging, tests)


def _note(msg: str) -> None:
    LAST_ERROR.append(msg)
    del LAST_ERROR[:-24]


def _capture_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _streams.get(dev.index)
    if s is None:
        s = _streams[dev.index] = torch.cuda.Stream(dev)
    return s


class QueryGraph:
    """One captured query: the graph, its static result batch and the device
    mismatch counter of its replayed values."""

    __slots__ = ("graph", "batch", "bad", "expected", "jit_gen", "rows_scanned", "spill", "checked", "replays", "sp",
                 "nbytes", "comm_calls", "comm_bytes", "comm_chunks", "keep", "global_check")

    def __init__(self, graph, batch, bad, expected, jit_gen, rows_scanned, spill, sp=None, nbytes=0):
        self.sp = sp                   # the capture's speculation (sites + device values, for reports)
        self.nbytes = nbytes           # device bytes of the graph's private memory pool
        self.comm_calls = 0            # collectives inside the graph (SPMD)
        self.comm_chunks = 0           # ... of which pipelined-exchange chunks past each exchange's first
        self.comm_bytes = 0
        self.keep = []
        self.global_check = False      # ``bad`` is summed over SPMD ranks inside the graph
        self.graph = graph
        self.batch = batch
        self.bad = bad
        self.expected = expected       # kept alive: read by the graph's compare kernel
        self.jit_gen = jit_gen
        self.rows_scanned = rows_scanned
        self.spill = spill
        self.checked = False           # first replay compared with the eager result
        self.replays = 0

    def current(self) -> bool:
        """Still built from the generated kernels that are loaded now."""
        return self.jit_gen == _jit.generation()

    def launch(self, ctx) -> None:
        """Launch the graph without waiting for it: the caller checks ``bad``
        with the result's host copy (engine.py _host_columns), one sync."""
        self.graph.replay()
        self.replays += 1
        STATS["replays"] += 1
        ctx.rows_scanned = self.rows_scanned
        ctx.spill = dict(self.spill)

    def replay(self, ctx) -> bool:
        """Launch the graph on the current stream; True when every replayed
        value matched the device (one sync)."""
        self.graph.replay()
        self.replays += 1
        STATS["replays"] += 1
        ctx.rows_scanned = self.rows_scanned
        ctx.spill = dict(self.spill)
        ok = int(self.bad.reshape(-1)[0].item()) == 0
        if not ok:
            STATS["mismatch"] += 1
            try:
                act = self.sp.actual[0].tolist() if self.sp is not None and self.sp.actual else []
                _note(f"mismatch: {self.sp.mismatch_sites(act)[:4]}")
            except Exception:   # noqa: BLE001 - diagnostics only
                pass
        return ok


def capture(engine, plan, log_: list, make_ctx) -> Optional[QueryGraph]:
    """Capture ``plan`` executed under a replay of the recording ``log_``.
    Returns None (query stays eager) when the capture is refused or fails."""
    dev = engine.device
    gen = _jit.generation()
    if gen is None:
        return None
    sp = _lib.Speculation("replay", log_)
    exp = sp.expected_values()
    expected = torch.tensor(exp or [0], dtype=torch.int64).to(dev)[:len(exp)]
    ctx = make_ctx()
    cur = torch.cuda.current_stream(dev)
    s = _capture_stream(dev)
    s.wait_stream(cur)
    g = torch.cuda.CUDAGraph()
    batch = bad = None
    # the graph's private pool is what capture adds to the reserved bytes
    # (engine.py charges it against the HBM budget)
    reserved0 = torch.cuda.memory_reserved(dev)
    _lib.set_speculation(sp)
    _lib.set_capturing(True)
    # torch raises before any synchronizing call (blocking copy, .item(),
    # nonzero) reaches HIP: such a site ends the capture cleanly instead of
    # invalidating it inside the runtime
    sync_mode = torch.cuda.get_sync_debug_mode()
    torch.cuda.set_sync_debug_mode(2)
    dump = _sw.debug_value("graph_dump")     # debugging: DOT dump of every captured graph
    if dump:
        g.enable_debug_mode()
    # no cyclic garbage collection inside the capture: a collected object's
    # tensors would be freed (and any synchronizing call in their teardown
    # raised, under the sync-debug mode above, inside a destructor: abort)
    # while the stream records
    gc_on = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.stream(s):
            g.capture_begin(pool=engine.graph_pool() if SHARED_POOL else None, capture_error_mode="thread_local")
            try:
                batch = engine._execute_plan(plan, ctx, fold_checks=True)
                if not sp.complete:
                    raise _lib.CaptureAbort("call sequence left the recording")
                bad = sp.device_mismatches(expected)
                comm = engine.comm
                if comm is not None and comm.spmd:
                    # SPMD: the mismatch count is summed over ranks inside the
                    # graph, so the one readback after a replay is already the
                    # agreement of every rank (no extra host round trip)
                    bad = comm.allreduce_tensor(bad.reshape(1).to(torch.int64), "sum")
            finally:
                g.capture_end()
    except _lib.CaptureAbort as e:
        engine._graph_pool = None
        STATS["aborted"] += 1
        _note(f"aborted: {e} :: " + " <- ".join(
            f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}" for f in traceback.extract_tb(e.__traceback__)[-4:][::-1]))
        log.debug("query graph not captured: %s", e)
        return None
    except RuntimeError as e:
        engine._graph_pool = None
        if "synchronizing" in str(e):      # raised by torch before the call: a clean abort
            STATS["aborted"] += 1
            _note("aborted (sync): " + traceback.format_exc(limit=-4))
            return None
        # a HIP call the capture refused: the runtime invalidated the capture.
        # End it for good (an invalidated capture can leave the stream in
        # capture mode, and every later launch of this thread would fail);
        # this engine stops capturing (a failed capture's allocator state is
        # not something to build on); the query stays eager.
        try:
            _lib.native().end_capture(s.cuda_stream)
        except Exception:  # noqa: BLE001 - best effort
            pass
        engine.graphs_disabled = True
        STATS["failed"] += 1
        _note("failed: " + traceback.format_exc(limit=-5))
        log.warning("query graph capture failed, graphs disabled for this engine: %s", e)
        torch.cuda.synchronize(dev)
        return None
    finally:
        if gc_on:
            gc.enable()
        torch.cuda.set_sync_debug_mode(sync_mode)
        if batch is None or bad is None:
            _lib.capture_keepalive()       # a failed capture keeps nothing
        _lib.set_capturing(False)
        _lib.set_speculation(None)
        cur.wait_stream(s)
    if dump:
        os.makedirs(dump, exist_ok=True)
        g.debug_dump(os.path.join(dump, f"graph_{STATS['captured']}.dot"))
    STATS["captured"] += 1
    nbytes = max(0, torch.cuda.memory_reserved(dev) - reserved0)
    qg = QueryGraph(g, batch, bad, expected, gen, ctx.rows_scanned, ctx.spill, sp, nbytes)
    qg.global_check = engine.comm is not None and engine.comm.spmd
    qg.keep = _lib.capture_keepalive()     # pinned host buffers its copy nodes read
    return qg
