"""QueryEngine: the user-facing SQL entry point.

Parity: reference crates/engine/src/lib.rs:27-62 — ``QueryEngine::new`` (registers
the ``capitalize`` UDF), ``register_table``, ``execute(sql) -> Vec<RecordBatch>``
(panics on error, :55-56), ``session_context``. Here ``execute`` runs the native
parser -> binder -> optimizer -> GPU operators and returns ``pyarrow.RecordBatch``es;
errors raise typed ``IglooError``s instead of panicking.
"""
from __future__ import annotations

import collections
import os
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import pyarrow as pa
import torch

from . import types as T
from .catalog import Catalog, Field, MemoryTable, TableSource
from .columnar import Batch, Column
from .exec.context import ExecContext
from .exec.planner import create_physical_plan
from .sql import parse
from .utils import switches as _sw
from .sql import template as TPL
from .sql.binder import Binder, IdGen
from .sql.logical import ColInfo, Plan, Project
from .sql.optimizer import optimize
from .utils.errors import ExecutionError, IglooError, NotSupported, PlanError, TableNotFound
from .exec import graphs as _graphs
from .ops import jit as _jit
from .utils import trace as _trace
from .utils.digest import digest
from .utils.log import get_logger

#: cache optimized logical plans per SQL text (parse + bind + optimize cost
#: ~1 ms of Python per TPC-H query); keyed on the catalog version and the
#: session settings, so any DDL or SET invalidates
PLAN_CACHE = True
PLAN_CACHE_SIZE = 256
#: statement templates (sql/template.py): fresh literal values reuse a
#: verified bound + optimized plan of the same statement shape
TEMPLATES = not _sw.debug("no_templates")
TEMPLATE_CACHE_SIZE = 256
#: replay the host readbacks of repeated queries over unchanged data (see
#: QueryEngine._execute_speculative)
SPECULATE = True
SPMD_SPECULATE = True
#: SPMD query graphs (collectives captured with the kernels; RCCL only)
SPMD_GRAPHS = True
#: SPMD: a query over replicated tables only splits its largest table by key range
SLICE_REPLICATED = True

log = get_logger("engine")


def default_device() -> str:
    try:
        if torch.cuda.is_available():
            return "cuda"
    except Exception:  # pragma: no cover
        pass
    return "cpu"


class QueryResult:
    """Materialised query output (host Arrow) + execution metrics."""

    def __init__(self, table: pa.Table, elapsed_ms: float, plan_text: str = ""):
        self.table = table
        self.elapsed_ms = elapsed_ms
        self.plan_text = plan_text

    @property
    def num_rows(self) -> int:
        return self.table.num_rows

    def to_arrow(self) -> pa.Table:
        return self.table

    def to_pandas(self):
        return self.table.to_pandas()

    def to_pylist(self):
        return self.table.to_pylist()

    def batches(self) -> List[pa.RecordBatch]:
        return self.table.to_batches() or [pa.RecordBatch.from_pylist([], schema=self.table.schema)]

    def __repr__(self):
        return pretty_format(self.table)


def _allocated(device, which: str) -> int:
    """Allocated device bytes ("current" / "peak") from the allocator's nested
    stats: ``torch.cuda.memory_allocated`` and ``max_memory_allocated``
    flatten the whole stats tree on every call (~0.1 ms each, twice per
    query on the timed path)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return int(torch._C._cuda_memoryStats(idx)["allocated_bytes"]["all"][which])


def _raise_deferred(deferred, flags) -> None:
    for v, msg in zip(flags, deferred[1]):
        if v:
            raise ExecutionError(msg)


class _ReplayMismatch(Exception):
    """A graph replay's values did not match the device (seen with its result copy)."""


_PAD = {}


def _pad(dev, n: int) -> torch.Tensor:
    """n (< 16) zero bytes on ``dev`` (made outside any graph capture)."""
    z = _PAD.get(dev)
    if z is None:
        z = _PAD[dev] = torch.zeros(16, dtype=torch.uint8, device=dev)
    return z[:n]


def _device_pack(ts: List[torch.Tensor], dev):
    """The device tensors ``ts`` as ONE byte buffer (one concatenation
    kernel; each piece padded to 16 bytes) and their (offset, bytes, dtype,
    shape) spans in it."""
    pieces, spans, off = [], [], 0
    for t in ts:
        b = t.reshape(-1)
        if b.numel() <= 1:
            b = b.as_strided((b.numel(),), (1,))     # (a one-element slice may carry any stride)
        elif not b.is_contiguous():
            b = b.contiguous()
        b = b.view(torch.uint8)
        n = b.numel()
        pieces.append(b)
        spans.append((off, n, t.dtype, tuple(t.shape)))
        pad = (-n) % 16
        if pad:
            pieces.append(_pad(dev, pad))
        off += n + pad
    return (torch.cat(pieces) if len(pieces) > 1 else pieces[0]), spans


def _pinned_copy(buf: torch.Tensor, spans) -> List[torch.Tensor]:
    """One non-blocking copy of ``buf`` into pinned memory, split into the
    tensors of ``spans`` (the caller synchronises before reading them)."""
    host = torch.empty(buf.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(buf, non_blocking=True)
    return [host[o:o + n].view(dt).reshape(shape) for o, n, dt, shape in spans]


def _result_layout(cols: List[Column], deferred=None, guard=None):
    """How a result goes to the host: (per-column plan, device tensors to
    copy in order, index of the deferred flags, index of the guard)."""
    pending: List[torch.Tensor] = []

    def cpu(t):
        if t is None:
            return None
        pending.append(t)
        return len(pending) - 1

    def move(c: Column):
        if not c.data.is_cuda or c.dtype.is_nested:
            return c          # (nested: rows are views into device children; to_arrow copies them)
        d = c.dictionary
        if d is not None and len(d) > 2 * len(c) + 1024:
            return c
        return (c.dtype, cpu(c.data), cpu(c.valid), cpu(c.offsets), move(d) if d is not None else None)
    plan = [move(c) for c in cols]
    fi = cpu(deferred[0]) if deferred is not None else None
    gi = cpu(guard.reshape(-1)[:1]) if guard is not None else None
    return plan, pending, fi, gi


def _host_columns(cols: List[Column], deferred=None, guard=None) -> List[Column]:
    """Result columns moved to the host with ONE synchronisation: every device
    buffer (values, validity, offsets, small dictionaries) travels in one
    device-side concatenation and one D2H copy (a copy per buffer costs ~18 us
    of host submission each, with the GPU idle), then the stream is
    synchronised once. (Packing inside the query graph instead measured
    slower: profiles/r6_ab_graph_result_pack_rejected.txt.) A string column
    that references a large device dictionary keeps its device path (it
    decodes only the referenced strings on the GPU)."""
    if not any(c.data.is_cuda for c in cols):
        if guard is not None and int(guard.reshape(-1)[0].item()):
            raise _ReplayMismatch()
        if deferred is not None:
            _raise_deferred(deferred, deferred[0].tolist())
        return cols
    plan, pending, fi, gi = _result_layout(cols, deferred, guard)
    dev = next(c.data.device for c in cols if c.data.is_cuda)
    host = _pinned_copy(*_device_pack(pending, dev)) if pending else []
    torch.cuda.current_stream(dev).synchronize()

    def build(x):
        if isinstance(x, Column):
            return x
        dt, di, vi, oi, d = x
        return Column(dt, host[di], None if vi is None else host[vi], offsets=None if oi is None else host[oi],
                      dictionary=build(d) if d is not None else None)
    out = [build(x) for x in plan]
    flags = host[fi] if fi is not None else None
    bad = host[gi] if gi is not None else None
    if bad is not None and int(bad[0]):
        raise _ReplayMismatch()      # the copied rows are not the query's: the caller re-executes
    if deferred is not None:
        # the query's deferred device error flags ride on the result copy
        _raise_deferred(deferred, flags.tolist())
    return out


def _confirm(prev, cur):
    """Replayable log from two recordings of the same query, or None when their
    call sequences differ. Sites whose values differ become volatile (None)."""
    if prev is None or len(prev) != len(cur) or any(a[0] != b[0] for a, b in zip(prev, cur)):
        return None
    return [(a[0], a[1] if a[1] == b[1] else None) for a, b in zip(prev, cur)]


class QueryEngine:
    def __init__(self, device: Optional[str] = None, catalog: Optional[Catalog] = None, comm=None,
                 config: Optional[dict] = None, cache_hbm_gb: Optional[float] = None,
                 cache_host_gb: Optional[float] = None, cache_dir: Optional[str] = None):
        from .cache.cdc import CdcManager
        from .cache.tiered import CacheConfig, TieredCache
        from .utils.memory import device_capacity
        self.device = torch.device(device or default_device())
        self.catalog = catalog or Catalog()
        self.comm = comm
        self.session: Dict[str, Any] = dict(config or {})
        # optimized logical plans by (SQL text, catalog version, session settings)
        self._plans: "collections.OrderedDict" = collections.OrderedDict()
        # verified statement templates by (template text, catalog version, session settings)
        self._templates: "collections.OrderedDict" = collections.OrderedDict()
        self.template_stats = {"recorded": 0, "verified": 0, "rejected": 0, "instantiated": 0, "stale": 0}
        self._prepared: Dict[str, tuple] = {}    # PREPARE name -> (statement AST, parameter types)
        self._graph_pool = None
        self.graphs_disabled = False    # set after a capture the runtime refused (exec/graphs.py)
        self._spec: Dict[Any, dict] = {}   # replayable host readbacks per (plan, catalog, cache generation)
        self._ids = IdGen()
        self._lock = threading.RLock()
        self.last_metrics: Dict[str, Any] = {}
        if self.device.type == "cuda":
            from .ops._lib import native
            native()  # fail loudly on a GPU box without the native extension
        # cache tier for external sources (reference crates/cache/src/lib.rs:12-56,
        # README "automatic cache invalidation via CDC"): resident decoded
        # columns in HBM, demoted to host memory / Arrow IPC files past the
        # budgets; the default HBM budget leaves a quarter of the device for
        # query working memory (288 GB MI355X -> 216 GB of cached columns)
        cap = device_capacity(self.device)
        hbm = cache_hbm_gb * 2**30 if cache_hbm_gb is not None else (0.75 * cap if cap else 32 * 2**30)
        host = cache_host_gb * 2**30 if cache_host_gb is not None else 32 * 2**30
        self.cache = TieredCache(CacheConfig(hbm_bytes=int(hbm), host_bytes=int(host), disk_path=cache_dir,
                                             device=str(self.device)))
        self.cdc = CdcManager(self.cache)
        self.hbm_peak_bytes = 0     # highest per-query HBM high-water mark (last_metrics["hbm_peak_bytes"])
        # device bytes the cache tier's resident columns and the query graphs'
        # private memory pools may hold together (exec/graphs.py); past it the
        # least recently replayed graphs are dropped (their pools return to
        # the allocator). The rest of HBM is query working memory.
        gb = (config or {}).get("hbm_budget_gb", os.environ.get("IGLOO_HBM_BUDGET_GB"))
        self.hbm_budget = int(float(gb) * 2**30) if gb not in (None, "") else (int(0.9 * cap) if cap else None)
        self._graphs: "collections.OrderedDict[int, dict]" = collections.OrderedDict()   # LRU of states with graphs
        self.graph_bytes = 0
        self.graph_stats = {"evicted": 0, "dropped_stale": 0}
        self._spec_current: Dict[Any, Any] = {}     # plan key -> its live speculation key
        self._query_sources: Dict[Any, list] = {}   # plan key -> cached table sources it reads
        #: SPMD: global NDV and global rows of base-table join keys
        #: ((catalog version, cache generation), table, column) -> (ndv, rows)
        self._gndv: Dict[Any, tuple] = {}

    # -------------------------------------------------------------- catalog
    def register_table(self, name: str, table: Union[TableSource, pa.Table, Batch, Dict[str, Column]],
                       cache: Optional[bool] = None, **kw):
        """Register a table. External sources (``cacheable`` connectors) are
        served through the cache tier unless ``cache=False``."""
        if isinstance(table, TableSource) and (cache if cache is not None else getattr(table, "cacheable", False)):
            from .cache.cdc import CachedTable
            table = CachedTable(name, table, self.cache, self.cdc)
        if isinstance(table, pa.Table):
            table = MemoryTable.from_arrow(table, device=self.device, **kw)
        elif isinstance(table, pa.RecordBatch):
            table = MemoryTable.from_arrow(pa.Table.from_batches([table]), device=self.device, **kw)
        elif isinstance(table, Batch):
            table = MemoryTable(table.columns, table.num_rows, **kw)
        elif isinstance(table, dict):
            table = MemoryTable(table, **kw)
        self.catalog.register_table(name, table)
        return table

    def deregister_table(self, name: str):
        self.cache.invalidate(f"{name}/")
        return self.catalog.deregister_table(name)

    def register_parquet(self, name: str, path: str, cache: Optional[bool] = None, **kw):
        from .connectors.parquet import ParquetTable
        return self.register_table(name, ParquetTable(path, **kw), cache=cache)

    def register_csv(self, name: str, path: str, schema=None, has_header: bool = True, delimiter: str = ",",
                     cache: Optional[bool] = None, **kw):
        from .connectors.csv import CsvTable
        return self.register_table(name, CsvTable(path, schema=schema, has_header=has_header, delimiter=delimiter,
                                                  **kw), cache=cache)

    def register_json(self, name: str, path: str, schema=None, cache: Optional[bool] = None):
        from .connectors.json import JsonTable
        return self.register_table(name, JsonTable(path, schema=schema), cache=cache)

    def register_iceberg(self, name: str, path: str, cache: Optional[bool] = None, **kw):
        from .connectors.iceberg import IcebergTable
        return self.register_table(name, IcebergTable(path, **kw), cache=cache)

    def session_context(self) -> "QueryEngine":
        return self

    # -------------------------------------------------------------- planning
    def logical_plan(self, sql: str, optimized: bool = True):
        stmts = parse(sql)
        if len(stmts) != 1:
            raise PlanError("expected exactly one statement")
        st = stmts[0]
        if st["k"] == "explain":
            st = st["c"][0]
        if st["k"] != "query":
            raise PlanError("not a query")
        b = Binder(self.catalog, self._ids, self.session)
        bq = b.bind_query(st)
        plan = optimize(bq.plan) if optimized else bq.plan
        return plan, bq.names

    def explain(self, sql: str, analyze: bool = False) -> str:
        r = self.sql(("EXPLAIN ANALYZE " if analyze else "EXPLAIN ") + sql)
        return "\n".join(r.table.column("plan").to_pylist())

    # -------------------------------------------------------------- execution
    def execute(self, sql: str) -> List[pa.RecordBatch]:
        """Run SQL; returns Arrow record batches (reference API shape)."""
        return self.sql(sql).batches()

    def query(self, sql: str) -> pa.Table:
        return self.sql(sql).table

    def sql_device(self, sql: str):
        """Run a query and leave its result in device memory: a
        ``interop.DeviceResult`` exported zero-copy through the Arrow C Device
        Data Interface (``__arrow_c_device_array__``) and DLPack, instead of
        the host Arrow table ``sql`` returns."""
        from .interop import DeviceResult
        plan, names = self.logical_plan(sql)
        with self._lock:
            batch = self._execute_plan(plan, self.make_context())
        cols = {}
        for ci, nm in zip(plan.schema, names):
            cols[nm] = batch.columns[ci.cid]
        return DeviceResult(cols, batch.num_rows, {nm: ci.nullable for ci, nm in zip(plan.schema, names)})

    def sql(self, sql: str) -> QueryResult:
        key = None
        if PLAN_CACHE:
            key = (sql, self.catalog.version, tuple(sorted((k, repr(v)) for k, v in self.session.items())))
            hit = self._plans.get(key)
            if hit is not None:
                self._plans.move_to_end(key)
                return self._exec_query(hit[0], hit[1], time.perf_counter(), cached=True, key=key)
        lx = tkey = None
        if key is not None and TEMPLATES:
            t0 = time.perf_counter()
            lx = TPL.lex(sql)
            if lx is not None:
                tkey = (lx.key,) + key[1:]
                ent = self._templates.get(tkey)
                if ent is not None and ent.verified and ent.matches(lx.texts):
                    got = ent.instantiate(lx.texts, Binder.literal_of)
                    if got is not None:
                        self._templates.move_to_end(tkey)
                        self.template_stats["instantiated"] += 1
                        self._cache_plan(key, got)
                        return self._exec_query(got[0], got[1], t0, key=key, planned="template")
                    self.template_stats["stale"] += 1
        stmts = parse(sql)
        if key is not None and len(stmts) == 1 and stmts[0]["k"] == "query":
            t0 = time.perf_counter()
            got = self._record_template(sql, stmts[0], lx, tkey) if tkey is not None else None
            plan, names = got if got is not None else self._plan_query(stmts[0])
            self._cache_plan(key, (plan, names))
            return self._exec_query(plan, names, t0, key=key)
        if not stmts:
            raise PlanError("empty SQL statement")
        res = None
        for st in stmts:
            res = self._run_statement(st)
        return res

    def _run_statement(self, st: dict) -> QueryResult:
        k = st["k"]
        t0 = time.perf_counter()
        if k == "query":
            return self._run_query(st, t0)
        if k == "explain":
            return self._explain(st["c"][0], bool(st.get("analyze")))
        if k == "set":
            from .sql.binder import Binder as _B
            v = Binder(self.catalog, self._ids).bind_expr(st["c"][0], __import__("igloo_amd.sql.binder", fromlist=["Scope"]).Scope([]))
            self.session[st["s"]] = getattr(v, "value", None)
            return QueryResult(pa.table({}), 0.0)
        if k == "show":
            if st["s"] == "columns":
                return self._describe(st["table"], full=True)
            if st["s"] == "all":
                keys = sorted(self.session)
                return QueryResult(pa.table({"name": pa.array(keys, pa.string()),
                                             "value": pa.array([str(self.session[k]) for k in keys], pa.string())}),
                                   0.0)
            if st["s"] != "tables":
                if st["s"] in self.session:
                    return QueryResult(pa.table({"name": [st["s"]], "value": [str(self.session[st["s"]])]}), 0.0)
                raise NotSupported(f"SHOW {st['s']}")
            names = self.catalog.table_names()
            return QueryResult(pa.table({"table_name": pa.array(names, pa.string())}), 0.0)
        if k == "drop_table":
            if self.catalog.deregister_table(st["s"]) is None and not st.get("if_exists"):
                raise PlanError(f"table '{st['s']}' does not exist")
            return QueryResult(pa.table({}), 0.0)
        if k == "create_view":
            name = st["s"]
            if self.catalog.get_view(name) is not None or self.catalog.get_table(name) is not None:
                if st.get("if_not_exists"):
                    return QueryResult(pa.table({}), 0.0)
                if not st.get("replace") or self.catalog.get_table(name) is not None:
                    raise PlanError(f"'{name}' already exists")
            view = dict(st["query"])
            cols = [c["s"] for c in (st.get("columns") or {}).get("c", [])]
            # bind once now: an invalid view fails at CREATE, like DataFusion
            bq = Binder(self.catalog, self._ids, self.session).bind_query(view)
            if cols:
                if len(cols) != len(bq.names):
                    raise PlanError(f"view '{name}' lists {len(cols)} columns for {len(bq.names)}")
                view["__columns"] = cols
            self.catalog.register_view(name, view)
            return QueryResult(pa.table({}), 0.0)
        if k == "drop_view":
            if self.catalog.get_view(st["s"]) is None:
                if not st.get("if_exists"):
                    raise PlanError(f"view '{st['s']}' does not exist")
                return QueryResult(pa.table({}), 0.0)
            self.catalog.drop_view(st["s"])
            return QueryResult(pa.table({}), 0.0)
        if k == "describe":
            return self._describe(st["s"])
        if k == "insert":
            return self._insert(st)
        if k == "truncate":
            src = self.catalog.get_table(st["s"])
            if not isinstance(src, MemoryTable):
                raise NotSupported("TRUNCATE of a table that is not in memory")
            empty = {f.name: src.columns[f.name] for f in src.schema()}
            from .ops.gather import take_many
            idx = torch.zeros(0, dtype=torch.int64, device=next(iter(empty.values())).device) if empty else None
            cols = dict(zip(empty, take_many(list(empty.values()), idx))) if empty else {}
            self.register_table(st["s"], MemoryTable(cols, 0, fields=list(src.schema())))
            return QueryResult(pa.table({"count": pa.array([src.num_rows()], pa.int64())}), 0.0)
        if k == "create_external_table":
            return self._create_external(st)
        if k == "prepare":
            types = [T.parse_type_name(t["s"]) for t in (st.get("types") or {}).get("c", [])]
            self._prepared[st["s"]] = (st["c"][0], types)
            return QueryResult(pa.table({}), 0.0)
        if k == "execute":
            return self._execute_prepared(st)
        if k == "deallocate":
            if self._prepared.pop(st["s"], None) is None:
                raise PlanError(f"prepared statement '{st['s']}' does not exist")
            return QueryResult(pa.table({}), 0.0)
        if k == "copy":
            return self._copy(st)
        if k == "create_table":
            if st.get("query"):
                b = Binder(self.catalog, self._ids, self.session)
                bq = b.bind_query(st["query"])
                batch = self._execute_plan(optimize(bq.plan))
                cols = {n: batch.columns[c.cid] for n, c in zip(bq.names, bq.plan.schema)}
                self.register_table(st["s"], MemoryTable(cols, batch.num_rows))
                return QueryResult(pa.table({"count": [batch.num_rows]}), 0.0)
            raise NotSupported("CREATE TABLE without AS SELECT")
        raise NotSupported(f"statement {k}")

    def _execute_prepared(self, st) -> QueryResult:
        """EXECUTE name(args): the prepared statement bound with ``$n`` =
        the n-th argument (constant expressions, cast to PREPARE's types)."""
        from .sql import binder as _bd
        name = st["s"]
        if name not in self._prepared:
            raise PlanError(f"prepared statement '{name}' does not exist")
        stmt, types = self._prepared[name]
        b = Binder(self.catalog, self._ids, self.session)
        vals = []
        for i, a in enumerate((st.get("args") or {}).get("c", [])):
            v = _bd._fold(b.bind_expr(a, _bd.Scope([])))
            if not isinstance(v, _bd.Lit):
                raise PlanError(f"EXECUTE {name}: argument {i + 1} is not a constant")
            if i < len(types) and v.dtype != types[i]:
                v = b._coerce_lit(v, types[i]) if v.value is not None else _bd.Lit(None, types[i])
            vals.append(v)
        if types and len(vals) != len(types):
            raise PlanError(f"EXECUTE {name}: expected {len(types)} arguments, got {len(vals)}")
        tok = _bd.PARAMS.set(vals)
        try:
            return self._run_statement(stmt)
        finally:
            _bd.PARAMS.reset(tok)

    def _copy(self, st) -> QueryResult:
        """COPY (query) | table TO 'path' [STORED AS PARQUET|CSV|JSON|ARROW]
        [OPTIONS (...)]: runs the query on the device and writes the result
        (format from STORED AS, else the path's extension; a path ending in
        '/' is a directory that gets one file). Returns the row count, like
        DataFusion's COPY (reference Cargo.lock:1329 datafusion-sql)."""
        import os as _os
        if st.get("query"):
            tab = self._run_statement(st["query"]).table
        else:
            src = self.catalog.get_table(st["s"])
            if src is None and self.catalog.get_view(st["s"]) is None:
                raise TableNotFound(f"table '{st['s']}' not found")
            tab = self.sql(f'SELECT * FROM "{st["s"]}"').table
        path = st["path"]
        fmt = (st.get("stored_as") or st.get("opt.format") or "").upper()
        if not fmt:
            ext = _os.path.splitext(path.rstrip("/"))[1].lower().lstrip(".")
            fmt = {"parquet": "PARQUET", "csv": "CSV", "json": "JSON", "ndjson": "JSON", "arrow": "ARROW"}.get(ext, "")
        if not fmt:
            raise PlanError(f"COPY: cannot infer the format of '{path}' (use STORED AS)")
        if path.endswith("/"):
            _os.makedirs(path, exist_ok=True)
            path = _os.path.join(path, "part-0." + fmt.lower())
        else:
            d = _os.path.dirname(path)
            if d:
                _os.makedirs(d, exist_ok=True)
        from .connectors import writers
        writers.write_table(tab, path, fmt, {k[4:]: v for k, v in st.items() if k.startswith("opt.")})
        return QueryResult(pa.table({"count": pa.array([tab.num_rows], pa.uint64())}), 0.0)

    def _describe(self, name: str, full: bool = False) -> QueryResult:
        """DESCRIBE t / SHOW COLUMNS FROM t (DataFusion's column layout)."""
        src = self.catalog.get_table(name)
        if src is not None:
            fields = [(f.name, f.dtype, f.nullable) for f in src.schema()]
        else:
            view = self.catalog.get_view(name)
            if view is None:
                raise TableNotFound(f"table '{name}' not found")
            plan, names = self._plan_query({"k": "query", "s": "", "c": [], "pos": 0,
                                            "body": {"k": "select", "s": "", "c": [], "pos": 0,
                                                     "items": {"k": "list", "s": "", "c": [{"k": "star", "s": "",
                                                                                            "c": [], "pos": 0}],
                                                               "pos": 0},
                                                     "from": {"k": "list", "s": "", "pos": 0,
                                                              "c": [{"k": "table", "s": name, "c": [], "pos": 0}]}}})
            fields = [(n, c.dtype, c.nullable) for n, c in zip(names, plan.schema)]
        cols = {"column_name": pa.array([f[0] for f in fields], pa.string()),
                "data_type": pa.array([str(f[1]) for f in fields], pa.string()),
                "is_nullable": pa.array(["YES" if f[2] else "NO" for f in fields], pa.string())}
        if full:
            cols = {"table_catalog": pa.array(["datafusion"] * len(fields), pa.string()),
                    "table_schema": pa.array(["public"] * len(fields), pa.string()),
                    "table_name": pa.array([name] * len(fields), pa.string()), **cols}
        return QueryResult(pa.table(cols), 0.0)

    def _insert(self, st) -> QueryResult:
        """INSERT INTO t [(cols)] VALUES ... | SELECT ...: appends to an
        in-memory table (the new rows are cast to the table's column types;
        unlisted columns are NULL)."""
        from .exec.joins import concat_columns
        from .sql.expr import Cast, Lit
        name = st["s"]
        src = self.catalog.get_table(name)
        if src is None:
            raise TableNotFound(f"table '{name}' not found")
        if not isinstance(src, MemoryTable):
            raise NotSupported(f"INSERT INTO '{name}': only in-memory tables accept inserts")
        fields = list(src.schema())
        target = [c["s"] for c in (st.get("columns") or {}).get("c", [])] or [f.name for f in fields]
        known = {f.name: f for f in fields}
        for c in target:
            if c not in known:
                raise PlanError(f"column '{c}' not found in '{name}'")
        b = Binder(self.catalog, self._ids, self.session)
        bq = b.bind_query(st["query"])
        if len(bq.plan.schema) != len(target):
            raise PlanError(f"INSERT has {len(bq.plan.schema)} columns but {len(target)} target columns")
        plan = bq.plan
        exprs = []
        by_name = dict(zip(target, plan.schema))
        for f in fields:
            ci = ColInfo(b.ids(), f.name, f.dtype, True)
            if f.name in by_name:
                e = by_name[f.name].ref()
                exprs.append((ci, e if e.dtype == f.dtype else Cast(e, f.dtype)))
            else:
                if not f.nullable:
                    raise PlanError(f"column '{f.name}' of '{name}' is NOT NULL and has no value")
                exprs.append((ci, Lit(None, f.dtype)))
        plan = Project(plan, exprs)
        batch = self._execute_plan(optimize(plan))
        dev = next(iter(src.columns.values())).device if src.columns else self.device
        new = {}
        for (ci, _), f in zip(exprs, fields):
            col = batch.columns[ci.cid].to(dev)
            if col.dtype.is_string and col.is_dict:
                from .ops import strings as S
                col = S.decode(col)
            old = src.columns[f.name]
            if old.is_dict:
                from .ops import strings as S
                old = S.decode(old)
            new[f.name] = concat_columns([old, col]) if src.num_rows() else col
        fl = [Field(f.name, f.dtype, f.nullable or new[f.name].valid is not None) for f in fields]
        self.register_table(name, MemoryTable(new, src.num_rows() + batch.num_rows, fields=fl))
        return QueryResult(pa.table({"count": pa.array([batch.num_rows], pa.int64())}), 0.0)

    def _create_external(self, st) -> QueryResult:
        name = st["s"]
        fmt = st.get("stored_as", "PARQUET").upper()
        loc = st.get("location")
        if not loc:
            raise PlanError("CREATE EXTERNAL TABLE requires LOCATION")
        cols = st.get("columns", {}).get("c", []) if st.get("columns") else []
        schema = [Field(c["s"], T.parse_type_name(c["type"]), not c.get("not_null")) for c in cols] or None
        if fmt == "PARQUET":
            self.register_parquet(name, loc)
        elif fmt == "CSV":
            self.register_csv(name, loc, schema=schema, has_header=bool(st.get("header")),
                              delimiter=st.get("delimiter", ","))
        elif fmt == "ICEBERG":
            self.register_iceberg(name, loc)
        elif fmt in ("JSON", "NDJSON"):
            self.register_json(name, loc, schema=schema)
        else:
            raise NotSupported(f"STORED AS {fmt}")
        return QueryResult(pa.table({}), 0.0)

    def _cache_plan(self, key, plan_names) -> None:
        self._plans[key] = plan_names
        while len(self._plans) > PLAN_CACHE_SIZE:
            self._plans.popitem(last=False)

    def _record_template(self, sql: str, st: dict, lx, tkey):
        """Plan ``st`` while recording it as a statement template
        (sql/template.py), verify the template against a plan of the same
        statement with perturbed literals, and keep it when they agree.
        Returns this statement's (plan, names) or None (plan it normally)."""
        slots = TPL.annotate(st, lx)
        if slots is None:
            return None
        try:
            with TPL.recording() as rec:
                bq = Binder(self.catalog, IdGen(), self.session).bind_query(st)
                plan = optimize(bq.plan)
        except IglooError:
            raise
        except Exception:       # noqa: BLE001 - recording failed: plan without a template
            return None
        ent = TPL.Template(plan, bq.names, lx, slots, rec)
        own = ent.instantiate(lx.texts, Binder.literal_of)
        if own is None:
            return None
        self.template_stats["recorded"] += 1
        ptexts = TPL.perturb(lx.texts, lx.kinds, slots)
        for s_ in ent.keyed:
            ptexts[s_] = lx.texts[s_]
        psql = TPL.render(sql, lx, ptexts)
        ok = False
        plx = TPL.lex(psql)
        if ptexts != lx.texts and plx is not None and plx.key == lx.key:
            try:
                pst = parse(psql)
                pbq = Binder(self.catalog, IdGen(), self.session).bind_query(pst[0])
                pplan = optimize(pbq.plan)
                inst = ent.instantiate(ptexts, Binder.literal_of)
                ok = inst is not None and inst[1] == pbq.names and TPL.signature(inst[0]) == TPL.signature(pplan)
            except Exception:   # noqa: BLE001 - the perturbed statement does not plan: unverified
                ok = False
        ent.verified = ok
        self.template_stats["verified" if ok else "rejected"] += 1
        self._templates[tkey] = ent
        while len(self._templates) > TEMPLATE_CACHE_SIZE:
            self._templates.popitem(last=False)
        return own

    def _plan_query(self, st: dict):
        b = Binder(self.catalog, self._ids, self.session)
        bq = b.bind_query(st)
        return optimize(bq.plan), bq.names

    def _run_query(self, st: dict, t0: float) -> QueryResult:
        plan, names = self._plan_query(st)
        return self._exec_query(plan, names, t0)

    def _exec_query(self, plan, names, t0: float, cached: bool = False, key=None, planned=None) -> QueryResult:
        """Execute an optimized logical plan. A cached plan is only the
        parse / bind / optimize output for the same SQL text, catalog version
        and session settings: every execution builds fresh physical operators
        and recomputes everything from the tables (scalar subqueries included)."""
        bq_names = names
        ctx = self.make_context()
        c0 = (self.comm.calls, self.comm.bytes_sent, self.comm.chunk_calls) if self.comm is not None else (0, 0, 0)
        from .ops._lib import HOST_STEPS, READBACKS
        h0 = sum(HOST_STEPS.values())
        r0 = READBACKS[0]
        cs0 = (self.cache.stats["hits"], self.cache.stats["misses"])
        gpu = self.device.type == "cuda"
        if gpu:
            # per-query HBM high-water mark and device-side span (one event pair;
            # the result readback below already synchronises the stream)
            torch.cuda.reset_peak_memory_stats(self.device)
            mem0 = _allocated(self.device, "current")
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        with _trace.Range("query"):
            batch, spec, st, table = self._execute_speculative(plan, ctx, key, bq_names)
        if table is None:
            guard = st.pop("pending_guard", None) if st is not None else None
            try:
                table = self._to_arrow(batch, plan.schema, bq_names, guard=guard)
            except _ReplayMismatch:
                # a checked graph's replayed values did not match this time:
                # drop it and run the query again with real readbacks
                self._graph_mismatch(st)
                ctx = self.make_context()
                with _trace.Range("query"):
                    batch, spec, st, table = self._execute_speculative(plan, ctx, key, bq_names)
                if table is None:
                    table = self._to_arrow(batch, plan.schema, bq_names)
        dev_metrics = {}
        if gpu:
            ev1.record()
            ev1.synchronize()
            peak = _allocated(self.device, "peak")
            self.hbm_peak_bytes = max(self.hbm_peak_bytes, peak)
            dev_metrics = {"device_span_ms": round(ev0.elapsed_time(ev1), 3), "hbm_peak_bytes": int(peak),
                           "hbm_query_bytes": int(max(0, peak - mem0))}
        hits, misses = self.cache.stats["hits"] - cs0[0], self.cache.stats["misses"] - cs0[1]
        if st is not None and spec in ("replayed", "recorded") and st["capture_next"]:
            st["digest"] = digest(table)      # the next execution's graph must reproduce it
        if spec != "graph":
            self.cache.enforce()   # derived structures built by this query count against the budget
        ms = (time.perf_counter() - t0) * 1e3
        self.last_metrics = {"elapsed_ms": ms, "rows": table.num_rows, "rows_scanned": ctx.rows_scanned,
                             "spill": dict(ctx.spill), "morsels": dict(ctx.morsels), "plan_cached": cached, "speculation": spec,
                             "plan_source": "cache" if cached else (planned or "planned"),
                             # work that left the GPU (ops/_lib.py note_host_step)
                             "host_steps": sum(HOST_STEPS.values()) - h0,
                             # blocking device -> host readbacks (result copy excluded)
                             "readbacks": READBACKS[0] - r0,
                             "cache": {"hits": hits, "misses": misses,
                                       "hit_ratio": round(hits / (hits + misses), 4) if hits + misses else None},
                             **dev_metrics}
        if self.comm is not None:
            # ``exchanges``: collectives with each pipelined exchange's chunks counted once
            self.last_metrics.update(collectives=self.comm.calls - c0[0], exchange_bytes=self.comm.bytes_sent - c0[1],
                                     exchanges=(self.comm.calls - c0[0]) - (self.comm.chunk_calls - c0[2]))
        return QueryResult(table, ms)

    def explain_fragments(self, sql: str, workers=("all-ranks",)) -> str:
        """Stage DAG of ``sql`` (fragments, placement, exchanges)."""
        from .parallel.fragments import DistributedPlanner, explain_fragments
        plan, _ = self.logical_plan(sql)
        return explain_fragments(DistributedPlanner(workers).plan(plan))

    def execute_logical(self, plan: Plan, names: Optional[List[str]] = None) -> pa.Table:
        """Run an (optimized) logical plan — e.g. one deserialized from a fragment
        request — and return its Arrow result."""
        names = names or [c.name for c in plan.schema]
        return self._to_arrow(self._execute_plan(plan), plan.schema, names)

    def make_context(self, analyze: bool = False) -> ExecContext:
        return ExecContext(self, self.device, self.comm, analyze)

    def _execute_speculative(self, plan: Plan, ctx: ExecContext, key, names=None):
        """Run the plan; for a repeated query over unchanged data, replay the
        host readbacks (sizes, ranges, strategy choices) of the previous
        executions instead of waiting on the device for each (ops/_lib.py
        Speculation): the host enqueues the whole query while the GPU runs it,
        and one sync at the end checks every replayed value against the device.
        A recording is replayed once two executions produced the same call
        sequence (values that differed between them are read back for real
        every time); a replay that leaves the recorded sequence continues with
        real readbacks and needs re-confirming; a value mismatch re-executes the query with
        real readbacks (after two, the query is no longer replayed).

        Only byte-identical SQL over unchanged data replays: a replayed value
        sizes device buffers before the device confirms it, so handing a new
        statement of the same template (literals masked) the readbacks of an
        earlier one is unsafe -- a value that matched across earlier statements
        but follows the parameters undersizes a buffer and the kernels writing
        it fault (tried: a GPU memory fault on TPC-H with fresh parameters).

        SPMD ranks (one per GPU) speculate too: replaying a readback changes
        only when the host waits, never which collectives a rank issues, so
        ranks in different modes stay aligned. Every rank joins ONE tiny
        all-reduce after each execution: it agrees on the validation (and on
        a fresh graph's first-result digest) and on whether every rank is
        ready to capture, so ranks capture their query graphs together; a rank
        that cannot runs eagerly, which issues the same collectives. Graphs
        with collectives inside need a device transport (RCCL): a gloo
        (host-staged) group never captures."""
        from .ops import _lib
        spmd = self.comm is not None and self.comm.spmd
        if not (SPECULATE and key is not None and self.device.type == "cuda" and (not spmd or SPMD_SPECULATE)):
            return self._execute_plan(plan, ctx), None, None, None
        comm = self.comm if spmd else None
        graphs_on = _graphs.GRAPHS and (comm is None or (comm.backend == "nccl" and SPMD_GRAPHS))

        def agree(*flags: bool) -> List[bool]:
            # SPMD ranks decide together: every rank joins this ONE tiny
            # all-reduce after every speculative-capable execution, so their
            # collective sequences stay aligned; a flag is set when any rank set it
            if comm is None:
                return [bool(f) for f in flags]
            return [v > 0 for v in comm.allreduce_ints([int(bool(f)) for f in flags])]
        # CDC: a graph replay never reaches CachedTable.scan (where scans poll
        # their source), so the probes of the tables this query read last time
        # run here, rate-limited the same way; a changed source invalidates its
        # cache entries and moves the cache generation, i.e. the key below
        srcs = self._query_sources.get(key, ())
        for s in srcs:
            try:
                s.poll()
            except Exception as e:  # noqa: BLE001 - a failing probe keeps the cached data
                log.warning("cdc poll of %s failed: %s", getattr(s, "name", s), e)
        # (a generated kernel that becomes available changes the code path and
        # so the readback call sites: the replay diverges, stays correct, and the
        # new sequence is confirmed by the next execution)
        skey = (key, self.catalog.version, self.cache.generation, tuple(s.cdc_version() for s in srcs))
        st = self._spec.get(skey)
        if st is None:
            old = self._spec_current.pop(key, None)
            if old is not None:
                # the data this query's recording (and graph) was built on changed
                ost = self._spec.pop(old, None)
                if ost is not None and ost.get("graph") is not None:
                    self.graph_stats["dropped_stale"] += 1
                    self._set_graph(ost, None)
            if len(self._spec) >= PLAN_CACHE_SIZE:
                self._set_graph(self._spec.pop(next(iter(self._spec))), None)
            st = self._spec[skey] = {"log": None, "candidate": None, "fails": 0, "graph": None,
                                     "capture_next": False, "digest": None, "graph_aborts": 0,
                                     "cache_keys": ()}
            self._spec_current[key] = skey
        replay = st["log"] is not None and st["fails"] < 2
        g = st["graph"] if graphs_on else None
        if g is not None and not g.current():
            # the generated-kernel set changed: the recording diverges from
            # here, and a new graph is captured once a replay completes again
            self._set_graph(st, None)
            g = None
        if g is None and st["capture_next"] and graphs_on and replay and st["fails"] == 0 \
                and st["graph_aborts"] < 2:
            # capture_next was agreed by every rank, so ranks normally capture
            # together; a rank whose capture is refused simply runs eagerly
            # (a graph and an eager execution issue the same collectives)
            st["capture_next"] = False
            if self.graphs_disabled or not self._capture(st, plan):
                st["graph_aborts"] += 1
            g = st["graph"]
        if g is not None and g.checked and (comm is None or g.global_check):
            # a verified graph: launch it and let the result's host copy carry
            # its mismatch count (one sync per query, not two). Under SPMD the
            # count was summed over the ranks inside the graph, so every rank
            # reads the same value and all re-execute together on a mismatch.
            g.launch(ctx)
            if comm is not None:
                comm.calls += g.comm_calls
                comm.chunk_calls += g.comm_chunks
                comm.bytes_sent += g.comm_bytes
            self._touch_graph(st)
            st["pending_guard"] = g.bad
            return g.batch, "graph", st, None
        if g is not None:
            ok = g.replay(ctx)
            table = None
            if ok and not g.checked:
                # first replay: its result must equal the eager execution's
                table = self._to_arrow(g.batch, plan.schema, names)
                ok = digest(table) == st["digest"]
                if not ok:
                    log.warning("query graph result differs from the eager execution; graph dropped")
                    _graphs.STATS["failed"] += 1
                    st["graph_aborts"] = 2
            if comm is not None:
                comm.calls += g.comm_calls
                comm.chunk_calls += g.comm_chunks
                comm.bytes_sent += g.comm_bytes
            # a checked graph's mismatch count is already summed over the ranks
            # inside the graph: every rank read the same value
            any_bad = (not ok) if (g.checked and g.global_check) else agree(not ok, True)[0]
            if not any_bad:
                g.checked = True
                self._touch_graph(st)
                return g.batch, "graph", st, table
            # a replayed value (or the first result) did not match on some
            # rank: every rank drops its graph and re-executes eagerly with
            # real readbacks (the same collectives on all)
            self._set_graph(st, None)
            st["fails"] += 1
            st["log"] = st["candidate"] = None
            replay = False
            ctx = self.make_context()
            log.warning("query graph: replayed values did not match the device; re-executing")
        for attempt in range(3):
            sp = _lib.Speculation("replay" if replay else "record", st["log"] if replay else None)
            _lib.set_speculation(sp)
            failed = None
            try:
                batch = self._execute_plan(plan, ctx, fold_checks=True)
            except Exception as e:  # noqa: BLE001 - re-raised unless a replayed value caused it
                # a replayed value that does not match the data can also stop
                # the host side of a query (a shape or range it cannot hold):
                # on one rank that is a mismatch like any other -- re-execute
                # with real readbacks. (SPMD ranks re-raise: the others may be
                # inside a collective this rank will not reach.)
                if sp.mode != "replay" or comm is not None:
                    raise
                failed = e
            finally:
                _lib.set_speculation(None)
            ok = failed is None and sp.validate()
            if failed is not None:
                log.warning("replayed readbacks stopped the query (%s); re-executing", failed)
            # would this rank capture next time (a complete replay, or a
            # recording confirmed by this run)? Agreed with the validation:
            # ranks capture only together
            ready = graphs_on and ok and st["fails"] == 0 and st["graph"] is None and st["graph_aborts"] < 2 \
                and not self.graphs_disabled and _jit.generation() is not None and (
                    sp.complete if sp.mode == "replay" else _confirm(st["candidate"], sp.log) is not None)
            bad, not_ready = agree(not ok, not ready)
            if not bad:
                break
            # some rank's replayed value did not match its device: every rank
            # re-executes with real readbacks (the same collectives on all)
            if replay:
                st["fails"] += 1
            st["log"] = st["candidate"] = None
            replay = False
            ctx = self.make_context()
            log.warning("speculative readbacks did not match the device; re-executing")
        self._query_sources[key] = [s for s in ctx.sources if hasattr(s, "poll")]
        st["cache_keys"] = tuple(dict.fromkeys(ctx.cache_keys))
        if not bad and not not_ready:
            st["capture_next"] = True       # _exec_query keeps this result's digest
        if sp.mode == "replay":
            if not sp.complete:
                # the call sequence changed: this run's own sequence must be
                # confirmed by the next execution before it is replayed
                st["log"], st["candidate"] = None, sp.fresh
            return batch, "replayed" if sp.complete else "partial", st, None
        st["log"] = _confirm(st["candidate"], sp.log)
        st["candidate"] = sp.log if st["log"] is None else None
        return batch, "recorded", st, None

    def _graph_mismatch(self, st: dict) -> None:
        """Drop ``st``'s graph after a replay whose values the device did not
        confirm; the query re-executes eagerly with real readbacks."""
        _graphs.STATS["mismatch"] += 1
        log.warning("query graph: replayed values did not match the device; re-executing")
        self._set_graph(st, None)
        st["fails"] += 1
        st["log"] = st["candidate"] = None

    def _capture(self, st: dict, plan: Plan) -> bool:
        """Capture ``plan`` under a replay of ``st``'s recording into a query graph."""
        if st["digest"] is None:
            return False
        c0 = (self.comm.calls, self.comm.bytes_sent, self.comm.chunk_calls) if self.comm is not None else (0, 0, 0)
        with _trace.Range("graph.capture"):
            g = _graphs.capture(self, plan, st["log"], self.make_context)
        if g is None:
            return False
        if self.comm is not None:
            # collectives recorded into the graph (counted again on every replay)
            g.comm_calls, g.comm_bytes = self.comm.calls - c0[0], self.comm.bytes_sent - c0[1]
            g.comm_chunks = self.comm.chunk_calls - c0[2]
            self.comm.calls, self.comm.bytes_sent, self.comm.chunk_calls = c0
        self._set_graph(st, g)
        return True

    # ------------------------------------------------------- graph memory
    def _set_graph(self, st: dict, g) -> None:
        """Attach (or drop, ``g=None``) ``st``'s query graph, keeping the
        graphs' pool bytes accounted against ``hbm_budget``."""
        old = st.get("graph")
        if old is not None:
            self._graphs.pop(id(st), None)
            self.graph_bytes -= old.nbytes
        st["graph"] = g
        if g is not None:
            self._graphs[id(st)] = st
            self.graph_bytes += g.nbytes
            self.enforce_graph_budget(keep=st)

    def _touch_graph(self, st: dict) -> None:
        if id(st) in self._graphs:
            self._graphs.move_to_end(id(st))
        if st["cache_keys"]:
            self.cache.touch(st["cache_keys"])   # the replay read these resident columns

    def enforce_graph_budget(self, keep: Optional[dict] = None) -> int:
        """Drop least recently replayed graphs while the cache tier's resident
        bytes plus the graphs' pool bytes exceed ``hbm_budget``; returns how
        many were dropped. A dropped graph's query runs eagerly (replayed
        readbacks) and may be captured again later."""
        if self.hbm_budget is None or not self._graphs:
            return 0
        n = 0
        used = self.cache.hbm_used
        while self._graphs and used + self.graph_bytes > self.hbm_budget:
            sid = next(iter(self._graphs))
            st = self._graphs[sid]
            if st is keep:
                if len(self._graphs) == 1:
                    break
                self._graphs.move_to_end(sid)
                continue
            self._set_graph(st, None)
            self.graph_stats["evicted"] += 1
            n += 1
        if n and self.device.type == "cuda":
            torch.cuda.empty_cache()      # the dropped graphs' private pools
        return n

    def close(self) -> None:
        """Drop every query graph (and its memory pool). Call before tearing
        down an RCCL process group: a live graph that captured collectives
        keeps ``destroy_process_group`` from returning (scripts/rccl_probe.py)."""
        for st in list(self._graphs.values()):
            self._set_graph(st, None)
        for st in self._spec.values():
            st["graph"] = None
        if self.device.type == "cuda":
            import gc
            gc.collect()
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()

    def graph_pool(self):
        """The private memory pool every query graph of this engine captures into."""
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        return self._graph_pool

    def _execute_plan(self, plan: Plan, ctx: Optional[ExecContext] = None, fold_checks: bool = False) -> Batch:
        """Run ``plan``. ``fold_checks``: the deferred device error flags are
        attached to the result (``Batch.deferred``) and checked by its host
        copy (``_to_arrow``), saving the query a readback; every caller passing
        it converts the result with ``_to_arrow``."""
        ctx = ctx or self.make_context()
        ctx.slices = self._slices_for(plan)
        node = create_physical_plan(plan)
        from .ops import hashing as _H
        tok = _H.TABLE_BYTES_LIMIT.set(ctx.budget // 4 if ctx.budget else None)
        try:
            out = node.execute(ctx)
        finally:
            _H.TABLE_BYTES_LIMIT.reset(tok)
        if self.comm is not None and self.comm.spmd:
            from .parallel.exchange import gather_all
            out = gather_all(out, ctx)
        if fold_checks and ctx.deferred_checks:
            out.deferred = ctx.take_deferred()
        else:
            ctx.check_deferred()
        return out

    def _slices_for(self, plan: Plan) -> Dict[int, str]:
        """SPMD: the replicated table a query over replicated tables only
        splits by key range (parallel/slicing.py)."""
        if self.comm is None or not self.comm.spmd or not SLICE_REPLICATED:
            return {}
        from .parallel.slicing import plan_slices
        return plan_slices(plan, self.comm)

    def _to_arrow(self, batch: Batch, schema: List[ColInfo], names: List[str], guard=None) -> pa.Table:
        arrays, fields = [], []
        host = _host_columns([batch.columns[ci.cid] for ci in schema], getattr(batch, "deferred", None), guard)
        for ci, nm, col in zip(schema, names, host):
            arr = col.to_arrow()
            want = ci.dtype.to_arrow() if ci.dtype.kind != "null" else pa.null()
            if arr.type != want:
                try:
                    arr = arr.cast(want)
                except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                    pass
            nullable = ci.nullable or arr.null_count > 0
            arrays.append(arr)
            fields.append(pa.field(nm, arr.type, nullable))
        return pa.Table.from_arrays(arrays, schema=pa.schema(fields))

    def _explain(self, st: dict, analyze: bool) -> QueryResult:
        b = Binder(self.catalog, self._ids, self.session)
        bq = b.bind_query(st)
        logical = optimize(bq.plan)
        node = create_physical_plan(logical)
        rows_t, rows_p = ["logical_plan", "physical_plan"], [logical.explain(), node.explain()]
        if analyze:
            from .ops._lib import HOST_STEPS
            ctx = self.make_context(analyze=True)
            ctx.slices = self._slices_for(logical)
            c0 = (self.comm.calls, self.comm.bytes_sent, self.comm.chunk_calls) if self.comm is not None else (0, 0, 0)
            h0 = dict(HOST_STEPS)
            t0 = time.perf_counter()
            node.execute(ctx)
            ctx.check_deferred()
            ms = (time.perf_counter() - t0) * 1e3
            rows_t = ["physical_plan_with_metrics"]
            txt = node.explain(ctx) + f"\ntotal: {ms:.3f} ms"
            for n in _walk_exec(node):
                if getattr(n, "order_log", None):
                    txt += "\njoin order: " + " ; ".join(n.order_log)
            if ctx.morsels["pipelines"]:
                m = ctx.morsels
                txt += (f"\nmorsels: {m['pipelines']} pipeline(s), {m['morsels']} morsels, {m['rows']} rows, "
                        f"{m['bytes']} bytes streamed (device budget {ctx.budget} bytes)")
            if ctx.spill["joins"] or ctx.spill.get("sorts"):
                txt += (f"\nspill: {ctx.spill['joins']} partitioned join(s), {ctx.spill['partitions']} partitions, "
                        f"{ctx.spill.get('sorts', 0)} external sort(s), {ctx.spill.get('sort_runs', 0)} sort runs, "
                        f"{ctx.spill['bytes']} bytes staged in host memory (device budget {ctx.budget} bytes)")
            if self.comm is not None and self.comm.spmd:
                txt += (f"\nexchange: {self.comm.calls - c0[0]} collectives, "
                        f"{self.comm.bytes_sent - c0[1]} bytes sent by this rank")
            host = {k: v - h0.get(k, 0) for k, v in HOST_STEPS.items() if v - h0.get(k, 0)}
            if self.device.type == "cuda":
                txt += "\nhost steps: " + (", ".join(f"{k} x{v}" for k, v in host.items()) if host else "none")
            if ctx.spans:
                txt += "\nphases (inclusive, synchronised):\n" + ctx.span_report()
            rows_p = [txt]
        return QueryResult(pa.table({"plan_type": rows_t, "plan": rows_p}), 0.0)


def _walk_exec(n):
    yield n
    for c in n.children:
        yield from _walk_exec(c)


def pretty_format(table: pa.Table, max_rows: int = 50) -> str:
    """ASCII table like arrow's print_batches (reference crates/igloo/src/main.rs:92)."""
    names = table.column_names
    rows = table.slice(0, max_rows).to_pylist()
    cells = [[("" if r[n] is None else str(r[n])) for n in names] for r in rows]
    widths = [max([len(n)] + [len(c[i]) for c in cells]) for i, n in enumerate(names)]
    sep = "+" + "+".join("-" * (w + 2) for w in widths) + "+"
    out = [sep, "|" + "|".join(f" {n:<{w}} " for n, w in zip(names, widths)) + "|", sep]
    for c in cells:
        out.append("|" + "|".join(f" {v:<{w}} " for v, w in zip(c, widths)) + "|")
    out.append(sep)
    if table.num_rows > max_rows:
        out.append(f"... {table.num_rows - max_rows} more rows")
    return "\n".join(out)


def print_batches(batches) -> None:
    if isinstance(batches, QueryResult):
        t = batches.table
    elif isinstance(batches, pa.Table):
        t = batches
    else:
        t = pa.Table.from_batches(list(batches)) if batches else pa.table({})
    print(pretty_format(t))
