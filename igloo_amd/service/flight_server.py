"""Arrow Flight / Flight SQL endpoint (coordinator and worker groups).

Parity: reference crates/api/src/lib.rs:40-184 (IglooFlightSqlService):
* GetFlightInfo: ``FlightDescriptor.cmd`` = UTF-8 SQL (empty -> InvalidArgument);
  the reference EXECUTES the whole query just to learn the schema (:91) —
  here the query is only planned (bind + optimize) and the schema comes from
  the plan; the endpoint ticket carries the query;
* DoGet: ``Ticket.ticket`` = UTF-8 SQL (bad UTF-8 -> InvalidArgument), result
  streamed as Arrow IPC; an empty result answers NotFound like the reference
  (:125-128), except for Flight SQL tickets, which stream a schema-only result;
* everything else was Unimplemented — here DoAction carries the control plane
  (register_worker, heartbeat, execute_task, get_data_for_task, list_workers,
  metrics, explain, health), ListFlights lists catalog tables, GetSchema plans,
  DoPut ingests a table into the HBM tier, and Handshake/middleware check an
  optional bearer token (reference auth.proto is an empty stub).

Flight SQL (protobuf ``Any`` commands decoded by ``protocol.unpack_any``; no
Flight SQL library ships here; service/flight_sql.py): statements
(``CommandStatementQuery`` / ``TicketStatementQuery``), metadata
(``CommandGetSqlInfo``, ``GetCatalogs``, ``GetDbSchemas``, ``GetTables`` with
or without schemas, ``GetTableTypes``, primary / exported / imported keys,
cross reference), prepared statements (DoAction ``CreatePreparedStatement`` /
``ClosePreparedStatement``, ``CommandPreparedStatementQuery`` with ``?``
parameters bound by DoPut) and updates (DoPut ``CommandStatementUpdate`` /
``CommandPreparedStatementUpdate``). GetFlightInfo and GetSchema answer every
command from its plan or fixed schema without running it.
"""
from __future__ import annotations

import json
import threading
import time
import uuid
from typing import Callable, Dict, Optional, Tuple

import pyarrow as pa
import pyarrow.flight as fl

from ..utils.errors import CommError, DeviceError, IglooError, PlanError, SqlParseError, TableNotFound
from ..utils.log import get_logger
from . import flight_sql as FS
from . import protocol as P

log = get_logger("flight")


class _TokenMiddlewareFactory(fl.ServerMiddlewareFactory):
    def __init__(self, token: str):
        self.token = token

    def start_call(self, info, headers):
        auth = headers.get("authorization") or headers.get("Authorization") or []
        ok = any(h == f"Bearer {self.token}" for h in auth)
        if not ok:
            raise fl.FlightUnauthenticatedError("missing or invalid bearer token")
        return None


class IglooFlightServer(fl.FlightServerBase):
    """Serves an engine (local GPU) or forwards queries to a runner callable
    (e.g. the coordinator's distributed executor)."""

    def __init__(self, engine, location: str = "grpc://127.0.0.1:50051", registry=None,
                 runner: Optional[Callable[[str], pa.Table]] = None, auth_token: Optional[str] = None,
                 task_handler: Optional[Callable[[P.TaskDefinition], P.TaskStatus]] = None,
                 fragment_runner: Optional[Callable[[bytes], pa.Table]] = None, **kw):
        mw = {"auth": _TokenMiddlewareFactory(auth_token)} if auth_token else None
        super().__init__(location, middleware=mw, **kw)
        self.engine = engine
        self.registry = registry
        self.runner = runner
        self.task_handler = task_handler
        self.fragment_runner = fragment_runner
        self._pending: Dict[str, Tuple[str, float]] = {}
        self._results: Dict[str, pa.Table] = {}
        self._lock = threading.Lock()
        self._session_lock = threading.Lock()   # per-request session settings (execute_query)
        self.metrics = {"queries": 0, "rows": 0, "errors": 0, "ms": 0.0}
        self._location = location
        self.prepared = FS.PreparedStatements()
        self.meta = FS.Metadata(engine) if engine is not None else None

    def start_background(self, timeout_s: float = 30.0, host: str = "127.0.0.1") -> "IglooFlightServer":
        """Serve on a daemon thread and return once the endpoint answers."""
        self._serve_thread = threading.Thread(target=self.serve, daemon=True, name="igloo-flight")
        self._serve_thread.start()
        client = fl.connect(f"grpc://{host}:{self.port}")
        deadline = time.time() + timeout_s
        while True:
            try:
                list(client.do_action(fl.Action("health", b""), fl.FlightCallOptions(timeout=1.0)))
                break
            except fl.FlightUnauthenticatedError:
                break  # up, just protected by a token
            except Exception:  # noqa: BLE001
                if time.time() > deadline:
                    raise
                time.sleep(0.02)
        client.close()
        return self

    # ------------------------------------------------------------- helpers
    @staticmethod
    def _sql_from_bytes(b: bytes) -> Tuple[str, bool, Optional[str]]:
        """-> (sql, is_flight_sql, statement handle)."""
        a = P.unpack_any(b) if b else None
        if a is not None:
            name, f = a
            if name == "CommandStatementQuery":
                return f.get(1, [b""])[0].decode(), True, None
            if name == "TicketStatementQuery":
                return "", True, f.get(1, [b""])[0].decode()
            raise NotImplementedError(f"Flight SQL command {name} is not supported")
        try:
            return b.decode("utf-8"), False, None
        except UnicodeDecodeError:
            raise ValueError("ticket/command is not valid UTF-8") from None

    @staticmethod
    def _flight_sql(b: bytes):
        """(command name, fields) of a Flight SQL command other than a
        statement query / ticket, else None."""
        a = P.unpack_any(b) if b else None
        if a is None or a[0] in ("CommandStatementQuery", "TicketStatementQuery"):
            return None
        return a

    def _command_schema(self, name: str, f) -> pa.Schema:
        sch = FS.metadata_schema(name, f)
        if sch is not None:
            return sch
        if name == "CommandPreparedStatementQuery":
            h = f.get(1, [b""])[0]
            st = self.prepared.get(h)
            if st["schema"] is None:
                if not _is_query(st["sql"]):
                    raise ValueError("prepared statement is an update: it has no result set (DoPut it)")
                st["schema"] = self._schema_of(self.prepared.sql_of(h))
            return st["schema"]
        raise NotImplementedError(f"Flight SQL command {name} is not supported")

    def _version(self) -> str:
        from .. import __version__
        return __version__

    def _run_with_session(self, sql: str, session_config) -> pa.Table:
        """Run with the request's session settings applied for this query only."""
        eng = self.engine
        if not session_config or eng is None or self.runner is not None:
            return self._run(sql)
        with self._session_lock:
            saved = dict(eng.session)
            eng.session.update(session_config)
            try:
                return self._run(sql)
            finally:
                eng.session.clear()
                eng.session.update(saved)

    def _run(self, sql: str) -> pa.Table:
        t0 = time.perf_counter()
        try:
            t = self.runner(sql) if self.runner is not None else self.engine.query(sql)
        except (SqlParseError, PlanError, TableNotFound) as e:
            self.metrics["errors"] += 1
            raise ValueError(f"{type(e).__name__}: {e}") from None
        except (DeviceError, CommError) as e:
            # the worker group (GPU / collective), not the query, failed: retryable elsewhere
            self.metrics["errors"] += 1
            raise fl.FlightUnavailableError(f"{type(e).__name__}: {e}") from None
        except IglooError as e:
            self.metrics["errors"] += 1
            raise fl.FlightServerError(f"{type(e).__name__}: {e}") from None
        self.metrics["queries"] += 1
        self.metrics["rows"] += t.num_rows
        self.metrics["ms"] += (time.perf_counter() - t0) * 1e3
        return t

    def _schema_of(self, sql: str) -> pa.Schema:
        try:
            plan, names = self.engine.logical_plan(sql)
        except (SqlParseError, PlanError, TableNotFound) as e:
            raise ValueError(f"{type(e).__name__}: {e}") from None
        return pa.schema([pa.field(n, c.dtype.to_arrow() if c.dtype.kind != "null" else pa.null(), c.nullable)
                          for c, n in zip(plan.schema, names)])

    # ------------------------------------------------------------ Flight API
    def get_flight_info(self, context, descriptor):
        if descriptor.descriptor_type == fl.DescriptorType.PATH:
            name = descriptor.path[0].decode() if isinstance(descriptor.path[0], bytes) else descriptor.path[0]
            sql = f"SELECT * FROM {name}"
            flight_sql = False
        else:
            if not descriptor.command:
                raise ValueError("empty SQL command")
            cmd = self._flight_sql(descriptor.command)
            if cmd is not None:
                # metadata / prepared statements: the command itself is the ticket
                schema = self._command_schema(*cmd)
                return fl.FlightInfo(schema, descriptor,
                                     [fl.FlightEndpoint(fl.Ticket(descriptor.command), [self._location])], -1, -1)
            sql, flight_sql, _ = self._sql_from_bytes(descriptor.command)
            if not sql.strip():
                raise ValueError("empty SQL command")
        schema = self._schema_of(sql)
        if flight_sql:
            handle = uuid.uuid4().hex
            with self._lock:
                self._pending[handle] = (sql, time.time())
            ticket = fl.Ticket(P.ticket_statement_query(handle.encode()))
        else:
            ticket = fl.Ticket(sql.encode())
        return fl.FlightInfo(schema, descriptor, [fl.FlightEndpoint(ticket, [self._location])], -1, -1)

    def get_schema(self, context, descriptor):
        if descriptor.descriptor_type == fl.DescriptorType.PATH:
            name = descriptor.path[0].decode() if isinstance(descriptor.path[0], bytes) else descriptor.path[0]
            return fl.SchemaResult(self._schema_of(f"SELECT * FROM {name}"))
        cmd = self._flight_sql(descriptor.command)
        if cmd is not None:
            return fl.SchemaResult(self._command_schema(*cmd))
        sql, _, _ = self._sql_from_bytes(descriptor.command)
        return fl.SchemaResult(self._schema_of(sql))

    def do_get(self, context, ticket):
        cmd = self._flight_sql(ticket.ticket)
        if cmd is not None:
            name, f = cmd
            if name == "CommandPreparedStatementQuery":
                sql = self.prepared.sql_of(f.get(1, [b""])[0])
                return fl.RecordBatchStream(self._run(sql))
            if self.meta is None:
                raise NotImplementedError("this endpoint has no catalog")
            return fl.RecordBatchStream(FS.metadata_result(self.meta, name, f, self._version()))
        sql, flight_sql, handle = self._sql_from_bytes(ticket.ticket)
        if handle is not None:
            with self._lock:
                ent = self._pending.pop(handle, None)
            if ent is None:
                raise KeyError(f"unknown statement handle {handle}")
            sql = ent[0]
        if not sql.strip():
            raise ValueError("empty SQL ticket")
        t = self._run(sql)
        if t.num_rows == 0 and not flight_sql:
            raise KeyError("No results")
        return fl.RecordBatchStream(t)

    def do_put(self, context, descriptor, reader, writer):
        if descriptor.descriptor_type == fl.DescriptorType.CMD:
            cmd = P.unpack_any(descriptor.command)
            if cmd is None:
                raise ValueError("DoPut command is not a Flight SQL command")
            name, f = cmd
            if name == "CommandPreparedStatementQuery":
                # bind parameter values (first row) for the next execution
                h = f.get(1, [b""])[0]
                self.prepared.bind(h, reader.read_all())
                writer.write(pa.py_buffer(P.pb_field(1, h)))     # DoPutPreparedStatementResult
                return
            if name == "CommandStatementUpdate":
                sql = f.get(1, [b""])[0].decode()
            elif name == "CommandPreparedStatementUpdate":
                h = f.get(1, [b""])[0]
                self.prepared.bind(h, reader.read_all())
                sql = self.prepared.sql_of(h)
            else:
                raise NotImplementedError(f"Flight SQL DoPut command {name} is not supported")
            res = self.engine.sql(sql)
            t = res.table
            n = int(t.column("count")[0].as_py()) if "count" in t.column_names and t.num_rows else -1
            writer.write(pa.py_buffer(FS.encode_update_result(n)))
            return
        name = descriptor.path[0].decode() if isinstance(descriptor.path[0], bytes) else descriptor.path[0]
        t = reader.read_all()
        self.engine.register_table(name, t)
        log.info("DoPut: registered %s (%d rows)", name, t.num_rows)

    def list_flights(self, context, criteria):
        for name in self.engine.catalog.table_names():
            src = self.engine.catalog.get_table(name)
            try:
                schema = src.arrow_schema()
                n = src.num_rows() or -1
            except IglooError:
                continue
            yield fl.FlightInfo(schema, fl.FlightDescriptor.for_path(name), [], n, -1)

    def list_actions(self, context):
        return [("register_worker", "WorkerInfo -> RegistrationAck"), ("heartbeat", "HeartbeatInfo -> HeartbeatResponse"),
                ("execute_task", "TaskDefinition -> TaskStatus"), ("get_data_for_task", "DataForTaskRequest -> IPC"),
                ("list_workers", "-> workers JSON"), ("metrics", "-> metrics JSON"), ("explain", "SQL -> plan text"),
                ("execute_fragment", "serialized fragment + input IPC -> IPC batch stream + QueryComplete"),
                ("execute_query", "QueryRequest JSON -> IPC batch stream + QueryComplete"), ("health", "-> ok"),
                ("CreatePreparedStatement", "Flight SQL ActionCreatePreparedStatementRequest -> Result"),
                ("ClosePreparedStatement", "Flight SQL ActionClosePreparedStatementRequest")]

    def do_action(self, context, action):
        kind, body = action.type, action.body.to_pybytes() if action.body is not None else b""
        if kind == "register_worker":
            if self.registry is None:
                raise NotImplementedError("this endpoint has no worker registry")
            yield fl.Result(self.registry.register(P.WorkerInfo.from_json(body)).to_json())
        elif kind == "heartbeat":
            if self.registry is None:
                raise NotImplementedError("this endpoint has no worker registry")
            yield fl.Result(self.registry.heartbeat(P.HeartbeatInfo.from_json(body)).to_json())
        elif kind == "execute_task":
            td = P.TaskDefinition.from_json(body)
            if self.task_handler is not None:
                st = self.task_handler(td)
            else:
                t0 = time.perf_counter()
                try:
                    res = self._run(td.payload)
                    with self._lock:
                        self._results[td.task_id] = res
                    st = P.TaskStatus("DONE", td.task_id, res.num_rows, (time.perf_counter() - t0) * 1e3)
                except Exception as e:  # noqa: BLE001 - reported to the caller
                    st = P.TaskStatus("FAILED", td.task_id, error=f"{type(e).__name__}: {e}")
            yield fl.Result(st.to_json())
        elif kind == "get_data_for_task":
            req = P.DataForTaskRequest.from_json(body)
            with self._lock:
                t = self._results.pop(req.task_id, None)
            if t is None:
                raise KeyError(f"no data for task {req.task_id}")
            sink = pa.BufferOutputStream()
            with pa.ipc.new_stream(sink, t.schema) as w:
                w.write_table(t)
            yield fl.Result(sink.getvalue())
        elif kind == "list_workers":
            yield fl.Result(json.dumps(self.registry.snapshot() if self.registry else []).encode())
        elif kind == "metrics":
            m = dict(self.metrics)
            m["engine"] = getattr(self.engine, "last_metrics", {})
            yield fl.Result(json.dumps(m, default=str).encode())
        elif kind == "explain":
            yield fl.Result(self.engine.explain(body.decode()).encode())
        elif kind == "execute_fragment":
            # streamed: one IPC stream per record batch, then QueryComplete
            from ..parallel.fragments import run_encoded_fragment, stream_results
            t0 = time.perf_counter()
            if self.fragment_runner is not None:
                t = self.fragment_runner(body)
            else:
                t = run_encoded_fragment(self.engine, body)
            self.metrics["fragments"] = self.metrics.get("fragments", 0) + 1
            for chunk in stream_results(t, (time.perf_counter() - t0) * 1e3):
                yield fl.Result(chunk)
        elif kind == "execute_query":
            # DistributedQueryService.ExecuteQuery(QueryRequest{sql, session_config})
            # -> stream of record batches + QueryComplete (reference distributed.proto)
            from ..parallel.fragments import stream_results
            req = P.QueryRequest.from_json(body)
            t0 = time.perf_counter()
            t = self._run_with_session(req.sql, req.session_config)
            for chunk in stream_results(t, (time.perf_counter() - t0) * 1e3):
                yield fl.Result(chunk)
        elif kind == "health":
            yield fl.Result(b"ok")
        elif kind == "CreatePreparedStatement":
            a = P.unpack_any(body)
            if a is None or a[0] != "ActionCreatePreparedStatementRequest":
                raise ValueError("CreatePreparedStatement expects an ActionCreatePreparedStatementRequest")
            sql = a[1].get(1, [b""])[0].decode()
            n = FS.count_params(sql)
            schema = None
            if _is_query(sql):
                try:
                    # the result schema from the plan (placeholders planned as NULL literals)
                    schema = self._schema_of(FS.bind_params(sql, [None] * n) if n else sql)
                except ValueError:
                    if not n:
                        raise            # an invalid query fails at prepare time
                    # (a placeholder NULL cannot be planned there, e.g. LIMIT ?: planned once bound)
            h, _ = self.prepared.create(sql, schema)
            yield fl.Result(FS.encode_prepared_result(h, schema, FS.parameter_schema(n) if n else None))
        elif kind == "ClosePreparedStatement":
            a = P.unpack_any(body)
            if a is None or a[0] != "ActionClosePreparedStatementRequest":
                raise ValueError("ClosePreparedStatement expects an ActionClosePreparedStatementRequest")
            self.prepared.close(a[1].get(1, [b""])[0])
        else:
            raise NotImplementedError(f"unknown action {kind}")

    def do_exchange(self, context, descriptor, reader, writer):
        raise NotImplementedError("DoExchange: intra-node exchanges use RCCL; inter-node shuffle is not enabled")


def _is_query(sql: str) -> bool:
    head = sql.lstrip().split(None, 1)[0].upper() if sql.strip() else ""
    return head in ("SELECT", "WITH", "VALUES", "EXPLAIN", "(")
