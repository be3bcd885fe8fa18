"""Flight client (reference crates/client is a println! placeholder).

``IglooClient(uri).query(sql)`` plans with GetFlightInfo and streams the
result with DoGet; ``flight_sql=True`` speaks Flight SQL
(CommandStatementQuery); ``execute_raw`` sends the SQL as the ticket like the
reference's do_get. Control-plane helpers wrap the DoAction messages.

CLI: ``python -m igloo_amd.service.client --sql "..." [--uri grpc://host:50051]``.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import List, Optional

import pyarrow as pa
import pyarrow.flight as fl

from . import protocol as P


class _Bearer(fl.ClientMiddleware):
    def __init__(self, token):
        self.token = token

    def sending_headers(self):
        return {"authorization": f"Bearer {self.token}"}


class _BearerFactory(fl.ClientMiddlewareFactory):
    def __init__(self, token):
        self.token = token

    def start_call(self, info):
        return _Bearer(self.token)


class IglooClient:
    def __init__(self, uri: str = "grpc://127.0.0.1:50051", token: Optional[str] = None, timeout: Optional[float] = None):
        mw = [_BearerFactory(token)] if token else None
        self.uri = uri
        self.client = fl.connect(uri, middleware=mw)
        self.options = fl.FlightCallOptions(timeout=timeout) if timeout else fl.FlightCallOptions()

    def close(self):
        self.client.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------- queries
    def query(self, sql: str, flight_sql: bool = False) -> pa.Table:
        cmd = P.command_statement_query(sql) if flight_sql else sql.encode()
        info = self.client.get_flight_info(fl.FlightDescriptor.for_command(cmd), self.options)
        tables = [self.client.do_get(ep.ticket, self.options).read_all() for ep in info.endpoints]
        if not tables:
            return info.schema.empty_table()
        return pa.concat_tables(tables) if len(tables) > 1 else tables[0]

    def schema(self, sql: str) -> pa.Schema:
        return self.client.get_flight_info(fl.FlightDescriptor.for_command(sql.encode()), self.options).schema

    def execute_raw(self, sql: str) -> pa.Table:
        return self.client.do_get(fl.Ticket(sql.encode()), self.options).read_all()

    def upload(self, name: str, table: pa.Table):
        w, _ = self.client.do_put(fl.FlightDescriptor.for_path(name), table.schema, self.options)
        w.write_table(table)
        w.close()

    def tables(self) -> List[str]:
        return [f.descriptor.path[0].decode() for f in self.client.list_flights(options=self.options)]

    # ------------------------------------------------------------ Flight SQL
    def _fsql(self, cmd: bytes) -> pa.Table:
        info = self.client.get_flight_info(fl.FlightDescriptor.for_command(cmd), self.options)
        tables = [self.client.do_get(ep.ticket, self.options).read_all() for ep in info.endpoints]
        return pa.concat_tables(tables) if len(tables) > 1 else (tables[0] if tables else info.schema.empty_table())

    def sql_info(self, ids=()) -> dict:
        """CommandGetSqlInfo: {info id: value}."""
        body = b"".join(P.pb_field(1, int(i)) for i in ids)
        t = self._fsql(P.pack_any("CommandGetSqlInfo", body))
        return {r["info_name"]: r["value"] for r in t.to_pylist()}

    def get_tables(self, table_pattern: Optional[str] = None, table_types=(), include_schema: bool = False
                   ) -> pa.Table:
        """CommandGetTables (LIKE pattern on the table name)."""
        body = (P.pb_field(3, table_pattern) if table_pattern is not None else b"") + \
            b"".join(P.pb_field(4, t) for t in table_types) + (P.pb_field(5, 1) if include_schema else b"")
        return self._fsql(P.pack_any("CommandGetTables", body))

    def get_catalogs(self) -> pa.Table:
        return self._fsql(P.pack_any("CommandGetCatalogs", b""))

    def get_db_schemas(self) -> pa.Table:
        return self._fsql(P.pack_any("CommandGetDbSchemas", b""))

    def prepare(self, sql: str) -> "PreparedStatement":
        """ActionCreatePreparedStatement: a server-side prepared statement."""
        res = self.action("CreatePreparedStatement", P.pack_any("ActionCreatePreparedStatementRequest",
                                                                 P.pb_field(1, sql)))
        body = P.pb_decode(P.pb_decode(res)[2][0])
        schema = pa.ipc.read_schema(pa.py_buffer(body[2][0])) if body.get(2) and body[2][0] else None
        return PreparedStatement(self, body[1][0], schema)

    # --------------------------------------------------------- control plane
    def action(self, kind: str, body: bytes = b"") -> bytes:
        res = list(self.client.do_action(fl.Action(kind, body), self.options))
        return res[0].body.to_pybytes() if res else b""

    def action_stream(self, kind: str, body: bytes = b""):
        """Every result body of a streaming action, in order."""
        for r in self.client.do_action(fl.Action(kind, body), self.options):
            yield r.body.to_pybytes()

    def execute_query(self, sql: str, session_config=None):
        """ExecuteQuery: (Arrow table, QueryComplete fields) with the given
        session settings applied on the server for this query only."""
        from ..parallel.fragments import collect_stream
        req = P.QueryRequest(sql=sql, session_config=dict(session_config or {}))
        return collect_stream(self.action_stream("execute_query", req.to_json()))

    def register_worker(self, info: P.WorkerInfo) -> P.RegistrationAck:
        return P.RegistrationAck.from_json(self.action("register_worker", info.to_json()))

    def heartbeat(self, hb: P.HeartbeatInfo) -> P.HeartbeatResponse:
        return P.HeartbeatResponse.from_json(self.action("heartbeat", hb.to_json()))

    def execute_task(self, td: P.TaskDefinition) -> P.TaskStatus:
        return P.TaskStatus.from_json(self.action("execute_task", td.to_json()))

    def get_data_for_task(self, task_id: str) -> pa.Table:
        b = self.action("get_data_for_task", P.DataForTaskRequest(task_id).to_json())
        return pa.ipc.open_stream(b).read_all()

    def list_workers(self) -> list:
        return json.loads(self.action("list_workers"))

    def metrics(self) -> dict:
        return json.loads(self.action("metrics"))

    def explain(self, sql: str) -> str:
        return self.action("explain", sql.encode()).decode()


class PreparedStatement:
    """A Flight SQL prepared statement; ``execute(params)`` binds the ``?``
    placeholders (DoPut) and runs it (GetFlightInfo + DoGet)."""

    def __init__(self, client: IglooClient, handle: bytes, schema: Optional[pa.Schema]):
        self.client, self.handle, self.schema = client, bytes(handle), schema

    def _cmd(self) -> bytes:
        return P.pack_any("CommandPreparedStatementQuery", P.pb_field(1, self.handle))

    def execute(self, params=None) -> pa.Table:
        if params is not None:
            t = params if isinstance(params, pa.Table) else \
                pa.table({f"p{i + 1}": [v] for i, v in enumerate(params)})
            w, r = self.client.client.do_put(fl.FlightDescriptor.for_command(self._cmd()), t.schema,
                                             self.client.options)
            w.write_table(t)
            w.done_writing()
            r.read()
            w.close()
        return self.client._fsql(self._cmd())

    def close(self) -> None:
        self.client.action("ClosePreparedStatement", P.pack_any("ActionClosePreparedStatementRequest",
                                                                P.pb_field(1, self.handle)))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="igloo-client")
    ap.add_argument("--uri", default="grpc://127.0.0.1:50051")
    ap.add_argument("--sql", "-s", required=False)
    ap.add_argument("--flight-sql", action="store_true")
    ap.add_argument("--token", default=None)
    a = ap.parse_args(argv)
    print("igloo-client starting up...")
    if not a.sql:
        return 0
    from ..engine import print_batches
    with IglooClient(a.uri, a.token) as c:
        print_batches(c.query(a.sql, flight_sql=a.flight_sql))
    return 0


if __name__ == "__main__":
    sys.exit(main())
