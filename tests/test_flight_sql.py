"""Flight SQL endpoint as a JDBC / ODBC-class client drives it: GetSqlInfo,
catalog browsing, prepared statements with bound parameters, updates.

No Flight SQL client library is importable here, so the requests are
protobuf ``Any`` messages encoded by hand in this file (field numbers from
arrow/flight/sql/FlightSql.proto) and sent through plain ``pyarrow.flight``;
results are compared with the engine's own answers.
"""
import pyarrow as pa
import pyarrow.flight as fl
import pytest

import igloo_amd as ig
from igloo_amd.service.flight_server import IglooFlightServer

PREFIX = "type.googleapis.com/arrow.flight.protocol.sql."


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _field(no: int, v) -> bytes:
    if isinstance(v, bool) or isinstance(v, int):
        return _varint(no << 3) + _varint(int(v))
    v = v.encode() if isinstance(v, str) else v
    return _varint((no << 3) | 2) + _varint(len(v)) + v


def _any(name: str, body: bytes = b"") -> bytes:
    return _field(1, PREFIX + name) + _field(2, body)


def _decode(b: bytes) -> dict:
    out, p = {}, 0
    while p < len(b):
        key, p = _read_varint(b, p)
        no, wt = key >> 3, key & 7
        if wt == 0:
            v, p = _read_varint(b, p)
        else:
            n, p = _read_varint(b, p)
            v, p = b[p:p + n], p + n
        out.setdefault(no, []).append(v)
    return out


def _read_varint(b, p):
    acc = shift = 0
    while True:
        c = b[p]
        p += 1
        acc |= (c & 0x7F) << shift
        if not c & 0x80:
            return acc, p
        shift += 7


@pytest.fixture(scope="module")
def flight():
    e = ig.QueryEngine(device="cpu")
    e.register_table("orders", pa.table({"o_id": pa.array([1, 2, 3, 4], pa.int64()),
                                         "o_cust": pa.array([10, 20, 10, 30], pa.int32()),
                                         "o_note": ["a", "b", "c", None]}))
    e.register_table("customer", pa.table({"c_id": pa.array([10, 20, 30], pa.int32()), "c_name": ["x", "y", "z"]}))
    s = IglooFlightServer(e, "grpc://127.0.0.1:0")
    s.start_background()
    c = fl.connect(f"grpc://127.0.0.1:{s.port}")
    yield e, s, c
    c.close()
    s.shutdown()


def _fetch(c, cmd: bytes) -> pa.Table:
    info = c.get_flight_info(fl.FlightDescriptor.for_command(cmd))
    t = c.do_get(info.endpoints[0].ticket).read_all()
    assert t.schema.equals(info.schema), (t.schema, info.schema)
    return t


def test_jdbc_style_handshake(flight):
    e, s, c = flight
    # 1. GetSqlInfo (connection setup): server name / version / read-only / quote char
    info = _fetch(c, _any("CommandGetSqlInfo", _field(1, 0) + _field(1, 1) + _field(1, 3) + _field(1, 504)))
    got = {r["info_name"]: r["value"] for r in info.to_pylist()}
    assert got[0] == "igloo-amd" and got[1] == ig.__version__ and got[3] is False and got[504] == '"'
    assert info.schema.field("value").type.mode == "dense"
    assert _fetch(c, _any("CommandGetSqlInfo")).num_rows >= 15        # no ids: every known one
    # 2. catalogs, schemas, table types
    assert _fetch(c, _any("CommandGetCatalogs")).column("catalog_name").to_pylist() == ["igloo"]
    sch = _fetch(c, _any("CommandGetDbSchemas", _field(1, "igloo")))
    assert sch.to_pylist() == [{"catalog_name": "igloo", "db_schema_name": "public"}]
    assert _fetch(c, _any("CommandGetDbSchemas", _field(2, "nope%"))).num_rows == 0
    assert "TABLE" in _fetch(c, _any("CommandGetTableTypes")).column("table_type").to_pylist()
    # 3. GetTables: name pattern, type filter, with schemas
    t = _fetch(c, _any("CommandGetTables", _field(3, "ord%") + _field(4, "TABLE") + _field(5, True)))
    assert t.column("table_name").to_pylist() == ["orders"]
    schema = pa.ipc.read_schema(pa.py_buffer(t.column("table_schema")[0].as_py()))
    assert schema.names == ["o_id", "o_cust", "o_note"] and schema.field("o_cust").type == pa.int32()
    assert sorted(_fetch(c, _any("CommandGetTables")).column("table_name").to_pylist()) == ["customer", "orders"]
    assert "table_schema" not in _fetch(c, _any("CommandGetTables")).column_names
    assert _fetch(c, _any("CommandGetTables", _field(4, "VIEW"))).num_rows == 0
    assert _fetch(c, _any("CommandGetPrimaryKeys", _field(3, "orders"))).num_rows == 0
    # GetSchema answers from the fixed schemas, without a run
    assert c.get_schema(fl.FlightDescriptor.for_command(_any("CommandGetCatalogs"))).schema.names == ["catalog_name"]
    # 4. a prepared query: create, describe, execute, close
    sql = "SELECT c_name, count(*) AS n FROM orders JOIN customer ON o_cust = c_id GROUP BY c_name ORDER BY c_name"
    res = list(c.do_action(fl.Action("CreatePreparedStatement",
                                     _any("ActionCreatePreparedStatementRequest", _field(1, sql)))))
    outer = _decode(res[0].body.to_pybytes())
    assert outer[1][0].decode().endswith("ActionCreatePreparedStatementResult")
    body = _decode(outer[2][0])
    handle = body[1][0]
    ds = pa.ipc.read_schema(pa.py_buffer(body[2][0]))
    assert ds.names == ["c_name", "n"]
    before = s.metrics["queries"]
    got = _fetch(c, _any("CommandPreparedStatementQuery", _field(1, handle)))
    assert s.metrics["queries"] == before + 1          # planning the FlightInfo ran nothing
    assert got.to_pylist() == e.query(sql).to_pylist() == [{"c_name": "x", "n": 2}, {"c_name": "y", "n": 1},
                                                           {"c_name": "z", "n": 1}]
    list(c.do_action(fl.Action("ClosePreparedStatement",
                               _any("ActionClosePreparedStatementRequest", _field(1, handle)))))
    with pytest.raises(KeyError):          # gRPC NOT_FOUND (pyarrow's ArrowKeyError)
        _fetch(c, _any("CommandPreparedStatementQuery", _field(1, handle)))


def test_prepared_parameters_and_updates(flight):
    e, s, c = flight
    sql = "SELECT o_id FROM orders WHERE o_cust = ? AND o_note <> ? ORDER BY o_id"
    res = list(c.do_action(fl.Action("CreatePreparedStatement",
                                     _any("ActionCreatePreparedStatementRequest", _field(1, sql)))))
    body = _decode(_decode(res[0].body.to_pybytes())[2][0])
    handle = body[1][0]
    assert len(pa.ipc.read_schema(pa.py_buffer(body[3][0]))) == 2      # parameter schema: two placeholders
    cmd = _any("CommandPreparedStatementQuery", _field(1, handle))
    # bind (10, 'c') with DoPut, then execute
    params = pa.table({"p1": pa.array([10], pa.int32()), "p2": ["c"]})
    w, r = c.do_put(fl.FlightDescriptor.for_command(cmd), params.schema)
    w.write_table(params)
    w.done_writing()
    ack = r.read()
    w.close()
    assert ack is not None and _decode(ack.to_pybytes())[1][0] == handle
    assert _fetch(c, cmd).column("o_id").to_pylist() == [1]
    # re-bind: another customer
    params = pa.table({"p1": pa.array([20], pa.int32()), "p2": ["zz"]})
    w, r = c.do_put(fl.FlightDescriptor.for_command(cmd), params.schema)
    w.write_table(params)
    w.done_writing()
    r.read()
    w.close()
    assert _fetch(c, cmd).column("o_id").to_pylist() == [2]
    # CommandStatementUpdate: DDL through DoPut, record count in the app metadata
    upd = _any("CommandStatementUpdate", _field(1, "CREATE TABLE big AS SELECT * FROM orders WHERE o_id > 1"))
    w, r = c.do_put(fl.FlightDescriptor.for_command(upd), pa.schema([]))
    w.done_writing()
    meta = r.read()
    w.close()
    assert _decode(meta.to_pybytes())[1][0] == 3
    assert "big" in e.catalog.table_names()
    t = _fetch(c, _any("CommandGetTables", _field(3, "big")))
    assert t.column("table_name").to_pylist() == ["big"]
