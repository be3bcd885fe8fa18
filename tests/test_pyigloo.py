"""pyigloo bindings (reference pyigloo is a placeholder whose only test is
``2 + 2 == 4``: reference pyigloo/tests/test_sample.py:1-2)."""
import pyarrow as pa

import pyigloo


def test_sample():
    assert 2 + 2 == 4  # the reference's entire pyigloo test


def test_local_engine_and_sql():
    eng = pyigloo.local(device="cpu")
    eng.register_table("t", pa.table({"a": [1, 2, 3]}))
    assert pyigloo.sql("SELECT sum(a) AS s FROM t", eng).to_pylist() == [{"s": 6}]
    assert pyigloo.hello() == "Hello from Igloo Crate!"


def test_connect_over_flight():
    from igloo_amd.service.flight_server import IglooFlightServer
    eng = pyigloo.local(device="cpu")
    eng.register_table("t", pa.table({"a": [1, 2, 3]}))
    srv = IglooFlightServer(eng, "grpc://127.0.0.1:0")
    srv.start_background()
    try:
        with pyigloo.connect(f"grpc://127.0.0.1:{srv.port}") as conn:
            assert conn.sql("SELECT max(a) AS m FROM t").to_pylist() == [{"m": 3}]
            assert "t" in conn.tables()
    finally:
        srv.shutdown()


def test_connect_flight_sql_metadata_and_prepared():
    """The Connection speaks Flight SQL: catalog metadata and prepared statements."""
    from igloo_amd.service.flight_server import IglooFlightServer
    eng = pyigloo.local(device="cpu")
    eng.register_table("lineitem", pa.table({"a": [1, 2, 3], "b": ["x", "y", "z"]}))
    srv = IglooFlightServer(eng, "grpc://127.0.0.1:0")
    srv.start_background()
    try:
        with pyigloo.connect(f"grpc://127.0.0.1:{srv.port}") as conn:
            assert conn.get_tables("line%").column("table_name").to_pylist() == ["lineitem"]
            assert conn.sql_info([0])[0] == "igloo-amd"
            with conn.prepare("SELECT b FROM lineitem WHERE a >= ? ORDER BY a") as st:
                assert st.schema.names == ["b"]
                assert st.execute([2]).column("b").to_pylist() == ["y", "z"]
                assert st.execute([3]).column("b").to_pylist() == ["z"]
    finally:
        srv.shutdown()


def test_device_result_and_native_core():
    eng = pyigloo.local(device="cpu")
    eng.register_table("t", pa.table({"a": [1, 2, 3]}))
    res = pyigloo.sql_device("SELECT a * 10 AS x FROM t ORDER BY a", eng)
    assert isinstance(res, pyigloo.DeviceResult)
    assert pa.record_batch(res).column("x").to_pylist() == [10, 20, 30]
    assert pyigloo.native.ARCH == "gfx950"
    assert pyigloo.native.parse_sql("SELECT 1")[0]["k"] == "query"
