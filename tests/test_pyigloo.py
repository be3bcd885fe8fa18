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
