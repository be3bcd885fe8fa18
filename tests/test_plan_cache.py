"""Plan cache (engine.QueryEngine.sql): repeated SQL reuses the optimized
logical plan but always re-executes against current table contents; DDL
(register / deregister / views) and session changes invalidate."""
import pyarrow as pa

import igloo_amd as ig


def test_plan_cache_hits_and_invalidation():
    e = ig.QueryEngine(device="cpu")
    e.register_table("t", pa.table({"a": [1, 2, 3]}))
    sql = "SELECT sum(a) AS s FROM t WHERE a > (SELECT min(a) FROM t)"
    assert e.sql(sql).to_pylist() == [{"s": 5}]
    assert e.last_metrics["plan_cached"] is False
    assert e.sql(sql).to_pylist() == [{"s": 5}]
    assert e.last_metrics["plan_cached"] is True
    # new data under the same name: re-planned, recomputed (incl. the scalar subquery)
    e.register_table("t", pa.table({"a": [10, 20, 30, 40]}))
    assert e.sql(sql).to_pylist() == [{"s": 90}]
    assert e.last_metrics["plan_cached"] is False
    # schema change: the cached plan's columns no longer exist
    e.register_table("t", pa.table({"b": [1], "a": [7]}))
    assert e.sql("SELECT a FROM t").to_pylist() == [{"a": 7}]


def test_session_setting_invalidates():
    e = ig.QueryEngine(device="cpu")
    e.register_table("t", pa.table({"a": [1, 2]}))
    e.sql("SELECT a FROM t")
    e.sql("SELECT a FROM t")
    assert e.last_metrics["plan_cached"] is True
    e.session["some_setting"] = 1
    e.sql("SELECT a FROM t")
    assert e.last_metrics["plan_cached"] is False
