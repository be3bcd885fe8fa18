"""Per-query metrics: cache hit ratio on every engine, and on
the GPU the query's HBM high-water mark and device-side span from one event pair."""
import pytest

import igloo_amd as ig
from igloo_amd.models.tpch import datagen, queries


def test_cache_metrics_cpu(tmp_path):
    import pyarrow as pa
    import pyarrow.parquet as pq
    pq.write_table(pa.table({"k": list(range(100)), "v": [i * 2 for i in range(100)]}), tmp_path / "t.parquet")
    e = ig.QueryEngine(device="cpu")
    e.register_parquet("t", str(tmp_path / "t.parquet"))
    e.sql("select sum(v) from t")
    m1 = e.last_metrics["cache"]
    e.sql("select sum(v) from t where k > 5")
    m2 = e.last_metrics["cache"]
    assert m1["misses"] >= 1
    assert m2["hits"] >= 1 and m2["hit_ratio"] is not None and 0 < m2["hit_ratio"] <= 1
    assert "device_span_ms" not in e.last_metrics


@pytest.mark.gpu
def test_device_metrics_gpu(gpu_device):
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, 0.01)
    e.sql(queries.QUERIES[3])
    m = e.last_metrics
    assert m["device_span_ms"] > 0 and m["hbm_peak_bytes"] > 0 and m["hbm_query_bytes"] >= 0
    assert e.hbm_peak_bytes >= m["hbm_peak_bytes"]
    assert m["device_span_ms"] <= m["elapsed_ms"] * 1.5 + 1.0


def test_having_constant_units():
    """exec/aggregate.py having_constant: the HAVING literal in the raw units
    of the aggregate state, fractional thresholds rounded per comparison."""
    from igloo_amd import types as T
    from igloo_amd.exec.aggregate import having_constant
    from igloo_amd.sql.expr import Lit
    dec2 = T.DataType("decimal", 15, 2)
    lit = Lit(30000, T.DataType("decimal", 5, 2))          # 300.00
    assert having_constant(">", lit, dec2, "sum", False) == 30000
    half = Lit(25, T.DataType("decimal", 2, 1))            # 2.5
    assert having_constant(">", half, T.INT64, "count", False) == 2
    assert having_constant(">=", half, T.INT64, "count", False) == 3
    assert having_constant("<", half, T.INT64, "count", False) == 3
    assert having_constant("<=", half, T.INT64, "count", False) == 2
    assert having_constant("=", half, T.INT64, "count", False) is None
    assert having_constant(">", Lit(3, T.INT64), dec2, "sum", False) == 300
    assert having_constant("<", Lit(-25.5, T.FLOAT64), T.FLOAT64, "sum", True) == -25.5
