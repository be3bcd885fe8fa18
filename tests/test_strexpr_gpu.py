"""String expressions on the GPU (csrc/kernels/strexpr.hip, ops/strings.py):
CAST to / from VARCHAR, CONCAT, general string CASE, string COALESCE,
char_length, and dictionary-column predicates / transforms evaluated over the
dictionary on the device. Each query's GPU result must equal the CPU engine's
(pyarrow compute), the native kernels must have run, and no host step may be
taken (EXPLAIN ANALYZE 'host steps: none')."""
import datetime
from decimal import Decimal

import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    import torch
    import igloo_amd as ig
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 3000
    t = pa.table({
        "k": pa.array(range(n), pa.int64()),
        "i": pa.array([(i * 7919) % 2001 - 1000 if i % 11 else None for i in range(n)], pa.int32()),
        "d": pa.array([Decimal(i * 37 - 50000).scaleb(-2) for i in range(n)], pa.decimal128(15, 2)),
        "dt": pa.array([datetime.date(1992, 1, 1) + datetime.timedelta(days=i) for i in range(n)], pa.date32()),
        "s": pa.array([None if i % 13 == 0 else f"v{i % 97}-ä{i % 5}" for i in range(n)], pa.string()),
        "c": pa.array(["red", "green", "blue", None][i % 4] for i in range(n)),
        "num": pa.array([str((i * 31) % 1000 - 500) for i in range(n)], pa.string()),
        "dec": pa.array([f"{(i * 13) % 9999 - 5000}.{i % 100:02d}" for i in range(n)], pa.string()),
        "day": pa.array([(datetime.date(1990, 1, 1) + datetime.timedelta(days=3 * i)).isoformat() for i in range(n)]),
    })
    g = ig.QueryEngine(device="cuda:0")
    c = ig.QueryEngine(device="cpu")
    g.register_table("t", t)
    c.register_table("t", t)
    return g, c


QUERIES = [
    "SELECT k, CAST(i AS VARCHAR) AS a, CAST(d AS VARCHAR) AS b, CAST(dt AS VARCHAR) AS e, CAST(k > 5 AS VARCHAR) AS f "
    "FROM t ORDER BY k",
    "SELECT k, CAST(num AS BIGINT) AS a, CAST(num AS INT) AS a2, CAST(dec AS DECIMAL(12, 2)) AS b, "
    "CAST(day AS DATE) AS e, CAST(dec AS DOUBLE) AS f FROM t ORDER BY k",
    "SELECT k, s || '#' || c AS a, concat(c, s) AS b, 'x' || num AS e FROM t ORDER BY k",
    "SELECT k, CASE WHEN k % 3 = 0 THEN s WHEN k % 3 = 1 THEN c ELSE 'other' END AS a FROM t ORDER BY k",
    "SELECT k, COALESCE(s, c, 'none') AS a, COALESCE(c, num) AS b FROM t ORDER BY k",
    "SELECT k, char_length(s) AS a, char_length(c) AS b, char_length(num) AS e FROM t ORDER BY k",
    "SELECT k, upper(c) AS a, substring(c from 2 for 2) AS b, lower(upper(c)) AS e FROM t ORDER BY k",
    "SELECT count(*) AS n FROM t WHERE c LIKE '%re%' AND c <> 'green'",
    "SELECT c, count(*) AS n FROM t WHERE c IN ('red', 'blue') GROUP BY c ORDER BY c",
    "SELECT substring(c from 1 for 1) AS p, count(*) AS n FROM t GROUP BY substring(c from 1 for 1) ORDER BY p",
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_string_expressions_match_cpu(engines, qi):
    from igloo_amd.ops._lib import HOST_STEPS
    g, c = engines
    sql = QUERIES[qi]
    h0 = sum(HOST_STEPS.values())
    got = g.query(sql)
    assert sum(HOST_STEPS.values()) == h0, dict(HOST_STEPS)
    want = c.query(sql)
    assert got.to_pylist() == want.to_pylist(), sql


def test_kernels_ran_and_bad_cast_raises(engines):
    from igloo_amd.ops._lib import KERNEL_CALLS
    from igloo_amd.utils.errors import IglooError
    g, _ = engines
    for k in ("fmt", "str_parse", "str_concat", "str_char_length"):
        assert KERNEL_CALLS[k] > 0, (k, dict(KERNEL_CALLS))
    with pytest.raises(IglooError):
        g.query("SELECT CAST(s AS BIGINT) AS x FROM t")
    txt = g.explain("SELECT k, CAST(d AS VARCHAR) || c AS a FROM t", analyze=True)
    assert "host steps: none" in txt, txt


def test_tpch_takes_no_host_steps():
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops._lib import HOST_STEPS
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, 0.01)
    h0 = dict(HOST_STEPS)
    for q in range(1, 23):
        e.query(queries.QUERIES[q])
    for sql in ("SELECT 42 AS answer", "SELECT capitalize(n_name) AS x FROM nation ORDER BY x"):
        e.query(sql)
    assert {k: v - h0.get(k, 0) for k, v in HOST_STEPS.items() if v != h0.get(k, 0)} == {}
