"""NOT IN (null-aware anti join) against sqlite, on the CPU engine and (gpu
marker) on the device: a NULL in the subquery empties the result, a NULL
probe value is never returned unless the subquery is empty, and columns
declared nullable that hold no NULL take the plain anti-join paths."""
import sqlite3

import pyarrow as pa
import pytest

import igloo_amd as ig

ROWS_T = [1, 2, 3, None, 5, 6, 7, 8]
CASES = {
    "no_nulls": ([2, 3, 9], [1, 2, 3, 4, 5, 6, 7, 8]),
    "build_null": ([2, None, 9], [1, 2, 3, 5]),
    "probe_null": ([2, 3, 9], ROWS_T),
    "empty_build": ([], ROWS_T),
}
QUERIES = [
    "SELECT x FROM t WHERE x NOT IN (SELECT y FROM s)",
    "SELECT x FROM t WHERE x NOT IN (SELECT y FROM s WHERE y > 2)",
    "SELECT count(*) AS n FROM t WHERE x NOT IN (SELECT y FROM s)",
]


def _sqlite(tv, sv, q):
    con = sqlite3.connect(":memory:")
    con.execute("CREATE TABLE t (x INTEGER)")
    con.execute("CREATE TABLE s (y INTEGER)")
    con.executemany("INSERT INTO t VALUES (?)", [(v,) for v in tv])
    con.executemany("INSERT INTO s VALUES (?)", [(v,) for v in sv])
    return sorted(con.execute(q).fetchall(), key=repr)


def _run(dev, tv, sv, q):
    e = ig.QueryEngine(device=dev)
    e.register_table("t", pa.table({"x": pa.array(tv, pa.int64())}))
    e.register_table("s", pa.table({"y": pa.array(sv, pa.int64())}))
    return sorted((tuple(r.values()) for r in e.query(q).to_pylist()), key=repr)


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_not_in_cpu(case, qi):
    sv, tv = CASES[case]
    assert _run("cpu", tv, sv, QUERIES[qi]) == _sqlite(tv, sv, QUERIES[qi])


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_not_in_gpu(gpu_device, case, qi):
    sv, tv = CASES[case]
    assert _run(gpu_device, tv, sv, QUERIES[qi]) == _sqlite(tv, sv, QUERIES[qi])
