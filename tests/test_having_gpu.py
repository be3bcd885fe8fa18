"""Fused sorted GROUP BY + HAVING (csrc/kernels/agg.hip sorted_having,
exec/operators.py HashAggExec._sorted_having) against the CPU engine: sums,
counts, min/max over int, decimal and float columns, every comparison, the
literal on either side, NULL values, and runs longer than the kernel follows
(the overflow flag sends the query to the general path)."""
import numpy as np
import pyarrow as pa
import pytest

import igloo_amd as ig
from igloo_amd.ops._lib import KERNEL_CALLS
from igloo_amd.utils.digest import digest

pytestmark = pytest.mark.gpu


def _table(n=300_000, seed=3, long_run=False):
    r = np.random.default_rng(seed)
    runs = r.integers(1, 8, n // 4)
    if long_run:
        runs[len(runs) // 2] = 5000          # one run past the kernel's 256-row follow limit
    k = np.repeat(np.arange(len(runs), dtype=np.int32) * 3 + 7, runs)[:n]
    m = k.size
    q = r.integers(1, 51, m).astype(np.int64)
    price = pa.array([None if i % 97 == 0 else int(x) for i, x in enumerate(r.integers(100, 10**7, m))], pa.int64())
    f = r.normal(0, 10, m)
    return pa.table({"k": pa.array(k), "q": pa.array(q), "p": price, "f": pa.array(f)})


@pytest.fixture(scope="module")
def engines():
    t = _table()
    tl = _table(seed=5, long_run=True)
    gpu, cpu = ig.QueryEngine(device="cuda:0"), ig.QueryEngine(device="cpu")
    for e in (gpu, cpu):
        e.register_table("t", t)
        e.register_table("tl", tl)
    return gpu, cpu


QUERIES = [
    "select k, sum(q) from {t} group by k having sum(q) > 250",
    "select k, sum(q) as s, count(*) as c from {t} group by k having 250 < sum(q)",
    "select k, count(*) from {t} group by k having count(*) >= 6",
    "select k, min(q), max(q) from {t} group by k having max(q) <= 3",
    "select k, sum(p) from {t} group by k having sum(p) > 30000000",
    "select k, sum(f) from {t} group by k having sum(f) < -25.5",
    "select k, sum(q) from {t} group by k having sum(q) = 100",
    "select k, sum(q) from {t} group by k having sum(q) <> 4",
    "select k, sum(cast(q as decimal(15,2))) from {t} group by k having sum(cast(q as decimal(15,2))) > 250.5",
]


@pytest.mark.parametrize("sql", QUERIES)
@pytest.mark.parametrize("tab", ["t", "tl"])
def test_sorted_having_matches_cpu(engines, sql, tab):
    gpu, cpu = engines
    q = sql.format(t=tab) + " order by k"
    before = KERNEL_CALLS["sorted_having"]
    got = gpu.sql(q).table
    want = cpu.sql(q).table
    assert digest(got) == digest(want), q
    if tab == "t" and "cast" not in sql:
        assert KERNEL_CALLS["sorted_having"] > before, q
