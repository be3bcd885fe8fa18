"""Fused sorted GROUP BY + HAVING (csrc/kernels/agg.hip sorted_having,
exec/aggregate.py HashAggExec._sorted_having) against the CPU engine: sums,
counts, min/max over int, decimal and float columns, every comparison, the
literal on either side, NULL values, and runs longer than the kernel follows
(the overflow flag sends the query to the general path). The streaming
variant (sorted_having_scan_kernel: COUNTs plus one NULL-free int32 SUM, no
run-length limit) runs on the int32 table and is checked kernel-level against
numpy and the general kernel, with runs crossing waves' spans."""
import numpy as np
import pyarrow as pa
import pytest

import igloo_amd as ig
from igloo_amd.ops._lib import KERNEL_CALLS
from igloo_amd.utils.digest import digest

pytestmark = pytest.mark.gpu


def _table(n=300_000, seed=3, long_run=False, q32=False):
    r = np.random.default_rng(seed)
    runs = r.integers(1, 8, n // 4)
    if long_run:
        runs[len(runs) // 2] = 5000          # one run past the kernel's 256-row follow limit
    k = np.repeat(np.arange(len(runs), dtype=np.int32) * 3 + 7, runs)[:n]
    m = k.size
    q = r.integers(1, 51, m).astype(np.int32 if q32 else np.int64)
    price = pa.array([None if i % 97 == 0 else int(x) for i, x in enumerate(r.integers(100, 10**7, m))], pa.int64())
    f = r.normal(0, 10, m)
    return pa.table({"k": pa.array(k), "q": pa.array(q), "p": price, "f": pa.array(f)})


@pytest.fixture(scope="module")
def engines():
    t = _table()
    tl = _table(seed=5, long_run=True)
    ti = _table(seed=9, long_run=True, q32=True)
    gpu, cpu = ig.QueryEngine(device="cuda:0"), ig.QueryEngine(device="cpu")
    for e in (gpu, cpu):
        e.register_table("t", t)
        e.register_table("tl", tl)
        e.register_table("ti", ti)
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
@pytest.mark.parametrize("tab", ["t", "tl", "ti"])
def test_sorted_having_matches_cpu(engines, sql, tab):
    gpu, cpu = engines
    q = sql.format(t=tab) + " order by k"
    before = KERNEL_CALLS["sorted_having"]
    got = gpu.sql(q).table
    want = cpu.sql(q).table
    assert digest(got) == digest(want), q
    if (tab == "t" or (tab == "ti" and "(q)" in sql and "max" not in sql)) and "cast" not in sql:
        assert KERNEL_CALLS["sorted_having"] > before, q


@pytest.mark.parametrize("vdt", ["int32", "int16", "int8"])
@pytest.mark.parametrize("k64", [False, True])
@pytest.mark.parametrize("shape,op,const", [("sum", ">", 700), ("sum", "<", 10), ("count", ">", 28),
                                            ("sum_count", ">", 700), ("count_sum", "<=", 2)])
def test_having_scan_kernel(monkeypatch, vdt, k64, shape, op, const):
    import torch
    from igloo_amd.ops import agg as A
    r = np.random.default_rng(11)
    runs = r.integers(1, 30, 400_000)
    runs[[0, 10, 200_000, 399_999]] = [513, 70_000, 3000, 100_000]   # runs across tiles and spans, at both ends
    k = np.repeat(np.arange(len(runs), dtype=np.int64) * 5 - 1000, runs)
    n = k.size
    q = r.integers(-20, 60, n).astype(np.int32)
    keys = torch.tensor(k if k64 else k.astype(np.int32), device="cuda")
    vals = torch.tensor(q.astype(vdt), device="cuda")
    cnt_spec, sum_spec = ("count", None, None), ("sum_int", vals, None)
    specs, hidx = {"sum": ([sum_spec], 0), "count": ([cnt_spec], 0), "sum_count": ([cnt_spec, sum_spec], 1),
                   "count_sum": ([cnt_spec, sum_spec], 0)}[shape]
    starts = np.flatnonzero(np.r_[True, k[1:] != k[:-1]])
    cnt = np.diff(np.r_[starts, n])
    sums = np.add.reduceat(q.astype(np.int64), starts)
    hv = sums if specs[hidx][0] == "sum_int" else cnt
    sel = {">": hv > const, "<": hv < const, "<=": hv <= const}[op]
    want = (starts[sel], [sums[sel] if s[0] == "sum_int" else cnt[sel] for s in specs])
    before = KERNEL_CALLS["sorted_having"]
    for env in ("1", "0") if vdt == "int32" else ("1",):     # int16 / int8: the streaming kernel only
        if env == "1":
            monkeypatch.delenv("IGLOO_DEBUG", raising=False)
        else:
            monkeypatch.setenv("IGLOO_DEBUG", "having_general")   # the run-folding kernel (C++ reads it per call)
        got = A.sorted_having(keys, specs, hidx, op, const)
        if got is None:
            assert env == "0"           # the general kernel gives up on the long runs
            continue
        rep, outs = got
        assert np.array_equal(rep.cpu().numpy(), want[0]), (env, shape, op)
        for o, w in zip(outs, want[1]):
            assert np.array_equal(o.cpu().numpy(), w), (env, shape, op)
    assert KERNEL_CALLS["sorted_having"] > before
