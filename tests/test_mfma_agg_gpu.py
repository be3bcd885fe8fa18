"""One-hot MFMA aggregation (csrc/kernels/fused.hip ff_mfma_agg_kernel:
v_mfma_i32_16x16x64_i8 over one-hot group ids x 7-bit value limbs) against
the LDS-atomic fused kernel and the CPU engine: exact decimal sums, counts,
negative values (signed top limb), filters, 1..16 groups."""
import pytest

pytestmark = pytest.mark.gpu

QUERIES = [
    # TPC-H Q1 shape: 4 groups, chained decimal products, counts, averages
    """SELECT l_returnflag, l_linestatus, sum(l_quantity) AS sq, sum(l_extendedprice) AS sp,
              sum(l_extendedprice * (1 - l_discount)) AS sd, sum(l_extendedprice * (1 - l_discount) * (1 + l_tax)) AS sc,
              avg(l_quantity) AS aq, avg(l_discount) AS ad, count(*) AS n
       FROM lineitem WHERE l_shipdate <= date '1998-09-02' GROUP BY l_returnflag, l_linestatus
       ORDER BY l_returnflag, l_linestatus""",
    # Q6 shape: no GROUP BY
    """SELECT sum(l_extendedprice * l_discount) AS revenue FROM lineitem
       WHERE l_shipdate >= date '1994-01-01' AND l_shipdate < date '1995-01-01'
         AND l_discount BETWEEN 0.05 AND 0.07 AND l_quantity < 24""",
    # negative values + 15 groups (shipmode x linestatus <= 14)
    """SELECT l_shipmode, l_linestatus, sum(l_discount - 0.06) AS s, sum(l_quantity * (l_tax - 0.05)) AS t,
              count(*) AS n
       FROM lineitem GROUP BY l_shipmode, l_linestatus ORDER BY l_shipmode, l_linestatus""",
]


@pytest.fixture(scope="module")
def engines():
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = ig.QueryEngine(device="cuda:0")
    datagen.register(g, 1.0)
    c = ig.QueryEngine(device="cpu")
    datagen.register(c, 1.0)
    return g, c


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_mfma_aggregation_matches(engines, qi, monkeypatch):
    from igloo_amd.exec import fused_jit
    from igloo_amd.ops import _lib
    monkeypatch.setattr(fused_jit, "ENABLED", False)   # the interpreted kernels under test
    g, c = engines
    sql = QUERIES[qi]
    N = _lib.native()
    prev = N.ff_set_mfma(True)
    try:
        _lib.KERNEL_CALLS.clear()
        got = g.sql(sql).table.to_pylist()
        assert _lib.KERNEL_CALLS["ff_aggregate"] > 0, dict(_lib.KERNEL_CALLS)
        N.ff_set_mfma(False)
        lds = g.sql(sql).table.to_pylist()
    finally:
        N.ff_set_mfma(prev)
    want = c.sql(sql).table.to_pylist()
    assert got == lds
    assert got == want
