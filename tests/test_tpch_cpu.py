"""All 22 TPC-H queries on the CPU path vs the sqlite oracle (SF 0.01)."""
import pytest

from igloo_amd.models.tpch import oracle, queries


@pytest.mark.parametrize("q", list(range(1, 23)))
def test_tpch_query_matches_sqlite(tpch_cpu, q):
    e, _, con = tpch_cpu
    got = [tuple(r.values()) for r in e.sql(queries.QUERIES[q]).table.to_pylist()]
    exp = oracle.run_sqlite(con, q)
    diff = oracle.rows_match(got, exp)
    assert not diff, f"Q{q}: {diff}"


def test_fused_spec_or_groups():
    """fused.Spec turns an OR of conjunctions into OR-group terms (kind >> 8),
    merging BETWEEN bounds per group and dropping never-true disjuncts."""
    import pyarrow as pa
    import torch
    from igloo_amd.columnar import Batch, Column
    from igloo_amd.exec import fused
    from igloo_amd.sql.expr import BinOp, ColRef, Lit
    from igloo_amd import types as T
    a, b = ColRef(1, "a", T.INT64), ColRef(2, "b", T.INT64)
    batch = Batch({1: Column(T.INT64, torch.arange(10)), 2: Column(T.INT64, torch.arange(10) % 3)}, 10)

    def rng(c, lo, hi):
        return BinOp("and", BinOp(">=", c, Lit(lo, T.INT64), T.BOOL), BinOp("<=", c, Lit(hi, T.INT64), T.BOOL), T.BOOL)

    pred = BinOp("or", BinOp("and", rng(a, 1, 3), BinOp("=", b, Lit(1, T.INT64), T.BOOL), T.BOOL),
                 BinOp("or", rng(a, 7, 8), rng(a, 5, 4), T.BOOL), T.BOOL)
    spec = fused.Spec(batch, None)
    spec.add_predicate(pred)
    assert not spec.always_false and spec.mask is None
    groups = sorted({k >> 8 for _, k, *_ in spec.terms})
    assert groups == [1, 2]     # the empty range 5..4 is dropped
    assert (0, 1 << 8, 1, 3, 0) in spec.terms and (0, 2 << 8, 7, 8, 0) in spec.terms
