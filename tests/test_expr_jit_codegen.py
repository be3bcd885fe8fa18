"""Generated expression kernels (exec/expr_jit.py): every composite
expression the TPC-H suite evaluates (projections, residual predicates, CASE,
date parts, IN lists, decimal arithmetic) generates a source that hiprtc
compiles for gfx950 on the host."""
import pytest

from igloo_amd.ops import _lib

pytestmark = pytest.mark.skipif(not _lib.have_native(), reason="native extension not built")


def test_tpch_expression_sources_compile(tpch_cpu, monkeypatch):
    from igloo_amd.exec import expr_eval, expr_jit
    from igloo_amd.models.tpch import queries
    e, _, _ = tpch_cpu
    sink = []
    monkeypatch.setattr(expr_jit, "_SOURCE_SINK", sink)
    monkeypatch.setattr(expr_eval, "_JIT_ON_CPU", True)
    monkeypatch.setattr(expr_jit.jit, "MODE", "sync")
    for q in range(1, 23):
        e.sql(queries.QUERIES[q])
    srcs = sorted(set(sink))
    assert len(srcs) >= 15, len(srcs)
    N = _lib.native()
    for s in srcs:
        assert len(N.jit_compile(s, "igloo_jit_expr", "gfx950")) > 1000


def test_expression_bounds():
    """Interval bounds of generated-kernel outputs (expr_jit._bound): decimal
    scaling through + - *, CASE arms, and None where a node could wrap or a
    column has no readback-free bound."""
    import torch
    from igloo_amd import types as T
    from igloo_amd.columnar import Batch, Column
    from igloo_amd.exec import expr_jit as J
    from igloo_amd.sql.expr import BinOp, Case, ColRef, Lit

    D = T.DECIMAL(15, 2)
    price = torch.tensor([90000, 10494950], dtype=torch.int64)
    price._igloo_bound = (90000, 10494950)
    disc = torch.tensor([0, 10], dtype=torch.int64)
    disc._igloo_bound = (0, 10)
    free = torch.tensor([5, 7], dtype=torch.int64)          # no bound known
    b = Batch({1: Column(D, price, None), 2: Column(D, disc, None), 3: Column(T.INT64, free, None)}, 2)
    rev = BinOp("*", ColRef(1, "p", D), BinOp("-", Lit(100, D), ColRef(2, "d", D), D), T.DECIMAL(31, 4))
    lo, hi = J._raw_bound(rev, b, rev.dtype)
    assert lo <= 90000 * 90 and hi >= 10494950 * 100 and hi < 10494950 * 100 + 100
    case = Case([(Lit(True, T.BOOL), rev)], Lit(0, T.DECIMAL(31, 4)), T.DECIMAL(31, 4))
    assert J._raw_bound(case, b, case.dtype)[0] <= 0
    assert J._bound(BinOp("+", ColRef(3, "f", T.INT64), Lit(1, T.INT64), T.INT64), b) is None
    big = BinOp("*", ColRef(1, "p", T.INT32), ColRef(1, "p", T.INT32), T.INT32)
    b32 = Batch({1: Column(T.INT32, price.to(torch.int32), None)}, 2)
    b32.columns[1].data._igloo_bound = (90000, 10494950)
    assert J._bound(big, b32) is None                       # would wrap in 32 bits


def test_date_part_bounds():
    """date_part bounds: fixed ranges for month / quarter / ..., the year
    range of a date column with a readback-free bound."""
    import torch
    from igloo_amd import types as T
    from igloo_amd.columnar import Batch, Column
    from igloo_amd.exec import expr_jit as J
    from igloo_amd.sql.expr import ColRef, Func

    DATE = T.DataType("date32")
    days = torch.tensor([8035, 10591], dtype=torch.int32)     # 1992-01-01 .. 1998-12-31
    days._igloo_bound = (8035, 10591)
    b = Batch({1: Column(DATE, days, None)}, 2)
    year = Func("date_part", [ColRef(1, "d", DATE)], T.INT32, ("year",))
    assert J._bound(year, b) == (1992, 1998)
    assert J._bound(Func("date_part", [ColRef(1, "d", DATE)], T.INT32, ("month",)), b) == (1, 12)
    del days._igloo_bound
    assert J._bound(year, b) is None
