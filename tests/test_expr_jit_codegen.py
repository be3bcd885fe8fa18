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
