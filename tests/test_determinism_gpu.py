"""Determinism cross-check: every host readback of every TPC-H
query (sizes, key ranges, strategy flags: the values speculation replays and
query graphs bake in) is identical across repeated executions, and so is every
result. A non-deterministic readback (e.g. hash-slot-order group ids feeding a
packed-key range, found this way in Q16) would make replayed executions fail
validation or, unguarded, index out of bounds."""
import pytest

pytestmark = pytest.mark.gpu


def test_tpch_readbacks_and_results_are_deterministic():
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops import _lib
    from igloo_amd.utils.digest import digest
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, 0.05)
    varying = []
    for q in range(1, 23):
        sql = queries.QUERIES[q]
        e.sql(sql)                          # one-time builds out of the way
        plan, names = e.logical_plan(sql)
        logs, digests = [], set()
        for _ in range(4):
            sp = _lib.Speculation("record")
            _lib.set_speculation(sp)
            try:
                batch = e._execute_plan(plan)
            finally:
                _lib.set_speculation(None)
            logs.append([v for _, v in sp.log])
            digests.add(digest(e._to_arrow(batch, plan.schema, names)))
        if any(l != logs[0] for l in logs[1:]):
            varying.append(q)
        assert len(digests) == 1, (q, digests)
    assert not varying, f"queries with run-to-run varying readbacks: {varying}"
