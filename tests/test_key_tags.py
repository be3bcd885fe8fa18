"""Readback-free key facts are verified against the data they describe
(a wrongly tagged ``_igloo_distinct`` / ``_igloo_unique`` tensor
would make inner joins silently drop rows). With ``CHECK_KEY_TAGS`` on,
every ``key_unique`` shortcut is checked against the join build's own
duplicate count and every ``key_bound`` against the keys' real range, over
the whole TPC-H suite (CPU: bounds; GPU: bounds and uniqueness tags)."""
import pytest

from igloo_amd.ops import hashing as H


def _suite(dev, monkeypatch):
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, oracle, queries as Q
    monkeypatch.setattr(H, "CHECK_KEY_TAGS", True)
    e = ig.QueryEngine(device=dev)
    tabs = datagen.register(e, 0.01)
    con = oracle.load_sqlite(datagen.to_arrow(tabs))
    bad = []
    for q in range(1, 23):
        rows = [[oracle.normalize(v) for v in r.values()] for r in e.sql(Q.QUERIES[q]).table.to_pylist()]
        exp = [tuple(str(x) if isinstance(x, str) else x for x in row) for row in oracle.run_sqlite(con, q)]
        d = oracle.rows_match([tuple(r) for r in rows], exp)
        if d:
            bad.append(f"Q{q}: {d}")
    assert not bad, bad


def test_key_facts_cpu(monkeypatch):
    _suite("cpu", monkeypatch)


@pytest.mark.gpu
def test_key_facts_gpu(gpu_device, monkeypatch):
    _suite(gpu_device, monkeypatch)


def test_bad_bound_tag_is_caught(monkeypatch):
    import torch
    monkeypatch.setattr(H, "CHECK_KEY_TAGS", True)
    k = torch.tensor([5, 9, 12], dtype=torch.int64)
    k._igloo_bound = (0, 10)
    with pytest.raises(AssertionError):
        H.key_bound(k)
