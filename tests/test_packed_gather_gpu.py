"""Row-packed gathers (ops/packed_gather.py, csrc/kernels/gather.hip
gather_packed) against the per-column gather of the same rows, and a join
query whose payload columns go through them against the packed-off run."""
import numpy as np
import pytest
import torch

from igloo_amd import types as T
from igloo_amd.columnar import Column
from igloo_amd.ops import packed_gather as PG
from igloo_amd.ops._lib import KERNEL_CALLS
from igloo_amd.ops.gather import take_many

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _resident(t):
    t = t.to(DEV)
    t._igloo_resident = True
    return t


def _cols(n, seed=0):
    g = np.random.default_rng(seed)
    a = torch.from_numpy(g.integers(-100, 100, n))                      # int64 -> int8 field
    b = torch.from_numpy(g.integers(0, 1 << 20, n).astype(np.int32))   # int32 -> int32 field
    c = torch.from_numpy(g.integers(-(1 << 40), 1 << 40, n))            # int64, not narrowable
    d = torch.from_numpy(g.random(n).astype(np.float32))
    e = torch.from_numpy(g.integers(0, 7, n).astype(np.int32))
    ev = torch.from_numpy(g.random(n) < 0.8)
    cols = [Column(T.INT64, _resident(a)), Column(T.INT32, _resident(b)), Column(T.INT64, _resident(c)),
            Column(T.FLOAT32, _resident(d)), Column(T.INT32, _resident(e), ev.to(DEV))]
    return cols, [a, b, c, d, e], ev


@pytest.mark.parametrize("neg,incr,i64", [(False, False, False), (True, False, True), (False, True, False)])
def test_packed_take_matches_columns(gpu_device, monkeypatch, neg, incr, i64):
    monkeypatch.setattr(PG, "MIN_ROWS", 1000)
    from igloo_amd.exec import fused
    monkeypatch.setattr(fused, "NARROW_MIN_ROWS", 1000)
    n = 300_000
    cols, host, ev = _cols(n, seed=int(neg) * 2 + int(incr))
    g = np.random.default_rng(7)
    if incr:
        idx = np.flatnonzero(g.random(n) < 0.05)
    else:
        idx = g.integers(0, n, 120_000)
        if neg:
            idx[::7] = -1
    it = torch.from_numpy(idx.astype(np.int64 if i64 else np.int32)).to(DEV)
    if incr:
        it._igloo_incr = True
    before = PG.STATS["gathers"]
    got = take_many(cols, it, neg=neg)
    torch.cuda.synchronize()
    assert PG.STATS["gathers"] == before + 1
    # int8 + int32 + int64 + float32 + int32/validity: all fit one 32-byte row
    assert all(getattr(c.data, "_igloo_packed", None) is None for c in cols[1:]) and cols[0].data._igloo_packed
    ii = torch.from_numpy(idx).long()
    ok = ii >= 0
    safe = ii.clamp(min=0)
    for k, (c, h) in enumerate(zip(got, host)):
        exp = torch.where(ok, h[safe], torch.zeros((), dtype=h.dtype))
        assert c.data.dtype == h.dtype
        assert torch.equal(c.data.cpu(), exp), k
        if k == 4:
            assert torch.equal(c.valid.cpu(), ev[safe] & ok)
        elif neg:
            assert torch.equal(c.valid.cpu(), ok)
        else:
            assert c.valid is None
    # a subset of the kept copy's columns reuses it (no second copy)
    sub = take_many([cols[0], cols[3]], it, neg=neg)
    assert len(cols[0].data._igloo_packed) == 1
    assert torch.equal(sub[1].data.cpu(), got[3].data.cpu())


def test_packed_gather_rejects_bad_fields(gpu_device):
    from igloo_amd.ops._lib import native, ptr
    src = torch.zeros(64, 16, dtype=torch.uint8, device=DEV)
    idx = torch.zeros(4, dtype=torch.int32, device=DEV)
    out = torch.empty(4, dtype=torch.int32, device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    with pytest.raises(RuntimeError):
        native().gather_packed(ptr(idx), False, 4, ptr(src), 64, 16, [(ptr(out), 2, 4, 4, 1)], s)   # misaligned
    with pytest.raises(RuntimeError):
        native().gather_packed(ptr(idx), False, 4, ptr(src), 64, 16, [(ptr(out), 16, 4, 4, 1)], s)  # past the row
    with pytest.raises(RuntimeError):
        native().gather_packed(ptr(idx), False, 4, ptr(src), 64, 12, [(ptr(out), 0, 4, 4, 1)], s)   # row bytes


def test_join_payload_through_packed_copy(gpu_device, monkeypatch):
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    monkeypatch.setattr(PG, "MIN_ROWS", 1)
    e = ig.QueryEngine(device=DEV)
    datagen.register(e, 0.05)
    sql = queries.QUERIES[9]
    monkeypatch.setattr(PG, "PACKED", False)
    ref = e.sql(sql).table
    monkeypatch.setattr(PG, "PACKED", True)
    c0 = KERNEL_CALLS["gather_packed"]
    got = e.sql(sql).table
    assert KERNEL_CALLS["gather_packed"] > c0
    assert got.equals(ref)
