"""The range-sliced SEMI / ANTI join (parallel/exchange.py
``_semi_by_range_marks``: the mark_keys / probe_marks kernels, a
reduce-scatter of dense key marks) checked on a one-rank communicator with a
synthetic ("range", W, kmin, chunk) placement: the GPU kernels must equal the
CPU branch and a Python reference, with NULL keys on both sides, right keys
outside the marked domain, and the resident-column path (sorted secondary
index, >= 1M keys). ADVICE r4: these GPU-only branches had no test at world > 1
paths' granularity; a world of one runs the identical kernels and collective."""
import random

import pytest
import torch

from igloo_amd import types as T
from igloo_amd.columnar import Batch, Column
from igloo_amd.exec.context import ExecContext
from igloo_amd.parallel.exchange import _semi_by_range_marks
from igloo_amd.sql import logical as L
from igloo_amd.sql.expr import ColRef


class _OneRank:
    world_size = 1
    rank = 0
    spmd = True
    calls = 0
    bytes_sent = 0

    def reduce_scatter_tensor(self, t, op):
        assert op == "max" and t.dim() == 2 and t.shape[0] == 1
        self.calls += 1
        return t[0].clone()


def _case(n_left, n_right, kmin, chunk, resident=False, seed=0):
    rnd = random.Random(seed)
    lk = [kmin + rnd.randrange(chunk) for _ in range(n_left)]
    lv = [rnd.random() > 0.1 for _ in range(n_left)]
    rk = [kmin - 50 + rnd.randrange(chunk + 100) for _ in range(n_right)]   # some outside [kmin, kmin+chunk)
    rv = None if resident else [rnd.random() > 0.1 for _ in range(n_right)]
    return lk, lv, rk, rv


def _reference(lk, lv, rk, rv, kind):
    have = {k for i, k in enumerate(rk) if rv is None or rv[i]}
    out = []
    for i, k in enumerate(lk):
        hit = lv[i] and k in have
        if (kind == "semi") == hit:
            out.append(i)
    return out


def _run(dev, lk, lv, rk, rv, kmin, chunk, kind, resident=False):
    ctx = ExecContext(device=dev, comm=_OneRank())
    lcol = Column(T.INT64, torch.tensor(lk, dtype=torch.int64, device=dev),
                  torch.tensor(lv, dtype=torch.bool, device=dev))
    rdata = torch.tensor(rk, dtype=torch.int64, device=dev)
    if resident:
        rdata._igloo_resident = True
    rcol = Column(T.INT64, rdata, None if rv is None else torch.tensor(rv, dtype=torch.bool, device=dev))
    rows = Column(T.INT64, torch.arange(len(lk), dtype=torch.int64, device=dev))
    lb = Batch({1: lcol, 3: rows}, len(lk), (("range", 1, kmin, chunk), 1))
    rb = Batch({2: rcol}, len(rk), ("hash", 2))
    j = L.Join(None, None, kind, [(ColRef(1, "lk", T.INT64), ColRef(2, "rk", T.INT64))])
    out = _semi_by_range_marks(lb, rb, j, ctx)
    assert out is not None
    assert ctx.comm.calls == 1
    return sorted(out.columns[3].data.cpu().tolist())


@pytest.mark.parametrize("kind", ["semi", "anti"])
def test_range_marks_cpu(kind):
    lk, lv, rk, rv = _case(3000, 5000, 1000, 4000)
    assert _run("cpu", lk, lv, rk, rv, 1000, 4000, kind) == _reference(lk, lv, rk, rv, kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["semi", "anti"])
@pytest.mark.parametrize("resident", [False, True])
def test_range_marks_gpu(gpu_device, kind, resident):
    from igloo_amd.ops._lib import KERNEL_CALLS
    n_right = (1 << 20) + 123 if resident else 5000
    lk, lv, rk, rv = _case(3000, n_right, 1000, 4000, resident=resident, seed=1)
    before = KERNEL_CALLS["mark_keys"], KERNEL_CALLS["probe_marks"]
    got = _run(gpu_device, lk, lv, rk, rv, 1000, 4000, kind, resident=resident)
    assert KERNEL_CALLS["mark_keys"] > before[0] and KERNEL_CALLS["probe_marks"] > before[1]
    assert got == _run("cpu", lk, lv, rk, rv, 1000, 4000, kind)
    assert got == _reference(lk, lv, rk, rv, kind)
