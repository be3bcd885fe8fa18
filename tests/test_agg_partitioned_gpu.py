"""Radix-partitioned GROUP BY aggregate (csrc/kernels/agg.hip agg_partitioned):
unclustered group ids past the LDS kernel's group count are bucketed by their
high bits and aggregated in LDS per bucket. Every aggregate kind against the
CPU path of ops/agg.py (a plain PyTorch reference of the same op): exact
128-bit integer SUMs past int64, narrow int32 SUMs, f64 SUM / MIN / MAX,
COUNT with NULLs, bitwise aggregates; out-of-range group ids are skipped."""
import numpy as np
import pytest
import torch

from igloo_amd.ops import agg as A
from igloo_amd.ops._lib import KERNEL_CALLS

pytestmark = pytest.mark.gpu


def _specs(rng, n, dev):
    big = torch.from_numpy(rng.integers(-2**62, 2**62, n, dtype=np.int64))
    small = torch.from_numpy(rng.integers(-10**6, 10**6, n).astype(np.int32))
    f = torch.from_numpy(rng.standard_normal(n) * 1e3)
    valid = torch.from_numpy(rng.random(n) < 0.8)
    cpu = [("sum_int", big, None), ("sum_int", small, None), ("sum_f64", f, valid), ("count", None, valid),
           ("count", None, None), ("min_int", big, valid), ("max_int", small, None), ("min_f64", f, None),
           ("max_f64", f, valid), ("and_int", big, None), ("or_int", small, valid), ("xor_int", big, None)]
    gpu = [(op, None if v is None else v.to(dev), None if m is None else m.to(dev)) for op, v, m in cpu]
    return cpu, gpu


@pytest.mark.parametrize("ngroups", [300_000, 70_001, 9_001])
def test_partitioned_aggregate_matches_cpu(gpu_device, ngroups):
    rng = np.random.default_rng(ngroups)
    n = 3_000_000
    gid = rng.integers(0, ngroups, n).astype(np.int32)
    gid[:1000] = -1                     # out-of-range ids (replayed group counts): skipped
    gid[1000:2000] = ngroups + 5
    cpu, gpu = _specs(rng, n, gpu_device)
    ok = torch.from_numpy((gid >= 0) & (gid < ngroups))
    ref = A._cpu(torch.from_numpy(gid)[ok], ngroups, [(op, None if v is None else v[ok], None if m is None else m[ok])
                                                     for op, v, m in cpu], int(ok.sum()))
    assert A._partitioned_ok(n, ngroups, 8)
    before = KERNEL_CALLS["agg_partitioned"]
    got = A.grouped_aggregate(torch.from_numpy(gid).to(gpu_device), ngroups, gpu, n, gpu_device)
    assert KERNEL_CALLS["agg_partitioned"] > before, "the partitioned kernels did not run"
    for (op, _, _), g, r in zip(cpu, got, ref):
        g = g.cpu()
        if op in ("sum_f64",):
            assert torch.allclose(g, r, rtol=1e-9, atol=1e-6), op
        elif op in ("min_f64", "max_f64"):
            assert torch.equal(g, r), op
        elif r.dim() == 2 or g.dim() == 2:
            assert A.wide_to_python(g) == A.wide_to_python(r), op
        else:
            assert torch.equal(g.to(torch.int64), r.to(torch.int64)), op
    assert got[0].dim() == 2, "the int64 SUM past 2^63 comes back as (lo, hi) pairs"


def test_partitioned_equals_global_atomics(gpu_device, monkeypatch):
    rng = np.random.default_rng(9)
    n, ngroups = 2_500_000, 500_000
    gid = torch.from_numpy(rng.integers(0, ngroups, n).astype(np.int32)).to(gpu_device)
    v = torch.from_numpy(rng.integers(-10**15, 10**15, n, dtype=np.int64)).to(gpu_device)
    specs = [("sum_int", v, None), ("count", None, None), ("max_int", v, None)]
    a = A.grouped_aggregate(gid, ngroups, specs, n, gpu_device)
    monkeypatch.setattr(A, "AGG_PARTITIONED", False)
    b = A.grouped_aggregate(gid, ngroups, specs, n, gpu_device)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
