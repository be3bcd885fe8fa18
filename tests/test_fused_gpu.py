"""Fused scan kernels (csrc/kernels/fused.hip) vs the node-by-node CPU evaluator.

Each query runs on the CPU engine (torch/pyarrow reference semantics) and on
the GPU, where scan filters and small-domain aggregates go through the fused kernels; the
results must be identical (decimals exact, floats to 1e-9 relative)."""
import datetime
import math
from decimal import Decimal

import numpy as np
import pyarrow as pa
import pytest

import igloo_amd as ig
from igloo_amd.ops._lib import KERNEL_CALLS

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["interp", "jit", "jit-mfma"])
def scan_mode(request, monkeypatch):
    """Every test runs on the interpreted kernels (fused.hip), on the generated
    ones (exec/fused_jit.py, compiled synchronously) and on the generated
    one-hot MFMA aggregation."""
    from igloo_amd.exec import fused_jit
    from igloo_amd.ops import jit
    monkeypatch.setattr(fused_jit, "ENABLED", request.param != "interp")
    monkeypatch.setattr(fused_jit, "MFMA", request.param == "jit-mfma")
    monkeypatch.setattr(jit, "MODE", "sync")
    return request.param


def _table(n=300_000, seed=3):
    r = np.random.default_rng(seed)
    price = r.integers(90_000, 10_500_000, n)            # decimal(15,2) scaled
    disc = r.integers(0, 11, n)                           # 0.00 .. 0.10
    tax = r.integers(0, 9, n)
    qty = r.integers(100, 5100, n)
    days = r.integers(8000, 10500, n).astype(np.int32)
    flag = r.choice(["A", "N", "R"], n)
    status = r.choice(["F", "O"], n)
    f = r.normal(0, 100, n)
    k = r.integers(-5, 6, n)
    return pa.table({
        "price": pa.array([Decimal(int(x)) / 100 for x in price], pa.decimal128(15, 2)),
        "disc": pa.array([Decimal(int(x)) / 100 for x in disc], pa.decimal128(15, 2)),
        "tax": pa.array([Decimal(int(x)) / 100 for x in tax], pa.decimal128(15, 2)),
        "qty": pa.array([Decimal(int(x)) / 100 for x in qty], pa.decimal128(15, 2)),
        "d": pa.array(days, pa.int32()).cast(pa.date32()),
        "flag": pa.array(flag, pa.string()).dictionary_encode(),
        "status": pa.array(status, pa.string()).dictionary_encode(),
        "f": pa.array(f, pa.float64()),
        "k": pa.array(k, pa.int64()),
    })


QUERIES = [
    # Q1 shape: filter + 2 dictionary group keys + decimal arithmetic
    """SELECT flag, status, sum(qty) AS sq, sum(price) AS sp, sum(price * (1 - disc)) AS sd,
              sum(price * (1 - disc) * (1 + tax)) AS sc, avg(qty) AS aq, avg(price) AS ap, avg(disc) AS ad,
              count(*) AS c
       FROM t WHERE d <= DATE '1998-12-01' - INTERVAL '90' DAY GROUP BY flag, status ORDER BY flag, status""",
    # Q6 shape: global aggregate, BETWEEN on decimals, date range
    """SELECT sum(price * disc) AS rev FROM t
       WHERE d >= DATE '1994-01-01' AND d < DATE '1995-01-01' AND disc BETWEEN 0.05 AND 0.07 AND qty < 24""",
    # floats, min/max, CASE, IN, integer group key with negative values
    """SELECT k, min(f) AS mn, max(f) AS mx, sum(f * 2.5) AS s, min(price) AS mp, max(d) AS md,
              sum(CASE WHEN flag = 'R' THEN price ELSE 0 END) AS cr, count(*) AS c
       FROM t WHERE k IN (-5, -1, 0, 3, 5) OR f > 150 GROUP BY k ORDER BY k""",
    # product chains (a prefix reused by the next aggregate) mixed with min/max
    # and duplicate arguments; price * price * disc leaves the 32-bit fast path
    """SELECT status, min(price * (1 - disc)) AS a, sum(price * (1 - disc)) AS b, max(price * (1 - disc) * (1 + tax)) AS c,
              sum(price * (1 - disc) * (1 + tax)) AS e, sum(price * price * disc) AS pp, avg(price) AS ap, sum(price) AS sp
       FROM t GROUP BY status ORDER BY status""",
    # empty filter result: global aggregates are NULL / 0
    "SELECT sum(price) AS s, count(*) AS c, min(f) AS m, avg(qty) AS a FROM t WHERE qty < 0",
    # plain filter through the VM mask kernel (no aggregate)
    "SELECT k, d FROM t WHERE NOT (f < -50 OR f > 50) AND price * 2 > 50000 AND d >= DATE '1995-01-01' "
    "AND flag <> 'N' ORDER BY k, d LIMIT 50",
    # decimal column vs literal of another scale / int literal; IN on a dictionary
    "SELECT count(*) AS c, sum(qty) AS s FROM t WHERE qty < 24 AND price > 1000.005 AND status IN ('F', 'X')",
    "SELECT count(*) AS c FROM t WHERE disc = 0.055",
    # OR of conjunctions (Q19 shape): OR-group terms, BETWEEN merged per group
    "SELECT count(*) AS c, sum(price * (1 - disc)) AS r FROM t WHERE status = 'F' AND "
    "((flag = 'A' AND qty BETWEEN 1 AND 11 AND k <= 2) OR (flag = 'R' AND status IN ('F') AND qty BETWEEN 10 AND 20) "
    "OR (qty >= 20 AND qty <= 30 AND d < DATE '1995-01-01'))",
    # a disjunct that never holds (value not in the dictionary) / one that always holds
    "SELECT count(*) AS c FROM t WHERE (flag = 'Z' AND k = 1) OR (k = 2 AND disc > 0.05)",
    "SELECT count(*) AS c FROM t WHERE (k = 1 AND disc < 0.02) OR flag <> 'Z'",
    # a disjunct the kernel cannot take (float): whole OR evaluated node by node
    "SELECT count(*) AS c, sum(qty) AS s FROM t WHERE (f > 10 AND k = 1) OR (k = 3 AND qty < 10)",
]


def _close(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-9) or (math.isnan(a) and math.isnan(b))
    return a == b


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_fused_matches_cpu(gpu_device, qi):
    t = _table()
    sql = QUERIES[qi]
    out = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("t", t)
        out[dev] = e.query(sql).to_pylist()
    assert len(out["cpu"]) == len(out[gpu_device])
    for rc, rg in zip(out["cpu"], out[gpu_device]):
        assert rc.keys() == rg.keys()
        for k in rc:
            assert _close(rc[k], rg[k]), (k, rc[k], rg[k])


def test_fused_kernels_used(gpu_device, scan_mode):
    e = ig.QueryEngine(device=gpu_device)
    e.register_table("t", _table(50_000))
    before = dict(KERNEL_CALLS)
    e.query(QUERIES[0])
    e.query(QUERIES[4])
    if scan_mode != "interp":
        aggs, mask = ("jit:igloo_jit_scan_agg", "jit:igloo_jit_scan_agg_mfma"), "jit:igloo_jit_scan_mask"
    else:
        aggs, mask = ("ff_aggregate",), "ff_mask"
    assert sum(KERNEL_CALLS[a] - before.get(a, 0) for a in aggs) > 0
    assert KERNEL_CALLS[mask] > before.get(mask, 0)


def test_fused_decimal_overflow_detected(gpu_device):
    big = pa.table({"a": pa.array([Decimal("9999999999999.99")] * 1000, pa.decimal128(15, 2)),
                    "b": pa.array([Decimal("9999999999999.99")] * 1000, pa.decimal128(15, 2))})
    e = ig.QueryEngine(device=gpu_device)
    e.register_table("t", big)
    with pytest.raises(Exception, match="overflow"):
        e.query("SELECT sum(a * b) FROM t")


def test_fused_narrow_columns_match_cpu(gpu_device, monkeypatch):
    """Resident int64/int32 columns narrowed to int8/int16/int32 shadows (the
    1/2-byte loads of ff_load) give the same answers as the CPU evaluator."""
    from igloo_amd.exec import fused
    monkeypatch.setattr(fused, "NARROW_MIN_ROWS", 0)
    t = _table(100_000, seed=9)
    eg = ig.QueryEngine(device=gpu_device)
    eg.register_table("t", t)
    ec = ig.QueryEngine(device="cpu")
    ec.register_table("t", t)
    for sql in QUERIES:
        a, b = ec.query(sql).to_pylist(), eg.query(sql).to_pylist()
        assert len(a) == len(b)
        for rc, rg in zip(a, b):
            for k in rc:
                assert _close(rc[k], rg[k]), (sql, k, rc[k], rg[k])
    import torch
    src = eg.catalog.get_table("t")
    widths = {getattr(c.data, "_igloo_narrow", c.data).dtype for c in src.columns.values()}
    assert torch.int8 in widths and torch.int16 in widths


def test_mask_tile_counts_feed_selection(gpu_device, scan_mode, monkeypatch):
    """The generated mask kernel writes each select tile's set-row count with
    the mask (exec/fused_jit.py tiled variant); the selection scans those
    instead of re-reading the mask. Results equal the CPU engine's; counts
    attached to a mask are consumed by its first selection and dropped when
    the mask changes in place."""
    import torch
    from igloo_amd.ops import select as S
    if scan_mode != "jit":
        pytest.skip("tiled counts come from the generated mask kernel")
    n = 1_000_003                               # 123 tiles, the last one partial
    r = np.random.default_rng(4)
    t = pa.table({"a": pa.array(r.integers(0, 1000, n), pa.int32()),
                  "b": pa.array(r.integers(0, 50, n), pa.int16())})
    seen = []
    real = S.attach_tile_counts

    def spy(mask, tc):
        ref = torch.nn.functional.pad(mask.to(torch.int64), (0, (-mask.numel()) % 8192)).view(-1, 8192).sum(1)
        seen.append(bool(torch.equal(tc[:-1], ref)))
        real(mask, tc)
    monkeypatch.setattr(S, "attach_tile_counts", spy)
    sql = "SELECT a, b FROM t WHERE a < 300 AND b >= 10"
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("t", t)
        res[dev] = sorted(e.query(sql).to_pylist(), key=lambda x: (x["a"], x["b"]))
    assert res["cpu"] == res[gpu_device]
    assert seen and all(seen), seen
    # consumed once; an in-place change drops them
    m = torch.from_numpy(r.random(n) < 0.3).to(gpu_device)
    ref = torch.nn.functional.pad(m.to(torch.int64), (0, (-n) % 8192)).view(-1, 8192).sum(1)
    tc = torch.cat([ref, torch.zeros(1, dtype=torch.int64, device=gpu_device)])
    real(m, tc)
    assert torch.equal(S.mask_to_indices(m).long(), torch.nonzero(m).flatten())
    assert m._igloo_tc is None
    real(m, tc.clone())
    m[:5] = True
    assert torch.equal(S.mask_to_indices(m).long(), torch.nonzero(m).flatten())
