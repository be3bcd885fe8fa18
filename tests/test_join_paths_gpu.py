"""Every physical join strategy vs the CPU engine on the same data.

The GPU picks among hash build/probe (with or without the Bloom pre-filter),
reverse builds for semi/anti/left joins against a much larger side, and the
binary-search path when the big side's key column is sorted. Thresholds are
lowered so small inputs exercise each path; results must equal the CPU
reference exactly (order-insensitive)."""
import numpy as np
import pyarrow as pa
import pytest
import torch

import igloo_amd as ig
from igloo_amd.exec import joins as J
from igloo_amd.ops import hashing as H

pytestmark = pytest.mark.gpu


def _tables(seed=5, n_big=200_000, n_small=3_000, sorted_big=True):
    r = np.random.default_rng(seed)
    k = r.integers(0, n_big // 4, n_big)
    if sorted_big:
        k = np.sort(k)
    big = pa.table({"bk": pa.array(k, pa.int64()), "bs": pa.array(r.integers(0, 7, n_big), pa.int64()),
                    "bv": pa.array(r.integers(-100, 100, n_big), pa.int64())})
    sk = r.integers(-10, n_big // 4 + 10, n_small)
    sv = pa.array(r.integers(0, 7, n_small), pa.int64())
    small = pa.table({"sk": pa.array(sk, pa.int64()), "ss": sv,
                      "sn": pa.array([None if i % 17 == 0 else int(x) for i, x in enumerate(sk)], pa.int64())})
    return big, small


QUERIES = [
    "SELECT sk, bv FROM small JOIN big ON sk = bk",
    "SELECT sk, bv FROM small JOIN big ON sk = bk AND bs <> ss",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk)",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs <> ss)",
    "SELECT sk FROM small WHERE NOT EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs <> ss)",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs < ss)",
    "SELECT sk FROM small WHERE NOT EXISTS (SELECT 1 FROM big WHERE bk = sk AND ss >= bs)",
    "SELECT sn, count(bv) AS c FROM small LEFT JOIN big ON sn = bk GROUP BY sn",
    "SELECT sn FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sn)",
    "SELECT sn FROM small WHERE NOT EXISTS (SELECT 1 FROM big WHERE bk = sn)",
    "SELECT sk, count(*) AS c FROM small JOIN big ON sk = bk GROUP BY sk",
]


def _norm(t):
    return sorted((tuple((k, v) for k, v in sorted(r.items())) for r in t.to_pylist()), key=repr)


@pytest.mark.parametrize("sorted_big,perm", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_join_paths_match_cpu(gpu_device, monkeypatch, sorted_big, perm, qi):
    """perm: the unsorted resident big side is joined through its secondary
    (sorted permutation) index instead of a hash probe."""
    monkeypatch.setattr(J, "PERM_INDEX", perm)
    monkeypatch.setattr(J, "PERM_INDEX_MAX_FRAC", 1)
    monkeypatch.setattr(J, "SEMI_MARKS_MIN_ROWS", 1000 if perm else 1 << 22)   # [NOT] EXISTS as index key marks
    monkeypatch.setattr(J, "SORTED_JOIN_MIN_ROWS", 1000)
    monkeypatch.setattr(H, "SORTED_CHECK_ROWS", 1000)
    monkeypatch.setattr(H, "BLOOM_MIN_RATIO", 2)
    big, small = _tables(sorted_big=sorted_big)
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("big", big)
        e.register_table("small", small)
        res[dev] = _norm(e.query(QUERIES[qi]))
    assert res["cpu"] == res[gpu_device]


def _phases(e, sql):
    txt = e.sql("EXPLAIN ANALYZE " + sql).table.column("plan").to_pylist()[0]
    return txt[txt.find("phases"):]


@pytest.mark.parametrize("skewed", [False, True])
def test_perm_index_default_gating(gpu_device, skewed):
    """Default thresholds (no monkeypatching): an unsorted resident 4.2M-row
    key column joined with 1000 keys goes through its secondary index when the
    matching ranges are small, and falls back to the hash join after the index
    search when a hot key makes the result too large. The chosen
    path is read from EXPLAIN ANALYZE's phase spans; answers match the CPU."""
    n = (1 << 22) + 100_000
    r = np.random.default_rng(11)
    k = r.permutation(n).astype(np.int64)
    if skewed:
        k[: n // 2] = 0                  # one hot key: half the column
        r.shuffle(k)
    big = pa.table({"bk": pa.array(k), "bv": pa.array(r.integers(0, 1000, n), pa.int64())})
    sk = r.choice(n, 1000, replace=False).astype(np.int64)
    sk[0] = 0
    small = pa.table({"sk": pa.array(sk)})
    sql = "SELECT count(*) AS c, sum(bv) AS s FROM small JOIN big ON sk = bk"
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("big", big)
        e.register_table("small", small)
        res[dev] = e.query(sql).to_pylist()
        if dev != "cpu":
            ph = _phases(e, sql)
            assert "join.index_search" in ph, ph
            if skewed:
                assert "join.index_expand" not in ph and "join.probe" in ph, ph
            else:
                assert "join.index_expand" in ph and "join.probe" not in ph, ph
    assert res["cpu"] == res[gpu_device]


def _index_tables(n=(1 << 22) + 50_000, n_small=40_000, seed=13):
    """A 4.2M-row resident big side whose key column repeats every key 8 times
    (unsorted: ``bk``; sorted copy: ``ok``) and a small key set."""
    r = np.random.default_rng(seed)
    k = r.permutation(np.repeat(np.arange(n // 8 + 1, dtype=np.int64), 8)[:n])
    big = pa.table({"bk": pa.array(k), "ok": pa.array(np.sort(k)), "bv": pa.array(r.integers(0, 1000, n), pa.int64())})
    small = pa.table({"sk": pa.array(r.choice(n // 8, n_small, replace=False).astype(np.int64)),
                      "sw": pa.array(r.integers(1, 5, n_small), pa.int64())})
    return big, small


INDEX_QUERIES = [
    # inner join, ~7.6 % of the big side: secondary index + sort back into row order
    ("SELECT count(*) AS c, sum(bv) AS s, sum(bv * sw) AS t FROM small JOIN big ON sk = bk", "join.index_sort"),
    # correlated aggregate (Q17 shape): the runtime key filter reads the index ranges
    ("SELECT sum(bv) AS s FROM small, big WHERE bk = sk AND bv < (SELECT avg(b2.bv) FROM big b2 WHERE b2.bk = sk)",
     None),
    # semi join of the big side with a small key set (sorted and unsorted key columns)
    ("SELECT count(*) AS c, sum(bv) AS s FROM big WHERE bk IN (SELECT sk FROM small WHERE sw = 1)", None),
    ("SELECT count(*) AS c, sum(bv) AS s FROM big WHERE ok IN (SELECT sk FROM small WHERE sw = 1)", None),
    # [NOT] EXISTS against a filtered scan sorted on the key (Q4 shape): index
    # nested loop, the scan filter evaluated on the candidate rows only
    ("SELECT count(*) AS c, sum(sw) AS s FROM small WHERE EXISTS (SELECT * FROM big WHERE ok = sk AND bv < 100)",
     "join.index_then_filter"),
    ("SELECT count(*) AS c, sum(sw) AS s FROM small WHERE NOT EXISTS (SELECT * FROM big WHERE ok = sk AND bv < 20)",
     "join.index_then_filter"),
    # Q21 shape: both, deferred past a multi-way join, with residuals on the candidate pairs
    ("SELECT count(*) AS c, sum(b1.bv) AS s FROM big b1, small WHERE b1.ok = sk AND sk < 50000 "
     "AND EXISTS (SELECT * FROM big b2 WHERE b2.ok = b1.ok AND b2.bv <> b1.bv AND b2.bv < 500) "
     "AND NOT EXISTS (SELECT * FROM big b3 WHERE b3.ok = b1.ok AND b3.bk <> b1.bk AND b3.bv < 30)",
     None),
]


@pytest.mark.parametrize("qi", range(len(INDEX_QUERIES)))
def test_index_paths_default_thresholds(gpu_device, qi, monkeypatch):
    """Mid-size secondary-index joins, index-range runtime key filters and
    semi joins (exec/joins.py inner_pairs, _index_key_filter) with the
    default thresholds, against the CPU engine."""
    big, small = _index_tables()
    sql, phase = INDEX_QUERIES[qi]
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("big", big)
        e.register_table("small", small)
        res[dev] = e.query(sql).to_pylist()
        if dev != "cpu" and phase:
            ph = _phases(e, sql)
            assert phase in ph, ph
    assert res["cpu"] == res[gpu_device]


@pytest.mark.parametrize("nullable", [False, True])
@pytest.mark.parametrize("pred", ["bv <> 5", "bv = 5", "bv > -90"])
def test_eager_count_masked_complement(gpu_device, monkeypatch, pred, nullable):
    """Q13 shape (LEFT JOIN ... COUNT per left key over a filtered resident
    right scan): a filter most rows pass subtracts the failing rows' per-key
    counts from the column's remembered histogram (exec/aggregate.py
    _full_key_hist); a selective one histograms the passing rows. Both equal
    the CPU engine's plain join + aggregate. ``nullable``: columns declared
    nullable without any NULL (as Parquet files declare them) take the path too."""
    from igloo_amd.exec import aggregate as AG
    calls = []
    real = AG._full_key_hist
    monkeypatch.setattr(AG, "_full_key_hist", lambda *a: calls.append(1) or real(*a))
    r = np.random.default_rng(3)
    n_big, n_small = 300_000, 40_000
    big = pa.table({"bk": pa.array(r.integers(1, n_small, n_big), pa.int64()),
                    "bv": pa.array(r.integers(-100, 100, n_big), pa.int64())},
                   schema=pa.schema([pa.field("bk", pa.int64(), nullable), pa.field("bv", pa.int64(), nullable)]))
    small = pa.table({"sk": pa.array(np.arange(n_small), pa.int64())},
                     schema=pa.schema([pa.field("sk", pa.int64(), False)]))
    sql = (f"SELECT c, count(*) AS n FROM (SELECT sk, count(bv) AS c FROM small LEFT JOIN big "
           f"ON sk = bk AND {pred} GROUP BY sk) t GROUP BY c")
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("big", big)
        e.register_table("small", small)
        res[dev] = _norm(e.query(sql))
        if dev != "cpu":
            assert _norm(e.query(sql)) == res[dev]        # again with the remembered histogram
    assert res["cpu"] == res[gpu_device]
    assert calls, "the masked eager COUNT path did not run"


@pytest.mark.parametrize("sorted_min", [1000, 1 << 40])
def test_in_place_filtered_probe_side(gpu_device, monkeypatch, sorted_min):
    """A filtered big scan in index form searches its table's own sorted key
    column under the filter mask (joins.py _in_place_side, masked_expand);
    TPC-H joins vs the gathered-key run, with the sorted path on and off."""
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops._lib import KERNEL_CALLS
    from igloo_amd.utils.digest import digest
    monkeypatch.setattr(J, "SORTED_JOIN_MIN_ROWS", sorted_min)
    monkeypatch.setattr(H, "CHECK_KEY_TAGS", True)     # inferred sorted / bound / unique tags must hold
    e = ig.QueryEngine(device=gpu_device)
    datagen.register(e, 0.05)
    for q in (3, 5, 7, 9, 10, 12, 21):
        monkeypatch.setattr(J, "IN_PLACE_MIN_DENSITY", 0.0)
        want = digest(e.query(queries.QUERIES[q]))
        monkeypatch.setattr(J, "IN_PLACE_MIN_DENSITY", 0.125)
        assert digest(e.query(queries.QUERIES[q] + " ")) == want, q
    if sorted_min == 1000:
        assert J.IN_PLACE_STATS["probes"] > 0 and KERNEL_CALLS["sorted_masked"] > 0


def test_in_place_exists_side(gpu_device, monkeypatch):
    """[NOT] EXISTS against a filtered scan in index form searches the
    table's own sorted key column under the filter mask (joins.py
    _in_place_semi; Q21's l3, Q4's lineitem) vs the compacted run."""
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.utils.digest import digest
    monkeypatch.setattr(J, "SORTED_JOIN_MIN_ROWS", 1000)
    e = ig.QueryEngine(device=gpu_device)
    datagen.register(e, 0.05)
    s0 = J.IN_PLACE_STATS["semis"]
    for q in (4, 16, 20, 21, 22):
        monkeypatch.setattr(J, "IN_PLACE_MIN_DENSITY", 0.0)
        want = digest(e.query(queries.QUERIES[q]))
        monkeypatch.setattr(J, "IN_PLACE_MIN_DENSITY", 0.125)
        assert digest(e.query(queries.QUERIES[q] + " ")) == want, q
    assert J.IN_PLACE_STATS["semis"] > s0


@pytest.mark.parametrize("kdt", [torch.int32, torch.int64])
@pytest.mark.parametrize("nb,dense,nulls", [(1000, False, False), (300_000, True, True), (300_000, False, True),
                                            (5_000_000, False, False), (5_000_000, True, False)])
def test_unique_lookup_matches_searchsorted(gpu_device, kdt, nb, dense, nulls, monkeypatch):
    """ops/hashing.py unique_lookup (ranges.hip unique_lookup: dense table or
    fenced binary search) against numpy searchsorted over distinct sorted keys."""
    rng = np.random.default_rng(nb + (7 if dense else 0))
    step = 1 if dense else 5
    keys = np.unique(rng.integers(0, nb * step * 2, nb)).astype(np.int64)
    q = rng.integers(-5, nb * step * 2 + 5, 3 * nb).astype(np.int64)
    qv = rng.random(q.size) > 0.1 if nulls else None
    big = torch.from_numpy(keys).to(kdt).to(gpu_device)
    if dense:
        monkeypatch.setattr(H, "DENSE_INDEX_MIN_QUERIES", 1)
    else:
        monkeypatch.setattr(H, "DENSE_INDEX", False)
    if nb >= 4_000_000:
        big._igloo_resident = True          # (the fence serves resident columns)
    hit, pos = H.unique_lookup(big, torch.from_numpy(q).to(kdt).to(gpu_device),
                               None if qv is None else torch.from_numpy(qv).to(gpu_device))
    lo = np.searchsorted(keys, q)
    want = (lo < keys.size) & (keys[np.minimum(lo, keys.size - 1)] == q)
    if qv is not None:
        want &= qv
    assert np.array_equal(hit.cpu().numpy(), want)
    assert np.array_equal(pos.cpu().numpy(), np.where(want, lo, 0))
    assert pos.dtype == torch.int32


@pytest.mark.parametrize("m", [1, 3, 4, 1000, 8192, 8195, 100_003, 1_000_003, 5_000_003])
@pytest.mark.parametrize("masked,negate,offset", [(False, False, 0), (True, False, 0), (True, True, 0),
                                                  (True, False, 1)])
def test_probe_bits_kernel_matches_scalar(gpu_device, m, masked, negate, offset):
    """hashtable.hip probe_bits_kernel (int32 keys, direct table with an
    exact bitmap: 4 rows per lane, vector loads) and probe_fold_kernel (the
    bitmap folded into LDS, from 4M probe rows) write the same hit words and
    counts as probe_hits_kernel -- tails, NULL masks, NOT EXISTS, and an
    unaligned probe view (the host falls back to the scalar kernel)."""
    from igloo_amd.ops._lib import native
    rng = np.random.default_rng(m)
    span = 100_000
    build = torch.from_numpy(rng.choice(np.arange(1, span + 1), 4000, replace=False).astype(np.int32)).to(gpu_device)
    base = torch.from_numpy(rng.integers(-10, span + 10, m + offset).astype(np.int32)).to(gpu_device)
    probe = base[offset:]
    valid = torch.from_numpy(rng.random(m) > 0.3).to(gpu_device) if masked else None
    table = H.JoinTable(build, None, defer_unique=False)
    if m >= H.BLOOM_MIN_RATIO * build.numel():
        # (the shape the vector kernel serves: direct table, exact bitmap in use)
        bits, bmask = table._bloom(m)
        assert table.direct and bits and bmask & (1 << 63), (table.direct, bits, bmask)
    outs = []
    for mode in (2, 1, 0):
        native().set_probe_bits(mode)
        try:
            outs.append(table.probe_select(probe, valid, negate=negate, want_build=not negate))
        finally:
            native().set_probe_bits(2)
    (p1, b1), (p0, b0) = outs[0], outs[2]
    for p, b in outs[1:]:
        assert torch.equal(p1, p)
        assert (b1 is None and b is None) or torch.equal(b1, b)
    keys = probe.cpu().numpy()
    hit = np.isin(keys, build.cpu().numpy())
    if valid is not None:
        hit &= valid.cpu().numpy()
    want = np.nonzero(~hit if negate else hit)[0]
    assert np.array_equal(p1.cpu().numpy(), want)


def test_probe_fold_kernel_wide_bitmap(gpu_device):
    """probe_fold_kernel with a bitmap wider than its 64 KiB LDS fold (2M-key
    span): folded hits are confirmed against the exact bitmap."""
    from igloo_amd.ops._lib import native
    rng = np.random.default_rng(11)
    span, m = 2_000_000, 5_000_001
    build = torch.from_numpy(rng.choice(np.arange(1, span + 1), 50_000, replace=False).astype(np.int32)).to(gpu_device)
    probe = torch.from_numpy(rng.integers(0, span + 2, m).astype(np.int32)).to(gpu_device)
    valid = torch.from_numpy(rng.random(m) > 0.5).to(gpu_device)
    table = H.JoinTable(build, None, defer_unique=False)
    bits, bmask = table._bloom(m)
    assert table.direct and bits and bmask & (1 << 63)
    outs = []
    for mode in (2, 0):
        native().set_probe_bits(mode)
        try:
            outs.append(table.probe_select(probe, valid))
        finally:
            native().set_probe_bits(2)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    hit = np.isin(probe.cpu().numpy(), build.cpu().numpy()) & valid.cpu().numpy()
    assert np.array_equal(outs[0][0].cpu().numpy(), np.nonzero(hit)[0])


@pytest.mark.parametrize("m", [8195, 100_003, 5_000_003])
def test_probe_bits_int64_keys(gpu_device, m):
    """The vector / folded bitmap probes over int64 probe keys (two 16-byte
    loads per 4 rows) agree with the scalar kernel and with numpy."""
    from igloo_amd.ops._lib import native
    rng = np.random.default_rng(m + 1)
    off = 10**12
    build = torch.from_numpy(off + rng.choice(np.arange(1, 200_001), 5000, replace=False).astype(np.int64)).to(gpu_device)
    probe = torch.from_numpy(off + rng.integers(-5, 200_010, m).astype(np.int64)).to(gpu_device)
    valid = torch.from_numpy(rng.random(m) > 0.2).to(gpu_device)
    table = H.JoinTable(build, None, defer_unique=False)
    outs = []
    for mode in (2, 1, 0):
        native().set_probe_bits(mode)
        try:
            outs.append(table.probe_select(probe, valid))
        finally:
            native().set_probe_bits(2)
    for p, b in outs[1:]:
        assert torch.equal(outs[0][0], p) and torch.equal(outs[0][1], b)
    hit = np.isin(probe.cpu().numpy(), build.cpu().numpy()) & valid.cpu().numpy()
    assert np.array_equal(outs[0][0].cpu().numpy(), np.nonzero(hit)[0])


def test_perm_index_keys_get_dense_ranges(gpu_device):
    """The sorted keys of a resident column's secondary index get the dense
    lower-bound table like a sorted resident column (built once, charged to
    the column): Q9's 1.1M green parts looked their l_partkey ranges up by
    bisection of 600M keys. Ranges equal torch.searchsorted's, including keys
    in long gaps and outside the key span."""
    from igloo_amd.utils.memory import derived_nbytes
    r = np.random.default_rng(3)
    k = torch.from_numpy(r.integers(0, 50_000, 400_000)).to(torch.int32).to(gpu_device)
    k[k % 7 == 3] += 200_000            # a sparse upper tail: long gaps in the key span
    k._igloo_resident = True
    skeys, perm = H.perm_index(k)
    q = torch.from_numpy(r.integers(-5, 260_000, 8192)).to(torch.int32).to(gpu_device)
    lo, cnt = H.sorted_ranges(skeys, q)
    assert getattr(skeys, "_igloo_dense", None), "no dense table on the index keys"
    ref_lo = torch.searchsorted(skeys, q)
    ref_cnt = torch.searchsorted(skeys, q, right=True) - ref_lo
    assert torch.equal(cnt, ref_cnt)
    assert torch.equal(lo[cnt > 0], ref_lo[cnt > 0])
    first = skeys._igloo_dense[2]
    assert derived_nbytes(k) >= skeys.numel() * 4 + perm.numel() * perm.element_size() + first.numel() * first.element_size()
