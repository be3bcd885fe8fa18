"""Numerics of every gfx950 kernel vs the CPU reference implementation of the
same op (torch / pyarrow on the host). Runs on a real MI355X."""
import numpy as np
import pyarrow as pa
import pytest
import torch

from igloo_amd import types as T
from igloo_amd.columnar import Column
from igloo_amd.ops import agg as A
from igloo_amd.ops import hashing as H
from igloo_amd.ops import misc as M
from igloo_amd.ops import strings as S
from igloo_amd.ops.select import mask_to_indices
from igloo_amd.ops.gather import take_many
from igloo_amd.ops.select import exclusive_scan, mask_to_indices

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rng(seed=0):
    return np.random.default_rng(seed)


@pytest.mark.parametrize("n", [0, 1, 17, 4096, 4097, 8192, 8193, 65536, 65537, 1_000_003])
def test_select(gpu_device, n):
    m = torch.from_numpy(_rng(n).random(n) < 0.3)
    ref = mask_to_indices(m)
    got = mask_to_indices(m.to(DEV)).cpu()
    assert got.dtype == ref.dtype and torch.equal(got, ref)


@pytest.mark.parametrize("n,dt", [(0, torch.int32), (5, torch.int32), (8191, torch.int64), (8192, torch.int32),
                                  (8193, torch.int32), (100_001, torch.int64), (3_000_000, torch.int32)])
def test_exclusive_scan(gpu_device, n, dt):
    c = torch.from_numpy(_rng(1).integers(0, 9, n)).to(dt)
    ref, rt = exclusive_scan(c)
    got, gt = exclusive_scan(c.to(DEV))
    assert rt == gt and torch.equal(got.cpu(), ref)
    if n:
        got2, dt_ = exclusive_scan(c.to(DEV), host_total=False)     # the total left on the device
        assert int(dt_.item()) == rt and torch.equal(got2.cpu(), ref)


def test_take_many_fixed_strings_nulls(gpu_device):
    r = _rng(2)
    n = 50_000
    vals = r.integers(-10**12, 10**12, n)
    strs = pa.array([None if i % 7 == 0 else "s" * (i % 13) + str(i) for i in range(n)], pa.large_string())
    cols = [Column(T.INT64, torch.from_numpy(vals)), Column.from_arrow(strs, dict_encode=False),
            Column(T.DATE32, torch.from_numpy(r.integers(0, 20000, n).astype(np.int32)),
                   torch.from_numpy(r.random(n) < 0.9))]
    idx = torch.from_numpy(r.integers(-1, n, 123_457).astype(np.int32))
    ref = take_many(cols, idx, neg=True)
    got = take_many([c.to(DEV) for c in cols], idx.to(DEV), neg=True)
    for a, b in zip(ref, got):
        assert a.to_arrow().equals(b.to_arrow())


@pytest.mark.parametrize("dense", [True, False])
@pytest.mark.parametrize("dups", [False, True])
def test_join_table(gpu_device, dense, dups):
    r = _rng(3)
    nb = 200_000
    span = nb if dense else 10**15
    bk = torch.from_numpy(r.choice(span, nb, replace=dups).astype(np.int64))
    pk = torch.cat([bk[: nb // 2], torch.from_numpy(r.integers(0, span, 300_000))])
    bvalid = torch.from_numpy(r.random(nb) < 0.95)
    cpu = H.JoinTable(bk, bvalid)
    gpu = H.JoinTable(bk.to(DEV), bvalid.to(DEV))
    assert cpu.unique == gpu.unique
    assert gpu.direct == dense
    rp, rb, rc = cpu.probe_pairs(pk)
    gp, gb, gc = gpu.probe_pairs(pk.to(DEV))
    assert torch.equal(rc, gc.cpu())
    a = sorted(zip(rp.tolist(), rb.tolist()))
    b = sorted(zip(gp.cpu().tolist(), gb.cpu().tolist()))
    assert a == b
    fm = gpu.probe_first(pk.to(DEV)).cpu()
    assert torch.equal(fm >= 0, rc > 0)
    ok = fm >= 0
    assert torch.equal(bk[fm[ok].long()], pk[ok])
    # duplicate keys take the CSR layout (contiguous runs of build rows)
    assert (gpu.cstart is not None) == (not gpu.unique)
    if gpu.cstart is not None:
        assert int(gpu.cstart[-1]) == int(bvalid.sum())
    # build-side match marks (right/full outer joins) through both layouts
    mc = torch.zeros(nb, dtype=torch.bool)
    mg = torch.zeros(nb, dtype=torch.bool, device=DEV)
    cpu.probe_pairs(pk, build_matched=mc)
    gpu.probe_pairs(pk.to(DEV), build_matched=mg)
    assert torch.equal(mc, mg.cpu())


@pytest.mark.parametrize("card", [1, 6, 1000, 3_000_000])
def test_group_ids(gpu_device, card):
    r = _rng(4)
    n = 2_000_000
    keys = torch.from_numpy(r.integers(0, card, n) * (1 if card < 10**4 else 7919))
    g, ng, rep = H.group_ids(keys.to(DEV))
    rg, rng_, rrep = H.group_ids(keys)
    assert ng == rng_
    g, rep = g.cpu().long(), rep.cpu().long()
    # same partition of rows: group of each row's key identical up to relabeling
    assert torch.equal(keys[rep][g], keys)
    assert torch.unique(keys[rep]).numel() == ng
    # representative is the first occurrence
    first = torch.full((ng,), n, dtype=torch.int64).scatter_reduce(0, g, torch.arange(n), reduce="amin")
    assert torch.equal(first, rep)


@pytest.mark.parametrize("ngroups", [1, 4, 300, 100_000])
def test_grouped_aggregate(gpu_device, ngroups):
    r = _rng(5)
    n = 1_000_000
    gid = torch.from_numpy(r.integers(0, ngroups, n).astype(np.int32))
    iv = torch.from_numpy(r.integers(-(2**40), 2**40, n))
    i32 = torch.from_numpy(r.integers(-1000, 1000, n).astype(np.int32))
    fv = torch.from_numpy(r.standard_normal(n))
    valid = torch.from_numpy(r.random(n) < 0.8)
    specs = [("sum_int", iv, None), ("sum_int", i32, valid), ("count", None, None), ("count", None, valid),
             ("min_int", iv, valid), ("max_int", i32, None), ("min_f64", fv, None), ("max_f64", fv, valid)]
    ref = A.grouped_aggregate(gid, ngroups, specs, n, "cpu")
    got = A.grouped_aggregate(gid.to(DEV), ngroups, [(o, None if v is None else v.to(DEV), None if m is None else m.to(DEV))
                                                    for o, v, m in specs], n, DEV)
    for (op, _, _), a, b in zip(specs, ref, got):
        assert torch.equal(a, b.cpu()), op
    # sum_f64 with tolerance (atomic order differs)
    fs = A.grouped_aggregate(gid.to(DEV), ngroups, [("sum_f64", fv.to(DEV), None)], n, DEV)[0].cpu()
    fr = A.grouped_aggregate(gid, ngroups, [("sum_f64", fv, None)], n, "cpu")[0]
    assert torch.allclose(fs, fr, rtol=1e-9, atol=1e-6)


def test_sum_int128_overflow(gpu_device):
    n = 100_000
    v = torch.full((n,), 2**62, dtype=torch.int64)
    gid = torch.zeros(n, dtype=torch.int32)
    got = A.grouped_aggregate(gid.to(DEV), 3, [("sum_int", v.to(DEV), None)], n, DEV)[0]
    assert A.wide_to_python(got)[0] == n * 2**62


def _str_col(vals, dict_encode=False):
    return Column.from_arrow(pa.array(vals, pa.large_string()), dict_encode=dict_encode)


WORDS = ["special", "requests", "forest green", "PROMO BRUSHED", "Customer xx Complaints", "", "a_b%c", "ünïcode"]


def _words(n, seed=6):
    r = _rng(seed)
    return [" ".join(r.choice(WORDS, r.integers(0, 5))) for _ in range(n)]


@pytest.mark.parametrize("pat", ["%special%requests%", "forest%", "%BRASS", "%", "", "_", "a\\_b\\%c%", "%n_c%",
                                 "%Customer%Complaints%", "special", "spec%cial", "special%special", "%al%al%",
                                 "%%", "%s", "f%n", "%e%e%e%e%", "%e%e%e%e%e%", "PROMO%", "%requests"])
def test_like(gpu_device, pat):
    # segment-bitmap kernel for '_'-free patterns, generic matcher otherwise
    vals = _words(20_000)
    c = _str_col(vals)
    ref = S.like(c, pat)
    got = S.like(c.to(DEV), pat).cpu()
    assert torch.equal(ref, got)
    assert torch.equal(S.like(c, pat, negate=True), S.like(c.to(DEV), pat, negate=True).cpu())


def test_like_long_strings_and_slices(gpu_device):
    # tiles whose bytes overflow the LDS stage (unstaged path), mixed with short
    # ones, and a sliced column whose character buffer starts mid-allocation
    r = _rng(9)
    vals = []
    for i in range(5000):
        w = " ".join(r.choice(WORDS, r.integers(0, 40 if i % 700 < 300 else 4)))
        vals.append(w)
    c = _str_col(vals)
    for pat in ("%special%requests%", "%green", "Customer%", "%ü%", "special%requests", "%s%s%", "%n_c%"):
        ref = S.like(c, pat)
        assert torch.equal(ref, S.like(c.to(DEV), pat).cpu())
    from igloo_amd.ops.gather import take
    idx = torch.arange(3, 4999, 3, dtype=torch.int32)
    sub_cpu = take(c, idx)
    sub_gpu = take(c.to(DEV), idx.to(DEV))
    assert torch.equal(S.like(sub_cpu, "%requests%"), S.like(sub_gpu, "%requests%").cpu())


def test_string_transforms(gpu_device):
    vals = [w.replace("ü", "u").replace("ï", "i") for w in _words(30_000, 7)]
    c = _str_col(vals)
    g = c.to(DEV)
    assert S.upper(g).to_arrow().equals(S.upper(c).to_arrow())
    for start, ln in [(1, 2), (3, None), (0, 3), (5, 0), (-2, 4)]:
        assert S.substr(g, start, ln).to_pylist() == S.substr(c, start, ln).to_pylist()
    for op in ["=", "<>", "<", ">="]:
        assert torch.equal(S.compare_const(g, op, "requests").cpu(), S.compare_const(c, op, "requests"))


def test_upper_unicode_falls_back_exactly(gpu_device):
    c = _str_col(["straße", "abc", None, "ÄÖü"])
    assert S.upper(c.to(DEV)).to_pylist() == ["STRASSE", "ABC", None, "ÄÖÜ"]


def test_dict_encode(gpu_device):
    vals = _words(50_000, 8)
    c = _str_col(vals).to(DEV)
    d = S.dict_encode(c)
    assert d.is_dict
    assert d.to_pylist() == vals
    assert len(d.dictionary) == len(set(vals))


@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_hash_partition(gpu_device, nparts):
    keys = torch.from_numpy(_rng(9).integers(0, 10**9, 777_777))
    perm, counts = M.hash_partition(keys.to(DEV), nparts)
    rperm, rcounts = M.hash_partition(keys, nparts)
    assert counts == rcounts
    assert torch.equal(perm.cpu().long(), rperm.long())


def test_date_part(gpu_device):
    d = torch.from_numpy(_rng(10).integers(-30000, 40000, 100_000).astype(np.int32))
    for f in ["year", "month", "day", "quarter", "dow", "doy"]:
        assert torch.equal(M.date_part(d.to(DEV), f).cpu(), M.date_part(d, f)), f


@pytest.mark.parametrize("card,n", [(1, 1000), (50, 100_000), (20_000, 1_000_000), (3_000_000, 6_000_000)])
def test_hll_ndv(gpu_device, card, n):
    g = _rng(11)
    k = torch.from_numpy(g.integers(0, card, n).astype(np.int32)).to(gpu_device)
    exact = torch.unique(k).numel()
    est = H.ndv(k)
    assert abs(est - exact) <= max(2, 0.05 * exact), (est, exact)
    # int64 keys with NULLs: nulls are not counted
    k64 = k.to(torch.int64) * 1_000_003
    valid = k % 2 == 0
    exact2 = torch.unique(k64[valid]).numel()
    est2 = H.ndv(k64, valid)
    assert abs(est2 - exact2) <= max(2, 0.05 * exact2), (est2, exact2)


def test_group_by_functional_dependency(gpu_device):
    """FD shortcut: a string key that is constant per int key is dropped from the
    grouping; one that is not must still split the groups (and NULLs count)."""
    import igloo_amd as ig
    n = 200_000
    g = _rng(12)
    k = g.integers(0, 5000, n)
    dep = np.array([f"name-{x:05d}" for x in k], dtype=object)
    nodep = dep.copy()
    nodep[::97] = "other"
    nullable = dep.copy()
    nullable[::101] = None
    t = pa.table({"k": pa.array(k, pa.int64()), "dep": pa.array(dep, pa.large_string()),
                  "nodep": pa.array(nodep, pa.large_string()), "nl": pa.array(nullable, pa.large_string()),
                  "v": pa.array(np.ones(n, dtype=np.int64))})
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("t", t)
        res[dev] = [e.query(f"SELECT k, {c}, sum(v) AS s FROM t GROUP BY k, {c} ORDER BY k, {c} NULLS FIRST")
                    .to_pylist() for c in ("dep", "nodep", "nl")]
    assert res["cpu"] == res[gpu_device]
    assert len(res["cpu"][1]) > len(res["cpu"][0]) and len(res["cpu"][2]) > len(res["cpu"][0])


@pytest.mark.parametrize("n", [3_000_000])
def test_sorted_group_ids_and_aggregate(gpu_device, n):
    """Clustered keys take the run-id + register-folding path; results must
    equal the hash path (and the CPU reference)."""
    g = _rng(13)
    k = torch.from_numpy(np.sort(g.integers(0, n // 3, n)).astype(np.int64))
    v = torch.from_numpy(g.integers(-10**12, 10**12, n).astype(np.int64))
    kd, vd = k.to(gpu_device), v.to(gpu_device)
    gid, ng, rep, srt = H.group_ids_ex(kd)
    assert srt and ng == torch.unique(k).numel()
    assert torch.equal(kd.index_select(0, rep.long()), torch.unique(k).to(gpu_device))
    specs = [("sum_int", vd, None), ("count", None, None), ("min_int", vd, None), ("max_int", vd, None)]
    fast = A.grouped_aggregate(gid, ng, specs, n, gpu_device, sorted_gids=True)
    slow = A.grouped_aggregate(gid, ng, specs, n, gpu_device, sorted_gids=False)
    for a_, b_ in zip(fast, slow):
        assert torch.equal(a_.cpu(), b_.cpu())
    # unsorted keys are detected as such
    assert not H.group_ids_ex(kd.flip(0))[3]


@pytest.mark.parametrize("runs", ["ones", "mixed", "long"])
def test_sorted_aggregate_chunked_vs_cpu(gpu_device, runs):
    """agg_sorted_chunk_kernel (8 rows per lane, cross-lane tail chains, atomics
    only at tile edges) against the CPU reference: runs of 1 row, mixed runs,
    and runs longer than a 512-row wave tile; NULLs; n not a tile multiple."""
    g = _rng(17)
    n = 1_000_003
    if runs == "ones":
        k = np.arange(n)
    elif runs == "mixed":
        k = np.sort(g.integers(0, n // 4, n))
    else:
        k = np.repeat(np.arange(n // 1500 + 1), 1500)[:n]
    gid = torch.from_numpy(np.unique(k, return_inverse=True)[1].astype(np.int32))
    ng = int(gid.max()) + 1
    v = torch.from_numpy(g.integers(-10**12, 10**12, n).astype(np.int64))
    f = torch.from_numpy(g.standard_normal(n))
    valid = torch.from_numpy(g.random(n) > 0.2)
    specs = [("sum_int", v, None), ("count", None, valid), ("min_int", v, valid), ("max_int", v, None),
             ("sum_f64", f, valid)]
    ref = A.grouped_aggregate(gid, ng, specs, n, "cpu")
    dspecs = [(op, x.to(gpu_device) if x is not None else None, m.to(gpu_device) if m is not None else None)
              for op, x, m in specs]
    got = A.grouped_aggregate(gid.to(gpu_device), ng, dspecs, n, gpu_device, sorted_gids=True)
    for (op, _, _), r, o in zip(specs, ref, got):
        if op == "sum_f64":
            assert torch.allclose(o.cpu(), r, rtol=1e-9, atol=1e-9)
        else:
            assert torch.equal(o.cpu(), r), op


def test_sorted_ranges_and_expand_vs_torch(gpu_device):
    """ranges.hip: fused lower/upper bound search + load-balanced range expansion
    against torch.searchsorted / repeat_interleave (fp32-free integer oracle)."""
    from igloo_amd.ops import hashing as H
    g = torch.Generator().manual_seed(7)
    for dtype in (torch.int32, torch.int64):
        # runs of 0..40 equal keys (long runs exercise the binary-search upper bound)
        reps = torch.randint(0, 41, (5000,), generator=g)
        big = torch.repeat_interleave(torch.arange(5000, dtype=dtype) * 3, reps)
        q = torch.randint(-5, 15010, (20000,), generator=g).to(dtype)
        qvalid = torch.rand(20000, generator=g) > 0.1
        lo_ref = torch.searchsorted(big, q)
        cnt_ref = torch.where(qvalid, torch.searchsorted(big, q, right=True) - lo_ref, torch.zeros_like(lo_ref))
        lo, cnt = H.sorted_ranges(big.to(gpu_device), q.to(gpu_device), qvalid.to(gpu_device))
        assert torch.equal(cnt.cpu(), cnt_ref)
        assert torch.equal(lo.cpu()[cnt_ref > 0], lo_ref[cnt_ref > 0])
        s, b = H.expand_ranges(lo, cnt, big.numel())
        s_ref, b_ref = H.expand_ranges(lo_ref, cnt_ref, big.numel())
        assert torch.equal(s.cpu().long(), s_ref.long()) and torch.equal(b.cpu().long(), b_ref.long())
        assert torch.equal(big[b.cpu().long()], q[s.cpu().long()])
    # consecutive-output walk: one range spanning many tiles, empty ranges
    # between short ones, a partial last tile (ranges.hip expand_ranges)
    cnt = torch.zeros(30000, dtype=torch.int64)
    cnt[5] = 70001
    cnt[100:20000:3] = torch.randint(1, 9, (len(range(100, 20000, 3)),), generator=g)
    cnt[29999] = 3
    lo = torch.randint(0, 10**6, (30000,), generator=g)
    s, b = H.expand_ranges(lo.to(gpu_device), cnt.to(gpu_device), 2 * 10**6)
    s_ref, b_ref = H.expand_ranges(lo, cnt, 2 * 10**6)
    assert torch.equal(s.cpu().long(), s_ref.long()) and torch.equal(b.cpu().long(), b_ref.long())


def test_sorted_match_pairs_vs_torch(gpu_device):
    """ranges.hip sorted_match: two-key join (first key sorted on the big side,
    second key compared inside each range) against a brute-force CPU oracle."""
    from igloo_amd.ops import hashing as H
    g = torch.Generator().manual_seed(11)
    for dtype in (torch.int32, torch.int64):
        reps = torch.randint(0, 9, (4000,), generator=g)
        big1 = torch.repeat_interleave(torch.arange(4000, dtype=dtype), reps)
        big2 = torch.randint(0, 6, (big1.numel(),), generator=g).to(dtype)
        s1 = torch.randint(-2, 4005, (30000,), generator=g).to(dtype)
        s2 = torch.randint(0, 6, (30000,), generator=g).to(dtype)
        s, b = H.sorted_match_pairs(big1.to(gpu_device), big2.to(gpu_device), s1.to(gpu_device), s2.to(gpu_device))
        s_ref, b_ref = H.sorted_match_pairs(big1, big2, s1, s2)  # CPU path: expand + compare
        assert torch.equal(s.cpu().long(), s_ref.long()) and torch.equal(b.cpu().long(), b_ref.long())
        assert torch.equal(big1[b.cpu().long()], s1[s.cpu().long()])
        assert torch.equal(big2[b.cpu().long()], s2[s.cpu().long()])
        # every true match is found
        want = sum(int(((big1 == s1[i]) & (big2 == s2[i])).sum()) for i in range(0, 30000, 997))
        got = sum(int((s.cpu().long() == i).sum()) for i in range(0, 30000, 997))
        assert got == want


def test_dense_range_index_vs_searchsorted(gpu_device, monkeypatch):
    """ranges.hip dense_index_build/dense_ranges: lower-bound table lookups equal
    torch.searchsorted ranges, including keys outside [min, max], NULL probes and
    long key gaps (suffix-min fix-up path)."""
    from igloo_amd.ops import hashing as H
    monkeypatch.setattr(H, "DENSE_INDEX_MIN_QUERIES", 0)
    g = torch.Generator().manual_seed(5)
    for dtype in (torch.int32, torch.int64):
        for jump in (0, 5000):   # a 5000-key hole > kGapFill: long-gap path
            keys = torch.arange(20000, dtype=dtype) * 2 + 7
            keys[10000:] += jump
            reps = torch.randint(0, 5, (20000,), generator=g)
            big = torch.repeat_interleave(keys, reps)
            q = torch.randint(0, 40000 + jump + 20, (50000,), generator=g).to(dtype)
            qvalid = torch.rand(50000, generator=g) > 0.05
            lo_ref = torch.searchsorted(big, q)
            cnt_ref = torch.where(qvalid, torch.searchsorted(big, q, right=True) - lo_ref, torch.zeros_like(lo_ref))
            bd = big.to(gpu_device)
            lo, cnt = H.sorted_ranges(bd, q.to(gpu_device), qvalid.to(gpu_device))
            assert H.dense_index(bd, build=False) is not None
            assert torch.equal(cnt.cpu(), cnt_ref)
            assert torch.equal(lo.cpu()[cnt_ref > 0], lo_ref[cnt_ref > 0])


def test_key_histogram_and_small_span_group_ids(gpu_device):
    """agg.hip key_histogram (32-bit atomics) vs torch.bincount, and the
    LDS-privatised direct GROUP BY build (span <= 16384) vs the CPU path."""
    g = _rng(23)
    n = 2_000_000
    keys = torch.from_numpy(g.integers(-50, 5000, n).astype(np.int32))
    valid = torch.from_numpy(g.random(n) > 0.3)
    ref = A.key_histogram(keys, 0, 4000, valid)
    got = A.key_histogram(keys.to(gpu_device), 0, 4000, valid.to(gpu_device))
    assert torch.equal(got.cpu(), ref)
    # radix-partitioned path (n >= 2^22, span >= 2^16; span not a bucket multiple)
    n2 = 5_000_000
    for dt, span in ((np.int32, 300_001), (np.int64, 1_500_000)):
        keys2 = torch.from_numpy(g.integers(-1000, span + 1000, n2).astype(dt))
        valid2 = torch.from_numpy(g.random(n2) > 0.1)
        ref2 = A.key_histogram(keys2, 7, span, valid2)
        got2 = A.key_histogram(keys2.to(gpu_device), 7, span, valid2.to(gpu_device))
        assert torch.equal(got2.cpu(), ref2)
        got3 = A.key_histogram(keys2.to(gpu_device), 7, span, None)
        assert torch.equal(got3.cpu(), A.key_histogram(keys2, 7, span, None))
    for span in (5, 700, 16000):
        k = torch.from_numpy(g.integers(100, 100 + span, n).astype(np.int64))
        gid, ng, rep = H.group_ids(k.to(gpu_device))
        assert ng == torch.unique(k).numel()
        kd = k.to(gpu_device)
        # rep is each group's FIRST row and gid maps rows back to it
        assert torch.equal(kd.index_select(0, rep.long()).index_select(0, gid.long()), kd)
        first = {}
        for i, v in enumerate(k[:50000].tolist()):
            first.setdefault(v, i)
        reps = dict(zip(kd.index_select(0, rep.long()).cpu().tolist(), rep.cpu().tolist()))
        for v, i in first.items():
            assert reps[v] == i


@pytest.mark.parametrize("direct", [True, False])
def test_probe_select_vs_probe_first(gpu_device, direct):
    """hashtable.hip probe_hits/probe_write (hit bits per 8192-row tile, then
    ordered writes of hit rows) == probe_first + compaction, for matches and
    misses (anti), with NULL probe keys and a partial last tile."""
    g = _rng(31)
    span = 50_000 if direct else 10**12
    build = torch.from_numpy(np.unique(g.integers(0, span, 20_000)).astype(np.int64)).to(gpu_device)
    m = 1_000_003
    probe = torch.from_numpy(g.integers(0, span if direct else 10**12, m).astype(np.int64))
    probe[::7] = build.cpu()[torch.randint(0, build.numel(), (len(probe[::7]),), generator=torch.Generator().manual_seed(1))]
    pd = probe.to(gpu_device)
    pvalid = torch.from_numpy(g.random(m) > 0.1).to(gpu_device)
    t = H.JoinTable(build)
    assert t.direct == direct and t.unique
    first = t.probe_first(pd, pvalid)
    for negate in (False, True):
        want = mask_to_indices(first < 0 if negate else first >= 0)
        pidx, bidx = t.probe_select(pd, pvalid, negate=negate)
        assert torch.equal(pidx.cpu().long(), want.cpu().long())
        if negate:
            assert bidx is None
        else:
            assert torch.equal(bidx.cpu().long(), first.index_select(0, want.long()).cpu().long())


def test_avg_wide_exact_rounding():
    """util.hip avg_wide: exact decimal AVG of 128-bit (lo, hi) and int64 sums,
    rounded half away from zero, vs Python integers."""
    import random
    import torch
    from igloo_amd.exec.aggregate import _avg
    from igloo_amd import types as T
    rnd = random.Random(7)
    vals = [0, 1, -1, 5, -5, 2**63 - 1, -(2**63), 2**90 + 12345, -(2**95) - 7, 10**30 + 3]
    vals += [rnd.randrange(-(2**100), 2**100) for _ in range(500)]
    cnts = [rnd.randrange(1, 10**9) for _ in vals]
    cnts[0] = 0
    lo = [((v + 2**128) % 2**64) - (2**64 if ((v + 2**128) % 2**64) >= 2**63 else 0) for v in vals]
    hi = [v >> 64 for v in vals]
    s = torch.tensor(list(zip(lo, hi)), dtype=torch.int64, device="cuda:0")
    c = torch.tensor(cnts, dtype=torch.int64, device="cuda:0")
    src, t = T.DECIMAL(15, 2), T.DECIMAL(19, 6)
    got = _avg(s, c, src, t).cpu().tolist()
    up = 10 ** 4
    for v, k, g in zip(vals, cnts, got):
        k = max(k, 1)
        num = v * up
        q = (abs(num) + k // 2) // k
        want = q if num >= 0 else -q
        if -(2**63) <= want < 2**63:
            assert g == want, (v, k, g, want)
    small = torch.tensor([7, -7, 100, -101], dtype=torch.int64, device="cuda:0")
    cs = torch.tensor([2, 2, 3, 3], dtype=torch.int64, device="cuda:0")
    assert _avg(small, cs, src, t).cpu().tolist() == [35000, -35000, 333333, -336667]


def test_sorted_ranges_with_search_fence():
    """ops/hashing.py search_fence + ranges.hip: binary searches over a large
    sorted resident column narrowed through every 256th key give the same
    (lo, cnt) as numpy searchsorted (duplicates, gaps, keys outside the range,
    runs longer than a fence window)."""
    import numpy as np
    import torch
    from igloo_amd.ops import hashing as H
    r = np.random.default_rng(5)
    n = 5_000_000
    k = np.sort(np.concatenate([r.integers(0, 2_000_000, n - 3000), np.full(3000, 777_777)])).astype(np.int32)
    big = torch.from_numpy(k).to("cuda:0")
    big._igloo_resident = True
    big._igloo_dense = False        # no dense table: the fenced binary search
    q = np.concatenate([r.integers(-10, 2_000_010, 200_000), [777_777, k[0], k[-1], -5, 3_000_000]]).astype(np.int32)
    lo, cnt = H.sorted_ranges(big, torch.from_numpy(q).to("cuda:0"))
    assert getattr(big, "_igloo_fence", None) is not None
    want_lo = np.searchsorted(k, q, side="left")
    want_cnt = np.searchsorted(k, q, side="right") - want_lo
    # a resident column without that memo builds its dense lower-bound table
    big2 = torch.from_numpy(k).to("cuda:0")
    big2._igloo_resident = True
    lo2, cnt2 = H.sorted_ranges(big2, torch.from_numpy(q).to("cuda:0"))
    assert getattr(big2, "_igloo_dense", None)
    hit = want_cnt > 0
    assert (cnt2.cpu().numpy() == want_cnt).all() and (lo2.cpu().numpy()[hit] == want_lo[hit]).all()
    got_cnt = cnt.cpu().numpy()
    got_lo = lo.cpu().numpy()
    assert (got_cnt == want_cnt).all()
    hit = want_cnt > 0
    assert (got_lo[hit] == want_lo[hit]).all()


def test_sorted_ranges_sorted_probe_keys(gpu_device, monkeypatch):
    """ranges.hip sorted_ranges, wave-cooperative path: non-decreasing probe keys
    (LDS-staged windows when 64 keys span <= 1024 build rows, windowed global
    searches when they do not), mixed with unsorted and NULL-holding waves,
    with and without the search fence, vs numpy searchsorted."""
    from igloo_amd.ops import hashing as H
    monkeypatch.setattr(H, "DENSE_INDEX", False)
    r = np.random.default_rng(9)
    for dt in (np.int32, np.int64):
        for n, fenced in ((300_000, False), (3_000_000, True)):
            k = np.sort(r.integers(0, n // 3, n)).astype(dt)
            k[n // 2: n // 2 + 5000] = k[n // 2]          # one run longer than a window
            big = torch.from_numpy(k).to(gpu_device)
            if fenced:
                big._igloo_resident = True
            dense = np.sort(r.integers(-5, n // 3 + 5, 100_000))              # windows fit
            sparse = np.sort(r.choice(n // 3 + 10, 20_000, replace=False))    # windows too wide
            shuffled = r.integers(-5, n // 3 + 5, 10_000)
            q = np.concatenate([dense, sparse, shuffled, [k[n // 2]] * 70]).astype(dt)
            for with_valid in (False, True):
                qv = None
                if with_valid:
                    v = np.ones(q.size, bool)
                    v[100_000 + 20_000 + 10_000 - 640: 100_000 + 20_000 + 10_000 - 600] = False
                    v[5000:5003] = False
                    qv = torch.from_numpy(v).to(gpu_device)
                lo, cnt = H.sorted_ranges(big, torch.from_numpy(q).to(gpu_device), qv)
                want_lo = np.searchsorted(k, q, side="left")
                want_cnt = np.searchsorted(k, q, side="right") - want_lo
                if with_valid:
                    want_cnt = np.where(v, want_cnt, 0)
                got_cnt, got_lo = cnt.cpu().numpy(), lo.cpu().numpy()
                assert (got_cnt == want_cnt).all(), (dt, n, with_valid)
                hit = want_cnt > 0
                assert (got_lo[hit] == want_lo[hit]).all(), (dt, n, with_valid)


def test_like_many_tiles_per_workgroup(gpu_device):
    """strings.hip like_seg: more tiles than workgroups (2.5M strings, 9766
    tiles over at most 8192 workgroups), so workgroups run several tiles and
    the next tile's register prefetch is exercised, staged and unstaged."""
    base = _words(20_000, seed=12)
    long_ = [" ".join(["special requests"] * 40)] * 3   # oversized tiles mixed in
    vals = (base * 125)[:2_499_997] + long_
    c = _str_col(vals)
    g = c.to(DEV)
    for pat in ("%special%requests%", "%green", "PROMO%", "%requests"):
        assert torch.equal(S.like(c, pat), S.like(g, pat).cpu()), pat


@pytest.mark.parametrize("words", [(1, 4), (4, 9), (8, 20)])
def test_like_tile_shapes(gpu_device, words):
    """like_seg over short, medium and long strings against the CPU matcher
    (LDS-staged tiles of strings; long strings fall back to direct reads)."""
    r = _rng(21)
    lo, hi = words
    vals = [" ".join(r.choice(WORDS, r.integers(lo, hi))) for _ in range(60_000)]
    c = _str_col(vals)
    g = c.to(DEV)
    for pat in ("%special%requests%", "%Customer%Complaints%", "forest%", "%BRASS", "%e%e%e%"):
        assert torch.equal(S.like(c, pat), S.like(g, pat).cpu()), pat
        assert torch.equal(S.like(c, pat, negate=True), S.like(g, pat, negate=True).cpu()), pat


def test_like_dword_filter_every_alignment(gpu_device, monkeypatch):
    """strings.hip like_dword_kernel (segments of >= 7 bytes: the aligned-dword
    prefilter) against the CPU matcher and the byte-window kernel it replaces:
    planted segments at every offset mod 16, near-misses sharing 4-byte
    windows, overlapping repeats, hits at string ends and in oversized tiles."""
    from igloo_amd.ops._lib import KERNEL_CALLS
    r = _rng(33)
    pieces = ["special", "requests", "specia", "pecial", "requestsrequests", "spespecial", "reques", "quests",
              "Customer", "Complaints", "x", "yy", "zzz", "ünï"]
    vals = []
    for i in range(40_000):
        pad = "." * int(r.integers(0, 16))
        body = "".join(r.choice(pieces, int(r.integers(0, 6))))
        vals.append(pad + body + ("." * int(r.integers(0, 3))))
    vals += ["special requests " * 200]          # one oversized tile
    c = _str_col(vals)
    g = c.to(DEV)
    for pat in ("%special%requests%", "%Customer%Complaints%", "%requests", "special%", "%pecial%", "special",
                "%requestsrequests%", "%special%special%"):
        ref = S.like(c, pat)
        before = KERNEL_CALLS["str_like_segments"]
        monkeypatch.delenv("IGLOO_DEBUG", raising=False)
        got = S.like(g, pat).cpu()
        monkeypatch.setenv("IGLOO_DEBUG", "like_nodword")
        old = S.like(g, pat).cpu()
        assert KERNEL_CALLS["str_like_segments"] == before + 2
        assert torch.equal(ref, got), pat
        assert torch.equal(ref, old), pat
        assert int(ref.sum()) > 0, pat


@pytest.mark.parametrize("ncols", [2, 3, 8])
def test_pack_keys_native(gpu_device, ncols):
    """csrc/kernels/util.hip pack_bits vs the plain int64 shift/OR formula."""
    g = torch.Generator().manual_seed(ncols)
    n = 100_003
    cols = []
    for c in range(ncols):
        lo = int(torch.randint(-1000, 1000, (1,), generator=g))
        hi = lo + int(torch.randint(1, 200, (1,), generator=g))
        dt = torch.int32 if c % 2 == 0 else torch.int64
        cols.append(torch.randint(lo, hi, (n,), generator=g).to(dt))
    ref_ranges = [(int(c.min()), int(c.max())) for c in cols]
    bits = [max(1, (hi - lo).bit_length()) for lo, hi in ref_ranges]
    ref = None
    for c, (lo, _), b in zip(cols, ref_ranges, bits):
        v = c.to(torch.int64) - lo
        ref = v if ref is None else (ref << b) | v
    got = H.pack_keys([c.to(DEV) for c in cols]).cpu()
    assert torch.equal(got, ref)
    # pair packing: one shared layout, both sides packed separately
    left = [c[: n // 3].to(DEV) for c in cols]
    right = [c[n // 3:].to(DEV) for c in cols]
    pl, pr = H.pack_keys_pair(left, right)
    assert torch.equal(torch.cat([pl, pr]).cpu(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("density", [0.0, 0.003, 0.3, 0.97, 1.0])
def test_compact_columns_matches_gather(gpu_device, density):
    """Fused mask compaction (select.hip tile_compact) of fixed-width columns
    of every width, with validity, dictionary codes and a plain-string
    column, equals mask -> indices -> gather."""
    import torch
    from igloo_amd import types as T
    from igloo_amd.columnar import Column
    from igloo_amd.ops.gather import take_many
    from igloo_amd.ops.select import compact_columns, mask_to_indices
    g = torch.Generator().manual_seed(3)
    n = 70_001
    m = (torch.rand(n, generator=g) < density).to(gpu_device)
    cols = [Column(T.INT8, torch.randint(-100, 100, (n,), generator=g, dtype=torch.int8).to(gpu_device)),
            Column(T.INT16, torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int16).to(gpu_device)),
            Column(T.INT32, torch.randint(0, 1 << 30, (n,), generator=g, dtype=torch.int32).to(gpu_device),
                   (torch.rand(n, generator=g) > 0.2).to(gpu_device)),
            Column(T.FLOAT64, torch.rand(n, generator=g, dtype=torch.float64).to(gpu_device)),
            Column(T.DECIMAL(30, 2), torch.randint(-2**40, 2**40, (n, 2), generator=g).to(gpu_device)),
            Column.from_values([f"s{i % 977}" for i in range(n)], T.UTF8, gpu_device)]
    cols = cols * 3          # 18 columns: two fused launches
    idx, got = compact_columns(m, cols)
    ref_idx = mask_to_indices(m)
    assert torch.equal(idx.cpu().long(), ref_idx.cpu().long())
    for a, b in zip(got, take_many(cols, ref_idx)):
        assert a.to_arrow().equals(b.to_arrow())


@pytest.mark.parametrize("prefix", [None, 2, 3])
def test_str_in_set(gpu_device, prefix):
    """One-pass string IN list (strings.hip in_set_kernel), plain and as
    substr(s, 1, L) IN (...), against the host evaluation."""
    g = _rng(11)
    words = ["13", "31", "1", "", "133", "ab", "aé", "ééx", "zz", "13x"]
    vals = [words[i] for i in g.integers(0, len(words), 5000)] + ["13-555", "31", "aéb"]
    arr = pa.array(vals, pa.large_string())
    col = Column.from_arrow(arr, device=DEV, dict_encode=False)
    consts = ["13", "31", "aé", "éé", "x"]
    got = S.in_set(col, consts, prefix_chars=prefix).cpu().tolist()
    if prefix is None:
        want = [v in consts for v in vals]
    else:
        want = [v[:prefix] in consts for v in vals]
    assert got == want
    # an empty constant and one past 8 bytes (the byte-compare path)
    for consts in (["", "13", "ab"], ["13", "aéb", "0123456789"]):
        got = S.in_set(col, consts, prefix_chars=prefix).cpu().tolist()
        want = [(v if prefix is None else v[:prefix]) in consts for v in vals]
        assert got == want, consts
