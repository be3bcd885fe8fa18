"""Radix sort / top-k kernels (csrc/kernels/sort.hip) against a numpy oracle.

ORDER BY semantics follow the reference's tests: ``ORDER BY ... ASC NULLS
FIRST`` (reference crates/engine/src/lib.rs:186-231) and ``ORDER BY age``
(crates/engine/tests/integration_test.rs:59). The oracle is a stable numpy
lexsort over (NULL flag, value) per column, NULLs tied with each other."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from igloo_amd.ops import _lib
from igloo_amd.ops import sort as SO

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def oracle(cols, n):
    """cols: [(np values, desc, nulls_first, np valid or None)] most significant first."""
    keys = []
    for v, desc, nf, valid in reversed(cols):   # np.lexsort: last key is primary
        v = v.astype(np.float64) if v.dtype.kind == "f" else v.astype(np.int64)
        if valid is not None:
            v = np.where(valid, v, 0)
        if desc:
            # order-reversing transform that keeps ties tied
            _, inv = np.unique(v, return_inverse=True)
            v = -inv
        keys.append(v)
        if valid is not None:
            keys.append(np.where(valid, 1, 0) if nf else np.where(valid, 0, 1))
    if not keys:
        return np.arange(n)
    return np.lexsort(keys)


def _to_dev(cols):
    out = []
    for v, desc, nf, valid in cols:
        out.append((torch.from_numpy(v).to(DEV), desc, nf, None if valid is None else torch.from_numpy(valid).to(DEV)))
    return out


DTYPES = [np.int8, np.int16, np.int32, np.int64, np.float64, np.float32, np.bool_]


def _col(rng, n, dtype, lo, hi, nulls):
    if dtype == np.bool_:
        v = rng.integers(0, 2, n).astype(np.bool_)
    elif np.dtype(dtype).kind == "f":
        v = rng.normal(0, 10 ** rng.integers(0, 6), n).astype(dtype)
        v[rng.random(n) < 0.1] = 0.0
        if n > 3:
            v[1] = -0.0
    else:
        info = np.iinfo(dtype)
        v = rng.integers(max(lo, info.min), min(hi, info.max), n, endpoint=True).astype(dtype)
    valid = (rng.random(n) > 0.2) if nulls else None
    return v, valid


@pytest.mark.parametrize("n", [0, 1, 7, 100, 4096, 4097, 70_000, 1_000_003])
@pytest.mark.parametrize("case", range(4))
def test_argsort_matches_numpy(gpu_device, n, case):
    rng = np.random.default_rng(1000 * case + n % 997)
    ncols = 1 + case % 3
    cols = []
    for c in range(ncols):
        dt = DTYPES[(case * 3 + c) % len(DTYPES)]
        lo, hi = [(0, 5), (-100, 100), (-2**40, 2**40), (-2**63, 2**63 - 1)][(case + c) % 4]
        v, valid = _col(rng, n, dt, lo, hi, nulls=(case + c) % 2 == 1)
        cols.append((v, bool((case + c) % 2), bool(c % 2), valid))
    perm = SO.argsort(_to_dev(cols), n, DEV).cpu().numpy()
    np.testing.assert_array_equal(perm, oracle(cols, n))


def test_wide_keys_split_into_groups(gpu_device):
    rng = np.random.default_rng(5)
    n = 50_000
    cols = [(rng.integers(-2**62, 2**62, n), False, True, None),
            (rng.integers(-2**62, 2**62, n), True, True, rng.random(n) > 0.5),
            (rng.integers(0, 3, n).astype(np.int32), False, False, None)]
    cols[0][0][::7] = 12345     # ties on the leading key
    perm = SO.argsort(_to_dev(cols), n, DEV).cpu().numpy()
    np.testing.assert_array_equal(perm, oracle(cols, n))


@pytest.mark.parametrize("n,k", [(5000, 1), (100_000, 10), (1_000_000, 100), (3_000_000, 20), (200_000, 5000),
                                 (500_000, 17)])
def test_topk_equals_sorted_prefix(gpu_device, n, k):
    rng = np.random.default_rng(n + k)
    cols = [(rng.integers(0, 1000, n).astype(np.int64), True, False, None),     # heavy ties
            (rng.normal(0, 1e6, n), False, False, None)]
    _lib.KERNEL_CALLS.clear()
    got = SO.topk(_to_dev(cols), n, k, DEV).cpu().numpy()
    np.testing.assert_array_equal(got, oracle(cols, n)[:k])
    assert _lib.KERNEL_CALLS["radix_select"] > 0 and _lib.KERNEL_CALLS["radix_sort"] > 0


def test_topk_skewed_single_value(gpu_device):
    n = 300_000
    v = np.zeros(n, np.int64)
    v[-5:] = -1
    got = SO.topk(_to_dev([(v, False, False, None)]), n, 10, DEV).cpu().numpy()
    np.testing.assert_array_equal(got, oracle([(v, False, False, None)], n)[:10])


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(data=st.lists(st.one_of(st.none(), st.integers(-2**31, 2**31 - 1)), min_size=0, max_size=6000),
       desc=st.booleans(), nf=st.booleans())
def test_hypothesis_nullable_int32(gpu_device, data, desc, nf):
    n = len(data)
    v = np.array([0 if x is None else x for x in data], np.int32)
    valid = np.array([x is not None for x in data], np.bool_)
    cols = [(v, desc, nf, valid)]
    perm = SO.argsort(_to_dev(cols), n, DEV).cpu().numpy()
    np.testing.assert_array_equal(perm, oracle(cols, n))


@pytest.mark.parametrize("n", [10, 5000, 2_000_000])
def test_perm_index_sort(gpu_device, n):
    rng = np.random.default_rng(n)
    k = rng.integers(1, 200_000, n).astype(np.int32)
    sk, perm = SO.perm_sort_int(torch.from_numpy(k).to(DEV))
    ref = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(perm.cpu().numpy(), ref)
    np.testing.assert_array_equal(sk.cpu().numpy(), k[ref])


def test_order_by_nulls_first_sql(gpu_device):
    """Reference test_capitalize_udf ordering on the GPU path."""
    import pyarrow as pa
    import igloo_amd as ig
    e = ig.QueryEngine(device=DEV)
    e.register_table("t", pa.table({"s": pa.array(["hello", "WoRlD", None, "rust", ""]),
                                    "k": pa.array([3, None, 1, 2, 5], pa.int64())}))
    r = e.sql("SELECT capitalize(s) AS c FROM t ORDER BY c ASC NULLS FIRST").table
    assert r.column("c").to_pylist() == [None, "", "HELLO", "RUST", "WORLD"]
    r = e.sql("SELECT k FROM t ORDER BY k DESC NULLS LAST LIMIT 3").table
    assert r.column("k").to_pylist() == [5, 3, 2]


@pytest.mark.parametrize("n", [0, 1, 9, 4096, 1_000_001, 20_000_003])
@pytest.mark.parametrize("dtype", [torch.int32, torch.int64])
def test_column_stats_and_run_bounds(gpu_device, n, dtype):
    from igloo_amd.ops import hashing as H
    g = torch.Generator().manual_seed(n)
    x = torch.randint(-10**6, 10**6, (n,), generator=g).to(dtype)
    valid = torch.rand(n, generator=g) > 0.3
    for v in (None, valid):
        rng, srt = H.column_stats(x.to(DEV), None if v is None else v.to(DEV))
        sel = x if v is None else x[v]
        if sel.numel():
            assert rng == (int(sel.min()), int(sel.max()))
        else:
            assert rng is None
        if v is None:
            assert srt == (n < 2 or bool((x[1:] >= x[:-1]).all()))
    s = torch.sort(x).values
    assert H.column_stats(s.to(DEV))[1] is True
    if n > 40:
        # one inversion exactly at a lane-run boundary (16 int32 / 8 int64 rows), and a
        # misaligned start (vector loads need 16-byte alignment: scalar path)
        run = 16 if dtype == torch.int32 else 8
        t = s.clone()
        t[run], t[run - 1] = s[run - 1] - 1, s[run - 1]
        assert H.column_stats(t.to(DEV))[1] is False
        sub = s.to(DEV)[1:]
        assert H.column_stats(sub) == ((int(s[1:].min()), int(s[1:].max())), True)
    if n > 1:
        bound = torch.empty(n, dtype=torch.bool, device=DEV)
        _lib.native().run_bounds(s.to(DEV).data_ptr(), dtype == torch.int64, n, bound.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
        ref = torch.ones(n, dtype=torch.bool)
        ref[1:] = s[1:] != s[:-1]
        assert torch.equal(bound.cpu(), ref)


def test_device_string_ranks_match_arrow_order():
    """ops/strings.py _device_ranks (8-byte big-endian chunks + LSD radix
    argsort) orders a plain-string dictionary exactly like Arrow's byte-wise
    UTF-8 sort: shared prefixes, empty strings, prefixes of each other,
    multi-byte characters, lengths across several chunks."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.compute as pc
    import torch
    from igloo_amd.columnar import Column
    from igloo_amd.ops import strings as S
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = np.random.default_rng(3)
    alphabet = list("abcAB z09") + ["é", "ß", "日"]
    vals = {"", "a", "ab", "abcdefgh", "abcdefghi", "abcdefgh\x01", "Customer#000000001", "Customer#000000010"}
    while len(vals) < 3000:
        vals.add("".join(r.choice(alphabet, size=int(r.integers(0, 30)))))
    vals = list(vals)
    r.shuffle(vals)
    d = Column.from_arrow(pa.array(vals, pa.large_string()), device="cuda:0", dict_encode=False)
    got = S._device_ranks(d).cpu().numpy()
    order = pc.array_sort_indices(pa.array(vals, pa.large_string())).to_numpy()
    want = np.empty(len(vals), dtype=np.int64)
    want[order] = np.arange(len(vals))
    assert (got == want).all()


@pytest.mark.parametrize("n", [2, 37, 256, 511, 512, 513, 1000, 4095, 4096])
@pytest.mark.parametrize("kdt,bits", [(torch.int64, 64), (torch.int64, 40), (torch.int32, 32), (torch.int32, 12)])
def test_small_sort_pairs_stable(gpu_device, n, kdt, bits):
    """One-workgroup sorts (sort.hip rs_small_kernel): the rank sort up to
    512 rows, radix passes over only the digits that vary above it; stable,
    bits outside [begin_bit, end_bit) ignored. Oracle: numpy stable argsort."""
    rng = np.random.default_rng(n * 7 + bits)
    width = 64 if kdt == torch.int64 else 32
    lo_bits = 4
    # few distinct values in the sorted range (ties exercise stability), noise
    # in the bits below begin_bit and constant high digits (skipped passes)
    v = rng.integers(0, max(2, n // 3), n).astype(np.uint64) << np.uint64(lo_bits)
    v |= rng.integers(0, 1 << lo_bits, n).astype(np.uint64)
    if bits < width:
        v &= np.uint64((1 << bits) - 1)
    else:
        v |= np.uint64(0x7000000000000000 if width == 64 else 0)
    if width == 32:
        v &= np.uint64(0xFFFFFFFF)
    keys_np = v.astype(np.uint64).view(np.int64) if width == 64 else v.astype(np.uint32).view(np.int32)
    vals_np = np.arange(n, dtype=np.int32)
    k, vv = SO.sort_pairs(torch.from_numpy(keys_np.copy()).to(DEV), torch.from_numpy(vals_np).to(DEV), bits,
                          begin_bit=lo_bits)
    masked = (v >> np.uint64(lo_bits)).astype(np.uint64)
    want = np.argsort(masked, kind="stable")
    assert np.array_equal(vv.cpu().numpy(), vals_np[want])
    assert np.array_equal(k.cpu().numpy(), keys_np[want])
