"""GPU Parquet page decode (csrc/kernels/parquet.hip) vs pyarrow's decoder.

Every case writes a file with pyarrow (the oracle reads it back with
pyarrow's CPU decoder) and decodes it with ``GpuParquetReader``: snappy,
ZSTD (csrc/kernels/zstd.hip) and uncompressed, data page v1 and v2,
dictionary, plain, DELTA_BINARY_PACKED, DELTA_LENGTH_BYTE_ARRAY and
BYTE_STREAM_SPLIT encodings, NULLs, multiple row groups and many small
pages, every physical type the engine maps (INT32/INT64/FLOAT/DOUBLE/
BOOLEAN/FLBA decimal/BYTE_ARRAY), and a ZSTD Iceberg table end to end.
"""
import decimal

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from igloo_amd import types as T
from igloo_amd.columnar import Column
from igloo_amd.connectors.gpu_parquet import GpuParquetReader
from igloo_amd.ops._lib import KERNEL_CALLS

pytestmark = pytest.mark.gpu


def _table(n, seed=0, nulls=True):
    rng = np.random.default_rng(seed)

    def maybe_null(vals):
        if not nulls:
            return vals
        return [None if (i * 7919) % 13 == 0 else v for i, v in enumerate(vals)]

    words = ["alpha", "beta", "gamma", "delta", "epsilon", "", "zeta-" * 9]
    return pa.table({
        "i32": pa.array(maybe_null(rng.integers(-2**31, 2**31 - 1, n).tolist()), pa.int32()),
        "i64": pa.array(maybe_null(rng.integers(-2**62, 2**62, n).tolist()), pa.int64()),
        "f32": pa.array(rng.standard_normal(n).astype(np.float32)),
        "f64": pa.array(maybe_null(rng.standard_normal(n).tolist()), pa.float64()),
        "dec": pa.array(maybe_null([decimal.Decimal(int(x)).scaleb(-2) for x in rng.integers(-10**13, 10**13, n)]),
                        pa.decimal128(15, 2)),
        "dec38": pa.array([decimal.Decimal(int(x)).scaleb(-4) for x in rng.integers(-10**15, 10**15, n)],
                          pa.decimal128(38, 4)),
        "d": pa.array(rng.integers(0, 20000, n).astype(np.int32), pa.int32()).cast(pa.date32()),
        "b": pa.array(maybe_null(rng.integers(0, 2, n).astype(bool).tolist()), pa.bool_()),
        "low": pa.array(maybe_null([words[int(x)] for x in rng.integers(0, len(words), n)]), pa.string()),
        "high": pa.array(maybe_null([f"row-{int(x)}-{'x' * int(x % 37)}" for x in rng.integers(0, 10**9, n)]),
                         pa.string()),
        "i16": pa.array(rng.integers(-30000, 30000, n).astype(np.int16)),
        "u32": pa.array(rng.integers(0, 2**32 - 1, n).astype(np.uint32)),
        "ts": pa.array(rng.integers(0, 2**40, n), pa.timestamp("ms")),
    })


def _check(path, t, device):
    r = GpuParquetReader([path])
    schema = pq.read_schema(path)
    cols = [(f.name, T.from_arrow_type(f.type)) for f in schema]
    groups = [(0, g) for g in range(len(r.metas[0].row_groups))]
    got, rejected = r.read(cols, groups, device)
    assert not rejected, rejected
    for name, dt in cols:
        want = Column.from_arrow(t.column(name), device="cpu", dtype=dt).to_arrow()
        have = got[name].to_arrow()
        assert have.type == want.type or have.cast(want.type).type == want.type, (name, have.type, want.type)
        if have.type != want.type:
            have = have.cast(want.type)
        assert have.to_pylist() == want.to_pylist(), name


@pytest.mark.parametrize("compression", ["none", "snappy", "zstd"])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("dictionary", [True, False])
def test_decode_matches_pyarrow(tmp_path, gpu_device, compression, version, dictionary):
    t = _table(30000, seed=sum(map(ord, compression + version)) + int(dictionary))
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=11000, compression=compression, data_page_version=version,
                   use_dictionary=dictionary, data_page_size=16384)
    before = KERNEL_CALLS["pq_decode"]
    _check(path, t, gpu_device)
    assert KERNEL_CALLS["pq_decode"] > before
    if compression == "snappy":
        assert KERNEL_CALLS["pq_snappy"] > 0
    if compression == "zstd":
        assert KERNEL_CALLS["pq_zstd"] > 0


@pytest.mark.parametrize("compression", ["none", "zstd"])
@pytest.mark.parametrize("version", ["1.0", "2.0"])
def test_delta_and_byte_stream_split(tmp_path, gpu_device, compression, version):
    rng = np.random.default_rng(17)
    n = 50000

    def nul(vals, every=11):
        return [None if i % every == 3 else v for i, v in enumerate(vals)]

    ext = [-2**31, 2**31 - 1, 0, -1]
    t = pa.table({
        "a32": pa.array(nul(ext + rng.integers(-2**31, 2**31 - 1, n - 4).tolist()), pa.int32()),
        "a64": pa.array(nul([-2**63, 2**63 - 1] + rng.integers(-2**63, 2**63 - 1, n - 2, dtype=np.int64).tolist()),
                        pa.int64()),
        "seq": pa.array(np.arange(n, dtype=np.int64) * 3 - 7),              # small deltas, bit width 0
        "slow": pa.array(np.repeat(np.arange(n // 100, dtype=np.int32), 100)),
        "s": pa.array(nul([("" if i % 17 == 0 else f"v{i % 977}-" + "x" * (i % 41)) for i in range(n)], 7),
                      pa.string()),
        "f": pa.array(nul(rng.standard_normal(n).tolist(), 5), pa.float64()),
        "g": pa.array(rng.standard_normal(n).astype(np.float32)),
    })
    enc = {"a32": "DELTA_BINARY_PACKED", "a64": "DELTA_BINARY_PACKED", "seq": "DELTA_BINARY_PACKED",
           "slow": "DELTA_BINARY_PACKED", "s": "DELTA_LENGTH_BYTE_ARRAY", "f": "BYTE_STREAM_SPLIT",
           "g": "BYTE_STREAM_SPLIT"}
    path = str(tmp_path / "d.parquet")
    pq.write_table(t, path, compression=compression, use_dictionary=False, column_encoding=enc,
                   data_page_version=version, row_group_size=20000, data_page_size=8192)
    md = pq.ParquetFile(path).metadata
    for i, name in enumerate(t.column_names):
        assert enc[name] in md.row_group(0).column(i).encodings, name
    before = KERNEL_CALLS["pq_zstd"]
    _check(path, t, gpu_device)
    assert (KERNEL_CALLS["pq_zstd"] > before) == (compression == "zstd")


def test_zstd_iceberg_table_on_gpu(tmp_path, gpu_device):
    """A ZSTD-written Iceberg table (the default codec of Iceberg's writer)
    scans with every column decoded on the GPU: no host fallback."""
    import igloo_amd as ig
    from igloo_amd.connectors import iceberg
    t = _table(40000, seed=9)
    root = str(tmp_path / "ice")
    iceberg.write_table(root, t, rows_per_file=15000)
    e = ig.QueryEngine(device=gpu_device)
    src = e.register_iceberg("ice", root)
    before = KERNEL_CALLS["pq_zstd"]
    got = e.query("select count(*) c, sum(i32) s, count(high) h, max(low) l, sum(f64) f from ice").to_pylist()[0]
    assert KERNEL_CALLS["pq_zstd"] > before
    assert src._inner.last_gpu_stats and not src._inner.last_gpu_stats["host_columns"]
    assert got["c"] == t.num_rows
    assert got["s"] == sum(v for v in t.column("i32").to_pylist() if v is not None)
    assert got["h"] == t.column("high").null_count * -1 + t.num_rows
    assert got["l"] == max(v for v in t.column("low").to_pylist() if v is not None)
    assert abs(got["f"] - sum(v for v in t.column("f64").to_pylist() if v is not None)) < 1e-6


def test_no_nulls_large_pages(tmp_path, gpu_device):
    t = _table(300000, seed=3, nulls=False)
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=120000, compression="snappy")
    _check(path, t, gpu_device)


def test_dictionary_output_and_fallback_pages(tmp_path, gpu_device):
    # a low-cardinality column stays dictionary-encoded; a column whose dictionary
    # overflows the writer's limit mixes dictionary and plain pages
    n = 200000
    t = pa.table({"k": pa.array([f"key{i % 11}" for i in range(n)]),
                  "u": pa.array([f"unique-value-{i:08d}" for i in range(n)])})
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=70000, dictionary_pagesize_limit=64 << 10)
    r = GpuParquetReader([path])
    got, rej = r.read([("k", T.UTF8), ("u", T.UTF8)], [(0, g) for g in range(3)], gpu_device)
    assert not rej
    assert got["k"].is_dict and len(got["k"].dictionary) == 11
    assert got["k"].to_arrow().to_pylist() == t.column("k").to_pylist()
    assert got["u"].to_arrow().to_pylist() == t.column("u").to_pylist()


def test_row_group_subset_and_multi_file(tmp_path, gpu_device):
    t1 = _table(9000, seed=5)
    t2 = _table(7000, seed=6)
    p1, p2 = str(tmp_path / "a.parquet"), str(tmp_path / "b.parquet")
    pq.write_table(t1, p1, row_group_size=3000)
    pq.write_table(t2, p2, row_group_size=3500, compression="none")
    r = GpuParquetReader([p1, p2])
    groups = [(0, 1), (1, 0), (1, 1)]
    got, rej = r.read([("i64", T.INT64), ("low", T.UTF8), ("dec", T.DECIMAL(15, 2))], groups, gpu_device)
    assert not rej
    want = pa.concat_tables([t1.slice(3000, 3000), t2])
    assert got["i64"].to_arrow().to_pylist() == want.column("i64").to_pylist()
    assert got["low"].to_arrow().to_pylist() == want.column("low").to_pylist()
    assert [None if v is None else str(v) for v in got["dec"].to_arrow().to_pylist()] == \
        [None if v is None else str(v) for v in want.column("dec").to_pylist()]


def test_engine_query_over_gpu_parquet(tmp_path, gpu_device):
    """TPC-H Q1/Q6 over Parquet files decoded on the GPU == the same data in memory."""
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    mem = ig.QueryEngine(device=gpu_device)
    tabs = datagen.register(mem, 0.05)
    li = datagen.to_arrow({"lineitem": tabs["lineitem"]})["lineitem"]
    pq.write_table(li, tmp_path / "lineitem.parquet", row_group_size=100000, compression="snappy")
    e = ig.QueryEngine(device=gpu_device)
    src = e.register_parquet("lineitem", str(tmp_path / "lineitem.parquet"))
    for q in (1, 6):
        a = e.query(queries.QUERIES[q])
        b = mem.query(queries.QUERIES[q])
        assert a.to_pylist() == b.to_pylist(), q
    assert src.last_gpu_stats and not src.last_gpu_stats["host_columns"]


def test_snappy_far_matches_beyond_lds_ring(tmp_path, gpu_device):
    """Pages whose snappy stream copies from 16-60 KiB back (beyond the
    kernel's LDS history ring): repeated 20-40 KB random blocks."""
    rng = np.random.default_rng(7)
    blocks = [bytes(rng.integers(97, 123, int(sz), dtype=np.uint8)) for sz in (20_000, 33_000, 41_000)]
    vals = []
    for i in range(60):
        b = blocks[i % 3]
        vals.append(b.decode() + f"-{i}")
    t = pa.table({"s": pa.array(vals, pa.string()),
                  "k": pa.array(np.tile(rng.integers(0, 2**40, 4096), 3), pa.int64())[:60]})
    path = str(tmp_path / "far.parquet")
    pq.write_table(t, path, compression="snappy", use_dictionary=False, data_page_size=1 << 20)
    _check(path, t, gpu_device)


def _uleb(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def test_corrupt_delta_header_is_rejected(tmp_path, gpu_device):
    """A DELTA_BINARY_PACKED header with more miniblocks than values per block
    (values per miniblock 0, which passed the old ``% 32`` check and spun or
    read past the page) must fail the scan cleanly. The header is rewritten in
    place: the first value's varint is shortened by one byte to make room for
    a two-byte miniblock count, so the page keeps its length."""
    from igloo_amd.utils.errors import ExecutionError
    n = 5000
    first = 2**40
    t = pa.table({"a": pa.array([first] + list(range(n - 1)), pa.int64())})
    path = str(tmp_path / "c.parquet")
    pq.write_table(t, path, compression="none", use_dictionary=False, column_encoding={"a": "DELTA_BINARY_PACKED"},
                   data_page_version="1.0")
    raw = bytearray(open(path, "rb").read())
    zz = first << 1
    hdr = _uleb(256) + b"\x04" + _uleb(n) + _uleb(zz)          # pyarrow: 256-value blocks, 4 miniblocks
    assert raw.count(hdr) == 1
    bad = _uleb(256) + _uleb(257) + _uleb(n) + _uleb(zz >> 7)   # 257 miniblocks in a 256-value block
    assert len(bad) == len(hdr)
    raw[raw.index(hdr):raw.index(hdr) + len(hdr)] = bad
    open(path, "wb").write(bytes(raw))
    r = GpuParquetReader([path])
    with pytest.raises(ExecutionError):
        r.read([("a", T.INT64)], [(0, 0)], gpu_device)


def test_pipelined_batches(tmp_path, gpu_device, monkeypatch):
    """Many small batches: positional reads run ahead on the read thread
    (READ_AHEAD batches) while earlier batches decode; results unchanged."""
    from igloo_amd.connectors import gpu_parquet as G
    monkeypatch.setattr(G, "BATCH_BYTES", 64 << 10)
    t = _table(40000, seed=99)
    path = str(tmp_path / "p.parquet")
    pq.write_table(t, path, row_group_size=9000, compression="snappy", data_page_size=8192)
    w0 = G.TOTALS["read_wait_s"]
    _check(path, t, gpu_device)
    r = GpuParquetReader([path])
    r.read([(f.name, T.from_arrow_type(f.type)) for f in pq.read_schema(path)],
           [(0, g) for g in range(len(r.metas[0].row_groups))], gpu_device)
    assert r.last_stats["batches"] > 3, r.last_stats
    assert G.TOTALS["read_wait_s"] >= w0
