"""Native Parquet metadata path (CPU): the C++ Thrift footer / page-header
decoder and page planner (csrc/io/parquet_meta.cpp) checked against pyarrow's
own view of the same files. The GPU page decode is covered by
tests/test_parquet_gpu.py."""
import decimal
import struct

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from igloo_amd import types as T
from igloo_amd.connectors.gpu_parquet import PHYS, FileMeta, GpuParquetReader
from igloo_amd.ops._lib import native
from igloo_amd.utils.errors import IoError


def _table(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    return pa.table({
        "i32": pa.array(rng.integers(-1000, 1000, n).astype(np.int32), pa.int32()),
        "i64": pa.array(rng.integers(-2**40, 2**40, n), pa.int64()),
        "f64": pa.array(rng.standard_normal(n), pa.float64()),
        "dec": pa.array([decimal.Decimal(int(x)).scaleb(-2) for x in rng.integers(-10**9, 10**9, n)],
                        pa.decimal128(15, 2)),
        "d": pa.array(rng.integers(8000, 11000, n).astype(np.int32), pa.int32()).cast(pa.date32()),
        "s": pa.array([f"str{int(x)}" for x in rng.integers(0, 50, n)], pa.string()),
        "b": pa.array(rng.integers(0, 2, n).astype(bool)),
        "nul": pa.array([None if x % 7 == 0 else int(x) for x in range(n)], pa.int64()),
    })


def test_footer_matches_pyarrow(tmp_path):
    t = _table()
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=1500, compression="snappy")
    ref = pq.ParquetFile(path).metadata
    m = FileMeta(path)
    assert m.num_rows == ref.num_rows == t.num_rows
    assert [l["name"] for l in m.leaves] == t.column_names
    assert len(m.row_groups) == ref.num_row_groups == 4
    for gi, g in enumerate(m.row_groups):
        rg = ref.row_group(gi)
        assert g["num_rows"] == rg.num_rows
        for ci, c in enumerate(g["chunks"]):
            rc = rg.column(ci)
            assert c["num_values"] == rc.num_values
            assert c["length"] == rc.total_compressed_size
            start = rc.dictionary_page_offset if rc.has_dictionary_page else rc.data_page_offset
            assert c["start"] == start
            assert c["codec"] == 1  # SNAPPY
    phys = {l["name"]: l["type"] for l in m.leaves}
    assert phys["i32"] == PHYS["INT32"] and phys["i64"] == PHYS["INT64"] and phys["s"] == PHYS["BYTE_ARRAY"]
    assert phys["dec"] == PHYS["FLBA"] and phys["b"] == PHYS["BOOLEAN"] and phys["f64"] == PHYS["DOUBLE"]
    leaf = {l["name"]: l for l in m.leaves}
    assert leaf["dec"]["logical"] == "decimal" and leaf["dec"]["scale"] == 2 and leaf["dec"]["precision"] == 15
    assert leaf["d"]["logical"] == "date" and leaf["s"]["logical"] == "string"
    assert all(l["max_def"] == 1 and l["max_rep"] == 0 for l in m.leaves)


def test_statistics_min_max(tmp_path):
    t = _table()
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=2000)
    m = FileMeta(path)
    ref = pq.ParquetFile(path).metadata
    ci = m.leaf_index["i32"]
    for gi, g in enumerate(m.row_groups):
        c = g["chunks"][ci]
        st = ref.row_group(gi).column(ci).statistics
        assert struct.unpack("<i", c["min"])[0] == st.min
        assert struct.unpack("<i", c["max"])[0] == st.max
        assert c["null_count"] == st.null_count == 0
    cn = m.leaf_index["nul"]
    assert sum(g["chunks"][cn]["null_count"] for g in m.row_groups) == t.column("nul").null_count


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("compression", ["none", "snappy", "zstd"])
def test_page_headers_and_plan(tmp_path, version, compression):
    t = _table(20000)
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, row_group_size=8000, compression=compression, data_page_version=version,
                   data_page_size=4096)
    m = FileMeta(path)
    N = native()
    for name in ("i32", "s", "nul", "dec"):
        li = m.leaf_index[name]
        leaf = m.leaves[li]
        chunks, off, row = [], 0, 0
        total = sum(g["chunks"][li]["length"] for g in m.row_groups)
        host = np.zeros(total + 64, dtype=np.uint8)
        hp = host.ctypes.data
        for g in m.row_groups:
            c = g["chunks"][li]
            N.pq_pread(path, [(c["start"], c["length"], hp + off)], 2)
            heads = N.pq_page_headers(hp + off, c["length"])
            data_pages = [h for h in heads if h["type"] in (0, 3)]
            assert sum(h["num_rows"] if h["type"] == 3 else h["num_values"] for h in data_pages) == g["num_rows"]
            if name != "s":
                assert len(data_pages) > 1  # small data_page_size: several pages per chunk
            chunks.append((off, c["length"], c["codec"], row, g["num_rows"]))
            off += c["length"]
            row += g["num_rows"]
        plan = N.pq_plan(hp, chunks, leaf["type"], leaf["max_def"], leaf["max_rep"])
        assert plan["unsupported"] == ""
        assert plan["num_pages"] * 72 == len(plan["pages"])   # sizeof(kern::PqPage)
        if compression != "none":
            assert plan["num_jobs"] > 0 and plan["dec_bytes"] > 0
            assert plan["num_zstd_jobs"] == (plan["num_jobs"] if compression == "zstd" else 0)
        else:
            assert plan["num_jobs"] == 0
        if name == "s":   # 50 distinct strings: dictionary-encoded in every row group
            assert plan["num_dict_pages"] == len(m.row_groups)
            assert plan["dict_entries"] == sum(
                len(set(t.column("s").slice(i * 8000, 8000).to_pylist())) for i in range(len(m.row_groups)))
            assert plan["plain_pages"] == 0


def test_plan_rejects_corrupt_chunk(tmp_path):
    t = _table(3000)
    path = str(tmp_path / "t.parquet")
    pq.write_table(t, path, compression="none")
    m = FileMeta(path)
    li = m.leaf_index["i64"]
    c = m.row_groups[0]["chunks"][li]
    host = np.zeros(c["length"] + 64, dtype=np.uint8)
    native().pq_pread(path, [(c["start"], c["length"], host.ctypes.data)], 1)
    # claim more rows than the chunk holds
    with pytest.raises(RuntimeError):
        native().pq_plan(host.ctypes.data, [(0, c["length"], 0, 0, 3001)], PHYS["INT64"], 1, 0)
    # truncated chunk
    with pytest.raises(RuntimeError):
        native().pq_plan(host.ctypes.data, [(0, c["length"] // 2, 0, 0, 3000)], PHYS["INT64"], 1, 0)


def test_unsupported_columns_are_reported(tmp_path):
    t = _table(1000)
    p1 = str(tmp_path / "z.parquet")
    pq.write_table(t, p1, compression="zstd")
    assert GpuParquetReader([p1]).supports("i32", T.INT32) is None          # ZSTD decodes on the GPU
    p0 = str(tmp_path / "g.parquet")
    pq.write_table(t, p0, compression="gzip")
    assert "codec" in GpuParquetReader([p0]).supports("i32", T.INT32)
    p2 = str(tmp_path / "n.parquet")
    pq.write_table(pa.table({"l": pa.array([[1, 2], [3]], pa.list_(pa.int64()))}), p2)
    assert FileMeta(p2).leaves[0]["max_rep"] == 1
    p3 = str(tmp_path / "ok.parquet")
    pq.write_table(t, p3)
    r = GpuParquetReader([p3])
    assert r.supports("dec", T.DECIMAL(15, 2)) is None
    assert r.supports("dec", T.DECIMAL(15, 3)) is not None  # scale mismatch: host path
    assert r.supports("s", T.UTF8) is None and r.supports("b", T.BOOL) is None


def test_not_parquet(tmp_path):
    p = tmp_path / "x.parquet"
    p.write_text("# This is a placeholder, not parquet\n" * 4)  # like the reference's data/sample.parquet
    with pytest.raises(IoError):
        FileMeta(str(p))
    with pytest.raises(IoError):
        FileMeta(str(tmp_path / "missing.parquet"))


def test_cpu_scan_unchanged(tmp_path):
    """On CPU the ParquetTable keeps the host decoder (the GPU path is chosen by device)."""
    import igloo_amd as ig
    t = _table(3000)
    pq.write_table(t, tmp_path / "t.parquet", row_group_size=1000)
    e = ig.QueryEngine(device="cpu")
    e.register_parquet("t", str(tmp_path / "t.parquet"))
    r = e.query("SELECT count(*) AS n, sum(i64) AS s, count(nul) AS c FROM t")
    assert r.column("n").to_pylist() == [3000]
    assert r.column("s").to_pylist() == [int(np.sum(t.column("i64").to_numpy()))]
    assert r.column("c").to_pylist() == [3000 - t.column("nul").null_count]
