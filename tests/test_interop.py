"""Zero-copy device results (igloo_amd/interop.py, csrc/runtime/arrow_device.cpp):
``QueryEngine.sql_device`` exports through the Arrow C Device Data Interface
(PyCapsules built by the native core) and DLPack. On the CPU the export is
imported back by pyarrow and compared with ``QueryEngine.query``; on the GPU
the ArrowDeviceArray must describe ROCm memory whose buffers ARE the result
columns' device buffers (no copy), and DLPack must hand the same memory to
torch."""
import decimal

import pyarrow as pa
import pytest
import torch

import igloo_amd as ig


def _engine(device):
    e = ig.QueryEngine(device=device)
    e.register_table("t", pa.table({
        "a": pa.array([1, 2, None, 4, 5], pa.int64()),
        "s": ["x", "yy", None, "zzz", "w"],
        "d": pa.array([decimal.Decimal("1.25"), decimal.Decimal("-2.50"), None, decimal.Decimal("3.00"),
                       decimal.Decimal("0.01")], pa.decimal128(15, 2)),
        "b": [True, False, None, True, False],
        "k": pa.array(["p", "q", "p", "r", "q"]).dictionary_encode(),
        "dt": pa.array([0, 1, 2, 3, 4], pa.int32()).cast(pa.date32()),
    }))
    return e


SQL = "SELECT a, s, d, b, k, dt, a * 2 AS a2, a > 1 AS big FROM t ORDER BY dt"


def test_arrow_c_device_roundtrip_cpu():
    e = _engine("cpu")
    r = e.sql_device(SQL)
    assert r.num_rows == 5 and r.names == ["a", "s", "d", "b", "k", "dt", "a2", "big"]
    got = pa.record_batch(r)                 # __arrow_c_device_array__ (CPU device)
    want = e.query(SQL)
    assert got.to_pylist() == want.to_pylist()
    assert pa.types.is_dictionary(got.schema.field("k").type)
    assert got.schema.field("d").type == pa.decimal128(15, 2)
    # the plain C data interface too, and DLPack of a fixed-width column
    class _Host:                             # the plain C data interface (host memory)
        __arrow_c_array__ = r.__arrow_c_array__
    assert pa.record_batch(_Host()).to_pylist() == want.to_pylist()
    assert torch.equal(torch.from_dlpack(r.to_dlpack("dt")), r["dt"])
    assert r.to_arrow().to_pylist() == want.to_pylist()


@pytest.mark.gpu
def test_arrow_c_device_zero_copy_gpu():
    from igloo_amd.ops._lib import native
    e = _engine("cuda:0")
    r = e.sql_device(SQL)
    schema_cap, array_cap = r.__arrow_c_device_array__()
    info = native().arrow_describe_device_array(array_cap)
    assert info["device_type"] == 10 and info["device_id"] == 0 and info["has_event"]     # ARROW_DEVICE_ROCM
    assert info["length"] == 5 and info["n_children"] == 8
    # zero copy: the exported data buffers are the result columns' device memory
    names = r.names
    for name in ("a", "dt", "a2"):
        kid = info["children"][names.index(name)]
        assert kid["buffers"][1] == r.columns[name].data.data_ptr(), name
    s_kid = info["children"][names.index("s")]
    assert s_kid["buffers"][2] == r.columns["s"].data.data_ptr()
    assert info["children"][names.index("k")]["has_dictionary"]
    # DLPack hands the same memory to torch
    t = torch.from_dlpack(r.to_dlpack("a2"))
    assert t.device.type == "cuda" and t.data_ptr() == r.columns["a2"].data.data_ptr()
    assert r.to_arrow().to_pylist() == e.query(SQL).to_pylist()
    del schema_cap, array_cap       # release callbacks run (keep-alive refs dropped under the GIL)
