"""Device-resident query results: zero-copy export through the Arrow C Device
Data Interface and DLPack.

``QueryEngine.sql`` hands results back as host Arrow tables (one D2H copy per
buffer, then pyarrow). A consumer on the same GPU (another HIP library, a
PyTorch model, a second engine) does not need that copy: ``sql_device``
returns a ``DeviceResult`` whose columns stay in HBM and are exported

* through ``__arrow_c_device_array__`` (Arrow PyCapsule protocol: an
  ArrowSchema for a struct of the columns and an ArrowDeviceArray with device
  type ROCm, the column buffers themselves as its buffers, and a HIP event
  recorded after the producing kernels as ``sync_event``), built by the
  native core (csrc/runtime/arrow_device.cpp);
* per column through DLPack (``torch.utils.dlpack`` / ``__dlpack__`` of the
  fixed-width data tensors);
* or copied to the host on request (``to_arrow``).

Layout conversions done on the device where the engine's representation
differs from Arrow's (no host round trip): validity byte masks -> bitmaps,
booleans -> bitmaps, 64-bit scaled decimals -> decimal128 (sign-extended).
Strings keep their int64 offsets (Arrow ``large_utf8``), dictionary columns
their int32 codes with the dictionary as a child array.

Reference parity: the reference's pyigloo is an empty cdylib
(reference pyigloo/src/lib.rs:1, pyigloo/Cargo.toml:11-19); SURVEY §7.1
names Arrow C Device / DLPack result interop.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import pyarrow as pa
import torch

from . import types as T
from .columnar import Column


def _bitmap(mask: torch.Tensor) -> torch.Tensor:
    """Byte mask -> Arrow validity / boolean bitmap (LSB first), on the mask's device."""
    n = mask.numel()
    pad = (-n) % 64
    m = mask.to(torch.uint8)
    if pad:
        m = torch.cat([m, torch.zeros(pad, dtype=torch.uint8, device=m.device)])
    w = (torch.ones(8, dtype=torch.uint8, device=m.device) << torch.arange(8, dtype=torch.uint8, device=m.device))
    return (m.view(-1, 8) * w).sum(1, dtype=torch.uint8).contiguous()


def _fmt(dt: T.DataType) -> str:
    k = dt.kind
    if dt.is_decimal:
        return f"d:{max(dt.precision, 1)},{dt.scale}"
    return {"int8": "c", "int16": "s", "int32": "i", "int64": "l", "uint8": "C", "float32": "f", "float64": "g",
            "bool": "b", "date32": "tdD", "null": "n"}.get(k) or ("U" if dt.is_string else None) or \
        _unsupported(dt)


def _unsupported(dt):
    raise TypeError(f"no Arrow C export for column type {dt}")


def _column_specs(c: Column, name: str, nullable: bool) -> Tuple[tuple, tuple]:
    """(schema spec, array spec) of one column for the native exporter; the
    array spec's last element keeps every tensor it points into alive."""
    n = len(c)
    keep: List[torch.Tensor] = []

    def addr(t: Optional[torch.Tensor]) -> int:
        if t is None:
            return 0
        t = t.contiguous()
        keep.append(t)
        return t.data_ptr()

    validity = addr(_bitmap(c.valid)) if c.valid is not None else 0
    null_count = -1 if c.valid is not None else 0      # -1: not computed (no device sync)
    dt = c.dtype
    if dt.is_string and c.is_dict:
        d = c.dictionary
        dschema, darray = _column_specs(d if not d.is_dict else d, "", False)
        sch = ("i", name, nullable, [], dschema)
        arr = (n, null_count, [validity, addr(c.data.to(torch.int32))], [], darray, keep)
        return sch, arr
    if dt.is_string:
        off = c.offsets.to(torch.int64)
        return ("U", name, nullable, [], None), (n, null_count, [validity, addr(off), addr(c.data)], [], None, keep)
    if dt.kind == "null":
        return ("n", name, True, [], None), (n, n, [], [], None, keep)
    if dt.kind == "bool":
        return ("b", name, nullable, [], None), (n, null_count, [validity, addr(_bitmap(c.data))], [], None, keep)
    if dt.is_decimal:
        x = c.data
        wide = x if x.dim() == 2 else torch.stack([x.to(torch.int64), x.to(torch.int64) >> 63], 1)
        return (_fmt(dt), name, nullable, [], None), (n, null_count, [validity, addr(wide)], [], None, keep)
    data = c.data
    want = {"int8": torch.int8, "int16": torch.int16, "int32": torch.int32, "int64": torch.int64,
            "float32": torch.float32, "float64": torch.float64, "date32": torch.int32, "uint8": torch.uint8}
    if dt.kind in want and data.dtype != want[dt.kind]:
        data = data.to(want[dt.kind])
    return (_fmt(dt), name, nullable, [], None), (n, null_count, [validity, addr(data)], [], None, keep)


class DeviceResult:
    """A query result left in device memory (see module docstring)."""

    def __init__(self, columns: Dict[str, Column], num_rows: int, nullable: Optional[Dict[str, bool]] = None):
        self.columns = columns
        self.num_rows = num_rows
        self.nullable = nullable or {k: c.valid is not None for k, c in columns.items()}

    @property
    def names(self) -> List[str]:
        return list(self.columns)

    @property
    def device(self) -> torch.device:
        for c in self.columns.values():
            return c.data.device
        return torch.device("cpu")

    def __len__(self) -> int:
        return self.num_rows

    def __getitem__(self, name: str) -> torch.Tensor:
        """The column's data tensor (fixed-width types: DLPack-exportable as is)."""
        c = self.columns[name]
        if c.dtype.is_string and not c.is_dict:
            raise TypeError(f"column {name!r} is a variable-width string column: use __arrow_c_device_array__")
        return c.data

    def to_dlpack(self, name: str):
        return torch.utils.dlpack.to_dlpack(self[name].contiguous())

    def _specs(self):
        kids_s, kids_a = [], []
        for name, c in self.columns.items():
            s, a = _column_specs(c, name, self.nullable.get(name, True))
            kids_s.append(s)
            kids_a.append(a)
        return ("+s", "", False, kids_s, None), (self.num_rows, 0, [0], kids_a, None, None)

    def __arrow_c_device_array__(self, requested_schema=None, **kwargs):
        """(ArrowSchema capsule, ArrowDeviceArray capsule): a struct array of the
        columns, buffers in place (ROCm device memory, or CPU for a CPU engine)."""
        from .ops._lib import native
        sch, arr = self._specs()
        dev = self.device
        if dev.type == "cuda":
            stream = torch.cuda.current_stream(dev).cuda_stream
            return native().arrow_export_device(sch, arr, dev.index if dev.index is not None else 0, stream)
        return native().arrow_export_device(sch, arr, -1, 0)

    def __arrow_c_array__(self, requested_schema=None):
        """Host memory only (the plain C data interface)."""
        if self.device.type != "cpu":
            raise TypeError("device-resident result: use __arrow_c_device_array__ (or to_arrow() to copy)")
        from .ops._lib import native
        sch, arr = self._specs()
        return native().arrow_export_host(sch, arr)

    def to_arrow(self) -> pa.Table:
        """Copy to the host as a pyarrow.Table."""
        from .engine import _host_columns
        cols = _host_columns(list(self.columns.values()))
        return pa.Table.from_arrays([c.to_arrow() for c in cols], names=self.names)
