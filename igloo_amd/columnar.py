"""Device-resident columnar data: ``Column`` and ``Batch``.

The reference moves arrow-rs ``RecordBatch``es between operators through
bounded channels (reference crates/engine/src/physical_plan.rs:10-17,
crates/engine/src/operators/parquet_scan.rs:44). Here a column lives in HBM as
torch tensors laid out like Arrow (values / validity / offsets / dictionary),
so kernels consume it without conversion and ``to_arrow`` is a D2H copy plus
buffer wrapping.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

from . import types as T
from .types import DataType
from .utils.errors import ExecutionError


class Column:
    """One column on a device.

    * fixed width: ``data`` is a 1-D tensor (or [n, 2] int64 for int128 decimals);
    * plain UTF8: ``offsets`` int64 [n+1] and ``data`` uint8 bytes;
    * dictionary UTF8: ``data`` int32 codes and ``dictionary`` a plain UTF8 Column.
    ``valid`` is an optional bool tensor (True = not null).
    """

    __slots__ = ("dtype", "data", "valid", "offsets", "dictionary", "_host_dict", "_sorted_dict", "_unified",
                 "_cache")

    def __init__(self, dtype: DataType, data: torch.Tensor, valid: Optional[torch.Tensor] = None,
                 offsets: Optional[torch.Tensor] = None, dictionary: Optional["Column"] = None):
        self.dtype = dtype
        self.data = data
        self.valid = valid
        self.offsets = offsets
        self.dictionary = dictionary
        self._host_dict = None
        self._cache = None
        self._sorted_dict = None
        self._unified = None      # content digest when used as a dictionary (parallel/exchange.py)

    # ------------------------------------------------------------------ shape
    def __len__(self) -> int:
        if self.offsets is not None:
            return self.offsets.numel() - 1
        return self.data.shape[0]

    @property
    def device(self) -> torch.device:
        return self.data.device

    @property
    def is_dict(self) -> bool:
        return self.dictionary is not None and not self.dtype.is_nested

    @property
    def nested(self) -> "Nested":
        """LIST / STRUCT columns: the child column(s) the rows point into."""
        assert self.dtype.is_nested and isinstance(self.dictionary, Nested), self
        return self.dictionary

    @property
    def is_plain_string(self) -> bool:
        return self.offsets is not None

    @property
    def is_wide(self) -> bool:
        return self.data.dim() == 2

    @property
    def nbytes(self) -> int:
        n = self.data.numel() * self.data.element_size()
        if self.valid is not None:
            n += self.valid.numel()
        if self.offsets is not None:
            n += self.offsets.numel() * 8
        if self.dictionary is not None:
            n += self.dictionary.nbytes
        return n

    def null_count(self) -> int:
        if self.valid is None:
            return 0
        return int((~self.valid).sum().item())

    # ------------------------------------------------------------ host helpers
    def dict_values(self) -> List[Optional[str]]:
        """Host copy of a dictionary column's values, cached on the dictionary
        itself: a resident table's dictionary is shared by every column built
        from it, so repeated queries convert it once."""
        assert self.dictionary is not None
        d = self.dictionary
        if d._host_dict is None:
            d._host_dict = d.to_arrow().to_pylist()
        return d._host_dict

    def derived(self) -> dict:
        """Per-column cache of small structures derived from its values (used on
        dictionaries: lookup tables per predicate, sort ranks, code maps)."""
        if self._cache is None:
            self._cache = {}
        return self._cache

    def to(self, device) -> "Column":
        device = torch.device(device)
        if self.device == device:
            return self
        return Column(self.dtype, self.data.to(device), None if self.valid is None else self.valid.to(device),
                      None if self.offsets is None else self.offsets.to(device),
                      None if self.dictionary is None else self.dictionary.to(device))

    # ------------------------------------------------------------ constructors
    @staticmethod
    def from_values(values: Sequence[Any], dtype: DataType, device="cpu") -> "Column":
        """Build from Python values (None = NULL)."""
        arr = pa.array(list(values), type=dtype.to_arrow() if dtype.kind != "null" else pa.null())
        return Column.from_arrow(arr, device=device, dtype=dtype)

    @staticmethod
    def full(value: Any, dtype: DataType, n: int, device) -> "Column":
        device = torch.device(device)
        if dtype.is_nested:
            return Column.from_arrow(pa.array([value] * n, dtype.to_arrow()), device=device, dtype=dtype)
        if value is None:
            if dtype.is_string:
                return Column(dtype, torch.zeros(0, dtype=torch.uint8, device=device),
                              torch.zeros(n, dtype=torch.bool, device=device),
                              offsets=torch.zeros(n + 1, dtype=torch.int64, device=device))
            td = dtype.torch_dtype if dtype.kind != "null" else torch.bool
            return Column(dtype, torch.zeros(n, dtype=td, device=device), torch.zeros(n, dtype=torch.bool, device=device))
        if dtype.is_string:
            b = value.encode("utf-8")
            d = Column.from_arrow(pa.array([value], pa.large_string()), device=device)
            return Column(dtype, torch.zeros(n, dtype=torch.int32, device=device), dictionary=d)
        return Column(dtype, torch.full((n,), value, dtype=dtype.torch_dtype, device=device))

    @staticmethod
    def from_arrow(arr, device="cpu", dtype: Optional[DataType] = None, dict_encode: Optional[bool] = None) -> "Column":
        device = torch.device(device)
        if isinstance(arr, pa.ChunkedArray):
            arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
        t = arr.type
        if dtype is None:
            dtype = T.from_arrow_type(t)
        n = len(arr)
        valid = None
        if arr.null_count > 0:
            valid = torch.from_numpy(np.array(arr.is_valid().to_numpy(zero_copy_only=False), dtype=np.bool_)).to(device)
        if dtype.kind == "list":
            if pa.types.is_fixed_size_list(t):
                arr = arr.cast(pa.list_(t.value_type))
            flat = arr.flatten()         # the child values of the non-null rows, in row order
            off = np.asarray(arr.value_lengths().fill_null(0).to_numpy(zero_copy_only=False), dtype=np.int64)
            lens = off.copy()
            starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if n else np.zeros(0, np.int64)
            child = Column.from_arrow(flat, device=device, dtype=dtype.child, dict_encode=False)
            data = torch.from_numpy(np.stack([starts, lens], axis=1).astype(np.int64)).to(device)
            return Column(dtype, data, valid, dictionary=Nested(child=child))
        if dtype.kind == "struct":
            kids = {}
            for i, (fname, ft) in enumerate(dtype.fields):
                kids[fname] = Column.from_arrow(arr.field(i), device=device, dtype=ft, dict_encode=False)
            return Column(dtype, torch.arange(n, dtype=torch.int64, device=device), valid,
                          dictionary=Nested(children=kids))
        if pa.types.is_dictionary(t):
            codes = np.array(arr.indices.cast(pa.int32()).fill_null(0).to_numpy(zero_copy_only=False))
            dic = Column.from_arrow(arr.dictionary.cast(pa.large_string()), device=device, dict_encode=False)
            return Column(T.UTF8, torch.from_numpy(codes.astype(np.int32)).to(device), valid, dictionary=dic)
        if dtype.is_string:
            arr = arr.cast(pa.large_string())
            if dict_encode is None:
                dict_encode = n >= 64 and _low_cardinality(arr)
            if dict_encode:
                return Column.from_arrow(pc.dictionary_encode(arr), device=device)
            bufs = arr.buffers()
            off = np.frombuffer(bufs[1], dtype=np.int64, count=n + 1, offset=arr.offset * 8).copy()
            base = off[0]
            off -= base
            data = np.frombuffer(bufs[2], dtype=np.uint8, count=int(off[-1]), offset=int(base)) if bufs[2] is not None and off[-1] > 0 else np.zeros(0, np.uint8)
            return Column(T.UTF8, torch.from_numpy(data.copy()).to(device), valid,
                          offsets=torch.from_numpy(off).to(device))
        if dtype.kind == "null":
            return Column(T.NULL, torch.zeros(n, dtype=torch.bool, device=device), torch.zeros(n, dtype=torch.bool, device=device))
        if dtype.is_decimal:
            at = arr.type
            if not pa.types.is_decimal(at):
                arr = arr.cast(dtype.to_arrow())
            elif at.scale != dtype.scale:
                arr = arr.cast(pa.decimal128(38, dtype.scale))
            vals = _decimal_to_int64(arr)
            return Column(dtype, torch.from_numpy(np.array(vals)).to(device), valid)
        if dtype.kind == "date32":
            arr = arr.cast(pa.date32())
            np_vals = arr.cast(pa.int32()).fill_null(0).to_numpy(zero_copy_only=False)
        elif dtype.kind == "timestamp":
            np_vals = arr.cast(pa.timestamp("us")).cast(pa.int64()).fill_null(0).to_numpy(zero_copy_only=False)
        elif dtype.kind == "bool":
            np_vals = arr.fill_null(False).to_numpy(zero_copy_only=False).astype(np.bool_)
        else:
            target = dtype.to_arrow()
            if arr.type != target:
                arr = arr.cast(target)
            np_vals = arr.fill_null(0).to_numpy(zero_copy_only=False)
        t_ = torch.from_numpy(np.array(np_vals, dtype=_NP[dtype.kind], copy=True)).to(device)
        return Column(dtype, t_, valid)

    # --------------------------------------------------------------- to arrow
    def to_arrow(self) -> pa.Array:
        n = len(self)
        validity = None
        if self.valid is not None:
            v = self.valid.cpu().numpy()
            if not v.all():
                validity = pa.array(v, pa.bool_()).buffers()[1]
        dt = self.dtype
        if dt.is_nested:
            return _nested_to_arrow(self, n, validity)
        if dt.is_string:
            if self.dictionary is not None and self.data.is_cuda and len(self.dictionary) > 2 * n + 1024:
                # small slice of a big dictionary (e.g. top-k rows of a grouped
                # result): decode on the device, ship only the referenced bytes
                from .ops.strings import decode
                return decode(self).to_arrow()
            if self.dictionary is not None:
                codes = self.data.cpu().numpy().astype(np.int32)
                dic = self.dictionary.to_arrow()
                if self.valid is not None:
                    idx = pa.array(codes, pa.int32(), mask=~self.valid.cpu().numpy())
                else:
                    idx = pa.array(codes, pa.int32())
                return pc.take(dic, idx) if n else pa.array([], pa.large_string())
            off = self.offsets.cpu().numpy().astype(np.int64)
            chars = self.data.cpu().numpy().astype(np.uint8)
            return pa.Array.from_buffers(pa.large_string(), n, [validity, pa.py_buffer(off), pa.py_buffer(chars)])
        if dt.kind == "null":
            return pa.nulls(n)
        if dt.is_decimal:
            x = self.data.cpu().numpy()
            if x.ndim == 1:
                lo = x.astype(np.int64)
                hi = np.where(lo < 0, -1, 0).astype(np.int64)
            else:
                lo, hi = x[:, 0].astype(np.int64), x[:, 1].astype(np.int64)
            buf = np.empty((n, 2), dtype=np.int64)
            buf[:, 0], buf[:, 1] = lo, hi
            p = max(dt.precision, 1)
            return pa.Array.from_buffers(pa.decimal128(p, dt.scale), n, [validity, pa.py_buffer(buf.tobytes())])
        x = self.data.cpu().numpy()
        if dt.kind == "date32":
            return pa.Array.from_buffers(pa.date32(), n, [validity, pa.py_buffer(x.astype(np.int32).tobytes())])
        if dt.kind == "timestamp":
            return pa.Array.from_buffers(pa.timestamp("us"), n, [validity, pa.py_buffer(x.astype(np.int64).tobytes())])
        if dt.kind == "bool":
            mask = None if self.valid is None else ~self.valid.cpu().numpy()
            return pa.array(x.astype(np.bool_), pa.bool_(), mask=mask)
        return pa.Array.from_buffers(dt.to_arrow(), n, [validity, pa.py_buffer(np.ascontiguousarray(x).tobytes())])

    def to_pylist(self) -> list:
        return self.to_arrow().to_pylist()

    def __repr__(self) -> str:
        rep = "dict" if self.is_dict else ("plain" if self.is_plain_string else "fixed")
        return f"Column({self.dtype}, n={len(self)}, {rep}, device={self.device})"


class Nested:
    """Child column(s) of a LIST (``child``) or STRUCT (``children``) column,
    carried in ``Column.dictionary`` so every operator that moves rows keeps
    them (rows are views: (start, length) pairs or row ids into the child)."""

    def __init__(self, child: Optional[Column] = None, children: Optional[Dict[str, Column]] = None):
        self.child = child
        self.children = children

    def to(self, device) -> "Nested":
        if self.child is not None:
            return Nested(child=self.child.to(device))
        return Nested(children={k: c.to(device) for k, c in self.children.items()})

    @property
    def nbytes(self) -> int:
        if self.child is not None:
            return self.child.nbytes
        return sum(c.nbytes for c in self.children.values())

    def __len__(self) -> int:
        if self.child is not None:
            return len(self.child)
        return len(next(iter(self.children.values()))) if self.children else 0


def _nested_to_arrow(col: "Column", n: int, validity) -> pa.Array:
    dt = col.dtype
    mask = None if col.valid is None else ~col.valid.cpu().numpy().astype(np.bool_)
    if dt.kind == "struct":
        rid = col.data.cpu().numpy().astype(np.int64)
        arrs = []
        for fname, ft in dt.fields:
            ch = col.nested.children[fname].to_arrow()
            arrs.append(pc.take(ch, pa.array(rid, pa.int64())) if n else pa.array([], ft.to_arrow()))
        return pa.StructArray.from_arrays(arrs, names=[f for f, _ in dt.fields],
                                          mask=pa.array(mask) if mask is not None else None)
    se = col.data.cpu().numpy().astype(np.int64).reshape(n, 2) if n else np.zeros((0, 2), np.int64)
    starts, lens = se[:, 0], se[:, 1]
    if mask is not None:
        lens = np.where(mask, 0, lens)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    idx = (np.repeat(starts - off[:-1], lens) + np.arange(off[-1], dtype=np.int64)) if off[-1] else np.zeros(0, np.int64)
    child = col.nested.child.to_arrow()
    vals = pc.take(child, pa.array(idx, pa.int64())) if len(idx) else pa.array([], dt.child.to_arrow())
    vals = vals.cast(dt.child.to_arrow())
    out = pa.ListArray.from_arrays(pa.array(off.astype(np.int32)), vals,
                                   mask=pa.array(mask) if mask is not None else None)
    return out


_NP = {
    "bool": np.bool_, "int8": np.int8, "int16": np.int16, "int32": np.int32, "int64": np.int64,
    "float32": np.float32, "float64": np.float64, "date32": np.int32, "timestamp": np.int64,
}


def _low_cardinality(arr: pa.Array) -> bool:
    sample = arr if len(arr) <= 200_000 else arr.slice(0, 200_000)
    nd = pc.count_distinct(sample).as_py()
    return nd <= 65536 and nd * 4 <= len(sample)


def _decimal_to_int64(arr: pa.Array) -> np.ndarray:
    """decimal128 array -> int64 unscaled values, or [n, 2] (lo, hi) int64
    pairs when some value needs more than 63 bits."""
    n = len(arr)
    if n == 0:
        return np.zeros(0, np.int64)
    arr = arr.cast(pa.decimal128(38, arr.type.scale)) if arr.type.precision > 38 else arr
    buf = arr.buffers()[1]
    raw = np.frombuffer(buf, dtype=np.int64, count=2 * n, offset=arr.offset * 16).reshape(n, 2)
    lo, hi = raw[:, 0], raw[:, 1]
    ok = (hi == np.where(lo < 0, -1, 0))
    if arr.null_count:
        ok |= ~arr.is_valid().to_numpy(zero_copy_only=False)
    if not ok.all():
        # past 63 bits: the [n, 2] (lo, hi) 128-bit layout (NULL rows zeroed)
        out = raw.copy()
        if arr.null_count:
            out[~arr.is_valid().to_numpy(zero_copy_only=False)] = 0
        return out
    out = lo.copy()
    if arr.null_count:
        out[~arr.is_valid().to_numpy(zero_copy_only=False)] = 0
    return out


class LazyColumn(Column):
    """Column ``cid`` of batch ``src`` taken at rows ``idx``, gathered only when
    its values are first read. ``take`` composes a further row selection into
    the index instead of gathering (ops/gather.py ``take_many``): TPC-H Q10's
    ORDER BY revenue LIMIT 20 over 3.9M customer groups gathers the names,
    addresses and comments of its 20 rows, not of 3.9M. Length and structure
    (dictionary / plain string / 128-bit) come from the source column without
    gathering. ``src`` may be a filtered lazy scan (``take_rows``)."""

    __slots__ = ("_src", "_cid", "_idx", "_mat", "_proto")

    def __init__(self, dtype: DataType, src, cid, idx: torch.Tensor):  # noqa: D401 - no Column.__init__
        self.dtype = dtype
        self._src, self._cid, self._idx, self._mat = src, cid, idx, None
        base = getattr(src, "src", None) if hasattr(src, "take_rows") else None
        self._proto = (base if base is not None else src).columns[cid]
        self._host_dict = None
        self._cache = None
        self._sorted_dict = None
        self._unified = None

    def materialize(self) -> Column:
        if self._mat is None:
            if hasattr(self._src, "take_rows"):
                self._mat = self._src.take_rows([self._cid], self._idx)[0]
            else:
                from .ops.gather import take
                self._mat = take(self._src.columns[self._cid], self._idx)
        return self._mat

    def taken(self, idx: torch.Tensor) -> "LazyColumn":
        """Still lazy: this column at its rows ``idx`` (no negatives)."""
        from .ops.gather import gather_tensor
        return LazyColumn(self.dtype, self._src, self._cid, gather_tensor(self._idx, idx))

    @property
    def pending(self) -> bool:
        return self._mat is None

    def __len__(self) -> int:
        return self._idx.numel()

    @property
    def device(self) -> torch.device:
        return self._idx.device

    @property
    def is_dict(self) -> bool:
        return self._proto.is_dict

    @property
    def is_plain_string(self) -> bool:
        return self._proto.is_plain_string

    @property
    def is_wide(self) -> bool:
        return self._proto.is_wide

    def _get(name):
        def get(self):
            return getattr(self.materialize(), name)

        def put(self, v):
            setattr(self.materialize(), name, v)
        return property(get, put)

    data = _get("data")
    valid = _get("valid")
    offsets = _get("offsets")
    dictionary = _get("dictionary")
    del _get


def batch_device(b) -> Optional[torch.device]:
    """Device of a batch's columns without materialising any: lazy batches
    (join results in index form, filtered scans) report theirs from their
    row-index tensors; a plain batch from its first column."""
    d = getattr(b, "device", None)
    if isinstance(d, torch.device):
        return d
    for c in b.columns.values():
        return c.device
    return None


class Batch:
    """An ordered set of equally long columns keyed by column id (or name)."""

    __slots__ = ("columns", "num_rows", "dist", "out_dist", "preamble", "deferred")

    def __init__(self, columns: Dict[Any, Column], num_rows: Optional[int] = None, dist=None):
        self.deferred = None      # query result: (device error flags, messages) checked with its host copy
        self.dist = dist          # ("hash", cid) | ("replicated",) | None  (SPMD row placement)
        self.out_dist = None
        self.preamble = None      # per-rank ints of the last exchange preamble (parallel/exchange.py)
        self.columns = dict(columns)
        if num_rows is None:
            num_rows = len(next(iter(self.columns.values()))) if self.columns else 0
        self.num_rows = num_rows

    def __getitem__(self, k) -> Column:
        return self.columns[k]

    def __contains__(self, k) -> bool:
        return k in self.columns

    def keys(self):
        return self.columns.keys()

    def select(self, keys: Iterable) -> "Batch":
        return Batch({k: self.columns[k] for k in keys}, self.num_rows)

    def to_arrow(self, names: Optional[Dict[Any, str]] = None) -> pa.Table:
        arrays, fields = [], []
        for k, c in self.columns.items():
            arrays.append(c.to_arrow())
            fields.append(names.get(k, str(k)) if names else str(k))
        return pa.Table.from_arrays(arrays, names=fields)

    @staticmethod
    def from_arrow(table: pa.Table, device="cpu") -> "Batch":
        return Batch({name: Column.from_arrow(table.column(name), device=device) for name in table.column_names},
                     table.num_rows)

    def to(self, device) -> "Batch":
        return Batch({k: c.to(device) for k, c in self.columns.items()}, self.num_rows)

    @property
    def nbytes(self) -> int:
        return sum(c.nbytes for c in self.columns.values())
