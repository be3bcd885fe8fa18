"""Logical data types and their device representation.

Device layout (Arrow-compatible in HBM):

* integers / floats / bool: one torch tensor of the natural dtype;
* DATE: int32 days since 1970-01-01 (Arrow date32);
* DECIMAL(p, s): int64 scaled by 10**s (TPC-H decimals are (15, 2)); wide
  results (p > 18, e.g. SUM) may hold an [n, 2] int64 (lo, hi) int128 tensor;
* UTF8: either plain (int64 offsets + uint8 bytes, Arrow large_string) or
  dictionary-encoded (int32 codes + a plain-string dictionary column);
* LIST(t): an [n, 2] int64 (start, length) view per row into a child column
  of type t (so a row gather is one 16-byte gather and the child values never
  move until the result is built); STRUCT: an int64 row id per row into one
  child column per field. The child columns ride in ``Column.dictionary``
  (a ``columnar.Nested`` payload), which every operator already carries
  along with the rows.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import pyarrow as pa
import torch

from .utils.errors import PlanError

INT_KINDS = ("int8", "int16", "int32", "int64")
FLOAT_KINDS = ("float32", "float64")


@dataclass(frozen=True)
class DataType:
    kind: str
    precision: int = 0
    scale: int = 0
    child: Optional["DataType"] = None     # LIST element type
    fields: Tuple = ()                     # STRUCT ((name, DataType), ...)

    @property
    def is_nested(self) -> bool:
        return self.kind in ("list", "struct")

    # ---------------------------------------------------------------- predicates
    @property
    def is_integer(self) -> bool:
        return self.kind in INT_KINDS

    @property
    def is_float(self) -> bool:
        return self.kind in FLOAT_KINDS

    @property
    def is_decimal(self) -> bool:
        return self.kind == "decimal"

    @property
    def is_numeric(self) -> bool:
        return self.is_integer or self.is_float or self.is_decimal

    @property
    def is_string(self) -> bool:
        return self.kind == "utf8"

    @property
    def is_temporal(self) -> bool:
        return self.kind in ("date32", "timestamp")

    # --------------------------------------------------------------- conversion
    @property
    def torch_dtype(self) -> torch.dtype:
        return _TORCH[self.kind]

    def to_arrow(self) -> pa.DataType:
        k = self.kind
        if k == "list":
            return pa.list_(self.child.to_arrow())
        if k == "struct":
            return pa.struct([pa.field(n, t.to_arrow()) for n, t in self.fields])
        if k == "decimal":
            return pa.decimal128(max(self.precision, 1), self.scale)
        if k == "utf8":
            return pa.large_string()
        if k == "timestamp":
            return pa.timestamp("us")
        return _ARROW[k]

    def __str__(self) -> str:
        if self.kind == "decimal":
            return f"Decimal128({self.precision}, {self.scale})"
        if self.kind == "list":
            return f"List({self.child})"
        if self.kind == "struct":
            return "Struct(" + ", ".join(f"{n} {t}" for n, t in self.fields) + ")"
        return _NAMES.get(self.kind, self.kind)

    __repr__ = __str__


BOOL = DataType("bool")
INT8 = DataType("int8")
INT16 = DataType("int16")
INT32 = DataType("int32")
INT64 = DataType("int64")
FLOAT32 = DataType("float32")
FLOAT64 = DataType("float64")
DATE32 = DataType("date32")
TIMESTAMP = DataType("timestamp")
UTF8 = DataType("utf8")
NULL = DataType("null")


def DECIMAL(p: int, s: int) -> DataType:
    return DataType("decimal", min(p, 38), s)


def LIST(child: DataType) -> DataType:
    return DataType("list", child=child)


def STRUCT(fields) -> DataType:
    return DataType("struct", fields=tuple((str(n), t) for n, t in fields))


_TORCH = {
    "bool": torch.bool,
    "int8": torch.int8,
    "int16": torch.int16,
    "int32": torch.int32,
    "int64": torch.int64,
    "float32": torch.float32,
    "float64": torch.float64,
    "date32": torch.int32,
    "timestamp": torch.int64,
    "decimal": torch.int64,
    "utf8": torch.uint8,
    "null": torch.bool,
    "list": torch.int64,
    "struct": torch.int64,
}
_ARROW = {
    "bool": pa.bool_(),
    "int8": pa.int8(),
    "int16": pa.int16(),
    "int32": pa.int32(),
    "int64": pa.int64(),
    "float32": pa.float32(),
    "float64": pa.float64(),
    "date32": pa.date32(),
    "null": pa.null(),
}
_NAMES = {
    "bool": "Boolean",
    "int8": "Int8",
    "int16": "Int16",
    "int32": "Int32",
    "int64": "Int64",
    "float32": "Float32",
    "float64": "Float64",
    "date32": "Date32",
    "utf8": "Utf8",
    "null": "Null",
    "timestamp": "Timestamp(us)",
}


def from_arrow_type(t: pa.DataType) -> DataType:
    if pa.types.is_dictionary(t):
        return from_arrow_type(t.value_type)
    if pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t):
        return LIST(from_arrow_type(t.value_type))
    if pa.types.is_struct(t):
        return STRUCT([(t.field(i).name, from_arrow_type(t.field(i).type)) for i in range(t.num_fields)])
    if pa.types.is_boolean(t):
        return BOOL
    for k in ("int8", "int16", "int32", "int64"):
        if t == _ARROW[k]:
            return DataType(k)
    if pa.types.is_uint8(t) or pa.types.is_uint16(t):
        return INT32
    if pa.types.is_uint32(t) or pa.types.is_uint64(t):
        return INT64
    if pa.types.is_float16(t) or pa.types.is_float32(t):
        return FLOAT32 if pa.types.is_float32(t) else FLOAT64
    if pa.types.is_float64(t):
        return FLOAT64
    if pa.types.is_date32(t) or pa.types.is_date64(t):
        return DATE32
    if pa.types.is_timestamp(t):
        return TIMESTAMP
    if pa.types.is_decimal(t):
        return DECIMAL(t.precision, t.scale)
    if pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_string_view(t):
        return UTF8
    if pa.types.is_null(t):
        return NULL
    raise PlanError(f"unsupported Arrow type {t}")


def parse_type_name(name: str) -> DataType:
    """SQL type name (as produced by the parser) -> DataType."""
    n = name.upper().replace(" ", "")
    base, args = n, []
    if "(" in n:
        base = n[: n.index("(")]
        args = [int(a) for a in n[n.index("(") + 1: -1].split(",") if a]
    if base in ("INT", "INTEGER", "INT4"):
        return INT32
    if base in ("BIGINT", "INT8", "LONG"):
        return INT64
    if base in ("SMALLINT", "INT2"):
        return INT16
    if base in ("TINYINT",):
        return INT8
    if base in ("DOUBLE", "FLOAT8", "FLOAT64"):
        return FLOAT64
    if base in ("FLOAT", "REAL", "FLOAT4", "FLOAT32"):
        return FLOAT32 if base != "FLOAT" else FLOAT64
    if base in ("DECIMAL", "NUMERIC"):
        p = args[0] if args else 38
        s = args[1] if len(args) > 1 else (0 if args else 10)
        return DECIMAL(p, s)
    if base in ("VARCHAR", "CHAR", "TEXT", "STRING", "CHARACTER", "BPCHAR"):
        return UTF8
    if base == "DATE":
        return DATE32
    if base in ("TIMESTAMP", "DATETIME"):
        return TIMESTAMP
    if base in ("BOOLEAN", "BOOL"):
        return BOOL
    raise PlanError(f"unknown type {name}")


def common_numeric(a: DataType, b: DataType) -> DataType:
    """Type both operands are coerced to for comparison / CASE / UNION."""
    if a == b:
        return a
    if a.kind == "list" and b.kind == "list":
        return LIST(common_numeric(a.child, b.child))
    if a.kind == "null":
        return b
    if b.kind == "null":
        return a
    if a.is_float or b.is_float:
        return FLOAT64
    if a.is_decimal or b.is_decimal:
        sa = a.scale if a.is_decimal else 0
        sb = b.scale if b.is_decimal else 0
        s = max(sa, sb)
        ia = (a.precision - a.scale) if a.is_decimal else 19
        ib = (b.precision - b.scale) if b.is_decimal else 19
        return DECIMAL(min(38, max(ia, ib) + s), s)
    if a.is_integer and b.is_integer:
        order = INT_KINDS
        return DataType(order[max(order.index(a.kind), order.index(b.kind))])
    if a.kind == b.kind:
        return a
    if {a.kind, b.kind} <= {"date32", "timestamp"}:
        return TIMESTAMP
    if a.is_string and b.is_temporal:
        return b
    if b.is_string and a.is_temporal:
        return a
    raise PlanError(f"incompatible types {a} and {b}")
