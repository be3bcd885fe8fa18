"""NDJSON table source (``CREATE EXTERNAL TABLE ... STORED AS JSON``).

Parity: DataFusion's JSON format (reference Cargo.lock:947
datafusion-datasource-json), reached through ``SessionContext::sql``
(reference crates/engine/src/lib.rs:54-57). The schema is inferred from the
first records (Int64 / Float64 / Boolean / Utf8; a nested object or array
becomes a Utf8 column holding its JSON text -- DataFusion infers Struct /
List there: parity unpinned) or given explicitly. On a GPU the file is
parsed by gfx950 kernels (connectors/gpu_json.py); on CPU, or when a value
does not parse as its column type, Arrow's JSON reader is used.
"""
from __future__ import annotations

import json as _json
import os
from typing import List, Optional, Sequence

import pyarrow as pa
import torch

from .. import types as T
from ..catalog import Field, TableSource
from ..columnar import Batch, Column
from ..utils.errors import IoError

INFER_RECORDS = 1000


def _infer(path: str) -> List[Field]:
    order, kinds = [], {}
    try:
        with open(path, "rb") as f:
            n = 0
            for line in f:
                line = line.strip()
                if not line:
                    continue
                rec = _json.loads(line)
                if not isinstance(rec, dict):
                    raise IoError(f"{path}: a JSON record must be an object")
                for k, v in rec.items():
                    if k not in kinds:
                        order.append(k)
                        kinds[k] = set()
                    if v is None:
                        continue
                    kinds[k].add("bool" if isinstance(v, bool) else "int" if isinstance(v, int) else
                                  "float" if isinstance(v, float) else "str" if isinstance(v, str) else "nested")
                n += 1
                if n >= INFER_RECORDS:
                    break
    except OSError as e:
        raise IoError(f"failed to open {path}: {e.strerror or e}") from e
    except ValueError as e:
        raise IoError(f"{path}: malformed JSON record: {e}") from e
    out = []
    for k in order:
        ks = kinds[k]
        if ks <= {"int"} and ks:
            t = T.INT64
        elif ks <= {"int", "float"} and ks:
            t = T.FLOAT64
        elif ks == {"bool"}:
            t = T.BOOL
        else:
            t = T.UTF8
        out.append(Field(k, t, True))
    return out


class JsonTable(TableSource):
    cacheable = True

    def __init__(self, path: str, schema: Optional[List[Field]] = None):
        self.path = path
        self._schema = schema
        self._table: Optional[pa.Table] = None
        self._rows: Optional[int] = None
        self.last_scan = ""

    def schema(self) -> List[Field]:
        if self._schema is None:
            if not os.path.exists(self.path):
                raise IoError(f"failed to open {self.path}: No such file or directory")
            self._schema = _infer(self.path)
        return self._schema

    def _load(self) -> pa.Table:
        if self._table is None:
            import pyarrow.json as pj
            fields = self.schema()
            sch = pa.schema([pa.field(f.name, pa.string() if f.dtype.is_string else f.dtype.to_arrow())
                             for f in fields])
            try:
                t = pj.read_json(self.path, parse_options=pj.ParseOptions(explicit_schema=sch,
                                                                          unexpected_field_behavior="ignore"))
            except pa.ArrowInvalid:
                # nested values in a string column: the JSON text of the value
                rows = [_json.loads(ln) for ln in open(self.path, "rb") if ln.strip()]
                cols = {}
                for f in fields:
                    vals = [r.get(f.name) for r in rows]
                    if f.dtype.is_string:
                        vals = [v if v is None or isinstance(v, str) else _json.dumps(v, separators=(",", ":"))
                                for v in vals]
                    cols[f.name] = pa.array(vals, pa.string() if f.dtype.is_string else f.dtype.to_arrow())
                t = pa.table(cols)
            self._table = t
        return self._table

    def num_rows(self) -> int:
        if self._rows is not None:
            return self._rows
        return self._load().num_rows

    @property
    def version(self):
        try:
            st = os.stat(self.path)
        except OSError:
            return None
        v = (st.st_mtime_ns, st.st_size)
        if getattr(self, "_ver", None) not in (None, v):
            self._table = None
            self._rows = None
        self._ver = v
        return v

    def scan(self, columns: Sequence[str], ctx) -> Batch:
        device = ctx.device if ctx is not None else torch.device("cpu")
        rank, world = 0, 1
        if ctx is not None and ctx.comm is not None:
            rank, world = ctx.comm.rank, ctx.comm.world_size
        out = None
        if device.type == "cuda" and columns:
            from .gpu_json import JsonParseError, read_json_gpu
            try:
                out = read_json_gpu(self.path, self.schema(), columns, device)
                self.last_scan = "gpu"
            except JsonParseError as e:
                self.last_scan = f"host: {e}"
        if out is not None:
            n = len(next(iter(out.values())))
            self._rows = n
            if world > 1:
                from ..ops.gather import take
                per = (n + world - 1) // world
                lo, hi = min(rank * per, n), min((rank + 1) * per, n)
                idx = torch.arange(lo, hi, dtype=torch.int64, device=device)
                out = {c: take(col, idx) for c, col in out.items()}
            n = len(next(iter(out.values())))
            return Batch({c: out[c] for c in columns}, n)
        t = self._load()
        if world > 1:
            per = (t.num_rows + world - 1) // world
            t = t.slice(rank * per, per)
        types = {f.name: f.dtype for f in self.schema()}
        cols = {c: Column.from_arrow(t.column(c), device=device, dtype=types[c]) for c in columns}
        if not self.last_scan.startswith("host"):
            self.last_scan = "host"
        return Batch(cols, t.num_rows)
