"""Plan serialization: logical plans <-> JSON, for shipping query fragments.

The reference declares a serialized-plan field for fragment dispatch but never
fills it: ``serialize_plan`` returns empty bytes and the worker side decodes a
dummy batch (reference crates/coordinator/src/distributed_executor.rs:203-222,
crates/api/proto/distributed.proto FragmentRequest.serialized_plan). Here the
optimized logical plan (every node, expression, type and subquery) round-trips
through a self-describing JSON document; table sources travel by name and are
resolved against the receiving engine's catalog, so a worker executes the
fragment over its own (HBM-resident) partition of the table.
"""
from __future__ import annotations

import dataclasses
import json
from decimal import Decimal
from typing import Any, Callable, Dict

from .. import types as T
from . import expr as E
from . import logical as L

_CLASSES: Dict[str, type] = {}
for _mod in (L, E):
    for _name in dir(_mod):
        _obj = getattr(_mod, _name)
        if isinstance(_obj, type) and dataclasses.is_dataclass(_obj):
            _CLASSES[_name] = _obj
_CLASSES["DataType"] = T.DataType

VERSION = 1


def to_obj(x: Any) -> Any:
    if x is None or isinstance(x, (bool, int, float, str)):
        return x
    if isinstance(x, Decimal):
        return {"__dec": str(x)}
    if isinstance(x, tuple):
        return {"__tuple": [to_obj(v) for v in x]}
    if isinstance(x, (set, frozenset)):
        return {"__set": sorted(to_obj(v) for v in x)}
    if isinstance(x, list):
        return [to_obj(v) for v in x]
    if isinstance(x, bytes):
        return {"__bytes": x.hex()}
    if dataclasses.is_dataclass(x) and not isinstance(x, type):
        # (a statement template's slot / derived literals serialize as literals)
        name = "Lit" if isinstance(x, E.Lit) else type(x).__name__
        if name not in _CLASSES:
            raise TypeError(f"cannot serialize {name}")
        d = {"__c": name}
        for f in dataclasses.fields(x):
            v = getattr(x, f.name)
            if isinstance(x, L.Scan) and f.name == "source":
                d["source"] = {"__table": x.table}
                continue
            d[f.name] = to_obj(v)
        if isinstance(x, L.Scan) and hasattr(x, "table_cols"):
            d["__table_cols"] = to_obj(list(x.table_cols))
        return d
    raise TypeError(f"cannot serialize {type(x).__name__}")


def from_obj(o: Any, resolve: Callable[[str], Any]) -> Any:
    if o is None or isinstance(o, (bool, int, float, str)):
        return o
    if isinstance(o, list):
        return [from_obj(v, resolve) for v in o]
    if "__dec" in o:
        return Decimal(o["__dec"])
    if "__tuple" in o:
        return tuple(from_obj(v, resolve) for v in o["__tuple"])
    if "__set" in o:
        return set(from_obj(v, resolve) for v in o["__set"])
    if "__bytes" in o:
        return bytes.fromhex(o["__bytes"])
    if "__table" in o:
        return resolve(o["__table"])
    cls = _CLASSES[o["__c"]]
    kw = {f.name: from_obj(o[f.name], resolve) for f in dataclasses.fields(cls) if f.name in o}
    obj = cls(**kw)
    if "__table_cols" in o:
        obj.table_cols = from_obj(o["__table_cols"], resolve)
    return obj


def dumps(plan: L.Plan) -> str:
    return json.dumps({"version": VERSION, "plan": to_obj(plan)}, separators=(",", ":"))


def loads(text: str, catalog) -> L.Plan:
    doc = json.loads(text)
    if doc.get("version") != VERSION:
        raise ValueError(f"unsupported plan version {doc.get('version')}")

    def resolve(name: str):
        src = catalog.get_table(name)
        if src is None:
            raise KeyError(f"table {name} not found")
        return src
    return from_obj(doc["plan"], resolve)
