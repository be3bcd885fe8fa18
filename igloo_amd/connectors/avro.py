"""Minimal Avro object-container-file reader/writer (Iceberg manifests).

No Avro library is available in this environment; Iceberg manifest lists and
manifests are Avro OCF files, so this implements the binary encoding (zigzag
varints, strings/bytes, records, arrays, maps, unions, enums, fixed, logical
types as their physical type) with the null and deflate codecs.
"""
from __future__ import annotations

import io
import json
import os
import struct
import zlib
from typing import Any, Dict, Iterator, List, Tuple

MAGIC = b"Obj\x01"


# ------------------------------------------------------------------ decoding
class _Reader:
    def __init__(self, buf: bytes):
        self.b = buf
        self.p = 0

    def long(self) -> int:
        shift = 0
        acc = 0
        while True:
            c = self.b[self.p]
            self.p += 1
            acc |= (c & 0x7F) << shift
            if not c & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)

    def raw(self, n: int) -> bytes:
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def bytes_(self) -> bytes:
        return self.raw(self.long())

    def eof(self) -> bool:
        return self.p >= len(self.b)


def _named(schema, names: Dict[str, Any]):
    if isinstance(schema, str) and schema in names:
        return names[schema]
    return schema


def _register(schema, names):
    if isinstance(schema, dict):
        if schema.get("type") in ("record", "enum", "fixed") and "name" in schema:
            names[schema["name"]] = schema
            if "namespace" in schema:
                names[schema["namespace"] + "." + schema["name"]] = schema
        if schema.get("type") == "record":
            for f in schema["fields"]:
                _register(f["type"], names)
        elif schema.get("type") == "array":
            _register(schema["items"], names)
        elif schema.get("type") == "map":
            _register(schema["values"], names)
    elif isinstance(schema, list):
        for s in schema:
            _register(s, names)


def _decode(r: _Reader, schema, names) -> Any:
    schema = _named(schema, names)
    if isinstance(schema, list):  # union
        return _decode(r, schema[r.long()], names)
    t = schema if isinstance(schema, str) else schema["type"]
    if isinstance(t, (dict, list)):
        return _decode(r, t, names)
    if t == "null":
        return None
    if t == "boolean":
        return r.raw(1) != b"\x00"
    if t in ("int", "long"):
        return r.long()
    if t == "float":
        return struct.unpack("<f", r.raw(4))[0]
    if t == "double":
        return struct.unpack("<d", r.raw(8))[0]
    if t == "bytes":
        return r.bytes_()
    if t == "string":
        return r.bytes_().decode("utf-8")
    if t == "fixed":
        return r.raw(schema["size"])
    if t == "enum":
        return schema["symbols"][r.long()]
    if t == "record":
        return {f["name"]: _decode(r, f["type"], names) for f in schema["fields"]}
    if t == "array":
        out = []
        while True:
            n = r.long()
            if n == 0:
                break
            if n < 0:
                n = -n
                r.long()
            for _ in range(n):
                out.append(_decode(r, schema["items"], names))
        return out
    if t == "map":
        out = {}
        while True:
            n = r.long()
            if n == 0:
                break
            if n < 0:
                n = -n
                r.long()
            for _ in range(n):
                k = r.bytes_().decode("utf-8")
                out[k] = _decode(r, schema["values"], names)
        return out
    raise ValueError(f"unsupported avro type {t}")


def read_ocf(path: str) -> Tuple[dict, List[dict]]:
    """Returns (writer schema, records)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != MAGIC:
        raise ValueError(f"{path}: not an Avro object container file")
    r = _Reader(data)
    r.p = 4
    meta = _decode(r, {"type": "map", "values": "bytes"}, {})
    sync = r.raw(16)
    schema = json.loads(meta["avro.schema"].decode())
    codec = meta.get("avro.codec", b"null").decode()
    names: Dict[str, Any] = {}
    _register(schema, names)
    out = []
    while not r.eof():
        count = r.long()
        size = r.long()
        block = r.raw(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec != "null":
            raise ValueError(f"unsupported avro codec {codec}")
        br = _Reader(block)
        for _ in range(count):
            out.append(_decode(br, schema, names))
        if r.raw(16) != sync:
            raise ValueError(f"{path}: bad sync marker")
    return schema, out


# ------------------------------------------------------------------ encoding
def _zz(n: int) -> bytes:
    n = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _encode(v, schema, names, out: io.BytesIO):
    schema = _named(schema, names)
    if isinstance(schema, list):
        for i, s in enumerate(schema):
            st = s if isinstance(s, str) else s.get("type")
            if (v is None) == (st == "null"):
                out.write(_zz(i))
                return _encode(v, s, names, out)
        raise ValueError("no union branch")
    t = schema if isinstance(schema, str) else schema["type"]
    if isinstance(t, (dict, list)):
        return _encode(v, t, names, out)
    if t == "null":
        return
    if t == "boolean":
        out.write(b"\x01" if v else b"\x00")
    elif t in ("int", "long"):
        out.write(_zz(int(v)))
    elif t == "double":
        out.write(struct.pack("<d", v))
    elif t == "float":
        out.write(struct.pack("<f", v))
    elif t in ("bytes", "string"):
        b = v.encode() if isinstance(v, str) else v
        out.write(_zz(len(b)))
        out.write(b)
    elif t == "record":
        for f in schema["fields"]:
            _encode(v.get(f["name"]), f["type"], names, out)
    elif t == "array":
        if v:
            out.write(_zz(len(v)))
            for x in v:
                _encode(x, schema["items"], names, out)
        out.write(_zz(0))
    elif t == "map":
        if v:
            out.write(_zz(len(v)))
            for k, x in v.items():
                _encode(k, "string", names, out)
                _encode(x, schema["values"], names, out)
        out.write(_zz(0))
    elif t == "enum":
        out.write(_zz(schema["symbols"].index(v)))
    elif t == "fixed":
        out.write(v)
    else:
        raise ValueError(t)


def write_ocf(path: str, schema: dict, records: List[dict], codec: str = "deflate"):
    names: Dict[str, Any] = {}
    _register(schema, names)
    body = io.BytesIO()
    for rec in records:
        _encode(rec, schema, names, body)
    block = body.getvalue()
    if codec == "deflate":
        c = zlib.compressobj(9, zlib.DEFLATED, -15)
        block = c.compress(block) + c.flush()
    sync = os.urandom(16)
    out = io.BytesIO()
    out.write(MAGIC)
    _encode({"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()},
            {"type": "map", "values": "bytes"}, {}, out)
    out.write(sync)
    out.write(_zz(len(records)))
    out.write(_zz(len(block)))
    out.write(block)
    out.write(sync)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(out.getvalue())
