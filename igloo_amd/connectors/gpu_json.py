"""GPU NDJSON reader: the file staged in HBM, records split at newlines
(csv_rows with no quote character) and parsed by ``json_parse``
(csrc/kernels/json.hip) into typed columns; strings are decoded by
``json_str_copy``. Parity: DataFusion's arrow-json ``STORED AS JSON``
(reference Cargo.lock:947 datafusion-datasource-json)."""
from __future__ import annotations

import os
from typing import Dict, Optional, Sequence

import torch

from .. import types as T
from ..columnar import Column
from ..ops._lib import launch, native, ptr, stream
from ..ops.select import exclusive_scan, offsets_from_lengths
from ..utils.errors import IoError
from .gpu_csv import KIND

ERRORS = {1: "malformed JSON record", 2: "value does not parse as the column type",
          3: "a record lacks a non-nullable field"}
MAX_FIELDS = 64


class JsonParseError(IoError):
    pass


def read_json_gpu(path: str, fields: Sequence, columns: Optional[Sequence[str]], device) -> Dict[str, Column]:
    device = torch.device(device)
    N = native()
    if len(fields) > MAX_FIELDS:
        raise JsonParseError(f"{len(fields)} fields: the GPU parser handles at most {MAX_FIELDS}")
    want = set(columns) if columns is not None else {f.name for f in fields}
    for f in fields:
        if f.name in want and KIND.get(f.dtype.kind) is None:
            raise JsonParseError(f"column {f.name}: type {f.dtype} is not parsed on the GPU")
    try:
        size = os.path.getsize(path)
    except OSError as e:
        raise IoError(f"failed to open {path}: {e.strerror or e}") from e
    host = torch.empty(size + 64, dtype=torch.uint8, pin_memory=True)
    if size:
        N.pq_pread(path, [(0, size, host.data_ptr())], 8)
    host[size:] = 0
    buf = torch.empty(size + 64, dtype=torch.uint8, device=device)
    buf.copy_(host, non_blocking=True)
    s = stream(buf)
    tiles = N.csv_num_tiles(size)
    state = torch.zeros(max(tiles, 1), dtype=torch.uint8, device=device)   # no quotes: every '\n' ends a record
    tile_rows = torch.empty(max(tiles, 1), dtype=torch.int64, device=device)
    N.csv_rows(ptr(buf), size, 0, 0, ptr(state), ptr(tile_rows), 0, 0, s)
    tile_off, nterm = exclusive_scan(tile_rows[:tiles]) if tiles else (tile_rows, 0)
    tail = host[:size].numpy().tobytes().rstrip(b" \t\r\n") if size else b""
    last_open = size > 0 and len(tail) > 0 and host[size - 1].item() != ord("\n")
    nrows = nterm + (1 if last_open else 0)
    rows_end = torch.empty(max(nrows, 1), dtype=torch.int64, device=device)
    if nterm:
        launch("csv_rows").csv_rows(ptr(buf), size, 0, 0, ptr(state), 0, ptr(tile_off), ptr(rows_end), s)
    if last_open:
        rows_end[nrows - 1] = size
    specs, outs = [], {}
    for f in fields:
        k = KIND.get(f.dtype.kind, 0) if f.name in want else 0
        if not k:
            specs.append((0, 0, 0, 0, 0))
            continue
        valid = torch.ones(nrows, dtype=torch.bool, device=device) if f.nullable else None
        if k == KIND["utf8"]:
            pos = torch.empty(max(nrows, 1), dtype=torch.int64, device=device)
            lenf = torch.empty(max(nrows, 1), dtype=torch.int64, device=device)
            specs.append((k, 0, ptr(pos), ptr(lenf), ptr(valid)))
            outs[f.name] = ("utf8", pos, lenf, valid)
        else:
            tdt = torch.bool if k == KIND["bool"] else (torch.int64 if k == KIND["decimal"] else f.dtype.torch_dtype)
            data = torch.empty(nrows, dtype=tdt, device=device)
            specs.append((k, f.dtype.scale if k == KIND["decimal"] else 0, ptr(data), 0, ptr(valid)))
            outs[f.name] = ("fixed", data, None, valid)
    cols_dev = torch.frombuffer(bytearray(N.csv_pack_columns(specs)), dtype=torch.uint8).to(device)
    names = b"".join(f.name.encode("utf-8") for f in fields)
    noff = [0]
    for f in fields:
        noff.append(noff[-1] + len(f.name.encode("utf-8")))
    names_dev = torch.frombuffer(bytearray(names + b"\0"), dtype=torch.uint8).to(device)
    noff_dev = torch.tensor(noff, dtype=torch.int32).to(device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    launch("json_parse").json_parse(ptr(buf), 0, ptr(rows_end), nrows, ptr(cols_dev), len(fields), ptr(names_dev),
                                    ptr(noff_dev), ptr(err), s)
    result: Dict[str, Column] = {}
    for f in fields:
        if f.name not in outs:
            continue
        kind, a, b, valid = outs[f.name]
        if kind == "fixed":
            result[f.name] = Column(f.dtype, a, valid)
            continue
        lens = torch.empty(max(nrows, 1), dtype=torch.int64, device=device)
        N.csv_str_lengths(ptr(b), nrows, ptr(lens), s)
        off, total = offsets_from_lengths(lens[:nrows])
        chars = torch.empty(total, dtype=torch.uint8, device=device)
        if total:
            launch("json_str_copy").json_str_copy(ptr(a), ptr(b), ptr(off), nrows, ptr(chars), s)
        result[f.name] = Column(T.UTF8, chars, valid, offsets=off)
    code = int(err.item())
    if code:
        raise JsonParseError(f"{path}: {ERRORS.get(code, code)}")
    for name, c in result.items():
        if c.valid is not None and bool(c.valid.all().item()):
            c.valid = None
    del host
    return result
