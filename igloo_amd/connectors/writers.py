"""Result writers for ``COPY ... TO`` (Parquet, CSV, NDJSON, Arrow IPC).

Parity: DataFusion's COPY statement (reference Cargo.lock:1329
datafusion-sql; the file sinks of datafusion-datasource-parquet / -csv /
-json). The query runs on the device; the Arrow result is encoded on the
host (file encoding is I/O bound: one pass over the result).
"""
from __future__ import annotations

import json as _json
from typing import Dict

import pyarrow as pa

from ..utils.errors import NotSupported, PlanError


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def write_table(tab: pa.Table, path: str, fmt: str, opts: Dict[str, str]) -> None:
    fmt = fmt.upper()
    if fmt == "PARQUET":
        import pyarrow.parquet as pq
        comp = opts.get("compression", opts.get("format.compression", "zstd")).lower()
        if comp.startswith("zstd"):
            comp = "zstd"
        pq.write_table(tab, path, compression=None if comp in ("none", "uncompressed") else comp)
    elif fmt == "CSV":
        import pyarrow.csv as pc
        header = _bool(opts.get("format.has_header", opts.get("header", "true")))
        delim = opts.get("format.delimiter", opts.get("delimiter", ","))
        if len(delim) != 1:
            raise PlanError("COPY: the CSV delimiter must be one character")
        pc.write_csv(tab, path, write_options=pc.WriteOptions(include_header=header, delimiter=delim))
    elif fmt in ("JSON", "NDJSON"):
        cols = tab.column_names
        with open(path, "w") as f:
            for row in tab.to_pylist():
                f.write(_json.dumps({c: _jsonable(row[c]) for c in cols}, separators=(",", ":")) + "\n")
    elif fmt in ("ARROW", "IPC"):
        with pa.OSFile(path, "wb") as sink, pa.ipc.new_file(sink, tab.schema) as w:
            w.write_table(tab)
    else:
        raise NotSupported(f"COPY ... STORED AS {fmt}")


def _jsonable(v):
    import datetime
    import decimal
    if isinstance(v, decimal.Decimal):
        return float(v)
    if isinstance(v, (datetime.date, datetime.datetime)):
        return v.isoformat()
    if isinstance(v, bytes):
        return v.hex()
    if isinstance(v, list):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {k: _jsonable(x) for k, x in v.items()}
    return v
