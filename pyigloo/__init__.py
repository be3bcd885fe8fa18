"""pyigloo — Python bindings for igloo on MI355X.

The reference's pyigloo is a placeholder (an empty cdylib with pyo3 commented
out and a ``2 + 2 == 4`` test: reference pyigloo/src/lib.rs:1,
pyigloo/__init__.py:1, pyigloo/tests/test_sample.py:1-2). Here the package is
the user-facing Python API over the native engine (pybind11 extension
``igloo_amd._native``: SQL parser, gfx950 kernels) and the Flight service:

    import pyigloo
    eng = pyigloo.local()                       # in-process engine on cuda:0 (or CPU)
    eng.register_parquet("t", "data/t.parquet")
    print(eng.sql("SELECT count(*) FROM t"))

    res = eng.sql_device("SELECT a, b FROM t")  # result stays in HBM:
    batch = pyarrow.record_batch(res)           #   Arrow C Device Data Interface (zero copy)
    a = torch.from_dlpack(res.to_dlpack("a"))   #   or DLPack, per column

    with pyigloo.connect("grpc://127.0.0.1:50051") as conn:   # remote coordinator (Flight SQL)
        table = conn.sql("SELECT 42 AS answer")                # -> pyarrow.Table
        conn.get_tables("line%")                               # catalog metadata
        with conn.prepare("SELECT * FROM t WHERE a = ?") as st:
            st.execute([7])

``pyigloo.native`` is the compiled core itself (SQL parser, gfx950 kernel
launchers, device runtime, Arrow C Device exporter).
"""
from __future__ import annotations

from typing import Optional

import igloo_amd as _ig
from igloo_amd import Catalog, MemoryCatalog, MemoryTable, QueryEngine, QueryResult, hello  # noqa: F401
from igloo_amd.utils.errors import IglooError  # noqa: F401

from igloo_amd.interop import DeviceResult  # noqa: F401

__all__ = ["connect", "local", "sql", "sql_device", "Connection", "QueryEngine", "QueryResult", "DeviceResult",
           "Catalog", "MemoryCatalog", "MemoryTable", "IglooError", "hello", "native", "__version__"]
__version__ = getattr(_ig, "__version__", "0.1.0")

_default: Optional[QueryEngine] = None


def local(device: Optional[str] = None, **kw) -> QueryEngine:
    """An in-process engine; ``device`` defaults to cuda:0 when a GPU is visible."""
    if device is None:
        import torch
        device = "cuda:0" if torch.cuda.is_available() else "cpu"
    return QueryEngine(device=device, **kw)


def _engine(engine: Optional[QueryEngine]) -> QueryEngine:
    global _default
    if engine is None:
        if _default is None:
            _default = local()
        engine = _default
    return engine


def sql(query: str, engine: Optional[QueryEngine] = None):
    """Run ``query`` on ``engine`` (or a lazily created default local engine);
    returns a pyarrow.Table."""
    return _engine(engine).query(query)


def sql_device(query: str, engine: Optional[QueryEngine] = None) -> DeviceResult:
    """Run ``query`` and keep the result on the device (zero-copy export)."""
    return _engine(engine).sql_device(query)


def __getattr__(name):
    if name == "native":        # the compiled core, loaded on first use
        from igloo_amd.ops._lib import native as _native
        return _native()
    raise AttributeError(name)


class Connection:
    """Arrow Flight (SQL) connection to a coordinator or worker group."""

    def __init__(self, uri: str = "grpc://127.0.0.1:50051", token: Optional[str] = None, timeout: float = 3600.0):
        from igloo_amd.service.client import IglooClient
        self._client = IglooClient(uri.replace("http://", "grpc://"), token, timeout=timeout)

    def sql(self, query: str, flight_sql: bool = True):
        return self._client.query(query, flight_sql=flight_sql)

    def explain(self, query: str) -> str:
        return self._client.explain(query)

    def tables(self):
        return self._client.tables()

    def get_tables(self, pattern: Optional[str] = None, include_schema: bool = False):
        """Flight SQL CommandGetTables -> pyarrow.Table."""
        return self._client.get_tables(pattern, include_schema=include_schema)

    def sql_info(self, ids=()) -> dict:
        return self._client.sql_info(ids)

    def prepare(self, query: str):
        """A server-side prepared statement (``?`` placeholders)."""
        return self._client.prepare(query)

    def upload(self, name: str, table) -> None:
        self._client.upload(name, table)

    def close(self):
        self._client.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def connect(uri: str = "grpc://127.0.0.1:50051", token: Optional[str] = None, timeout: float = 3600.0) -> Connection:
    return Connection(uri, token, timeout)
