"""igloo_amd — MI355X-native distributed SQL query engine.

A from-scratch re-design of igloo-io/igloo for AMD Instinct MI355X (gfx950):
native C++ SQL frontend, hand-written CDNA4 HIP kernels for every physical
operator, RCCL (torch.distributed "nccl") exchanges over xGMI between
one-process-per-GPU workers, Arrow Flight service, connectors, tiered cache.
"""
from __future__ import annotations

import torch  # noqa: F401  (must load first: the native extension binds to torch's HIP runtime)

from .catalog import Catalog, Field, MemoryCatalog, MemoryTable, TableSource
from .columnar import Batch, Column
from .engine import QueryEngine, QueryResult, pretty_format, print_batches
from .utils.errors import (CommError, DeviceError, ExecutionError, IglooError, IoError, NotSupported, PlanError,
                           SqlParseError, TableNotFound)

__version__ = "0.1.0"


def hello() -> str:
    """Reference crates/igloo/src/lib.rs:4-6."""
    return "Hello from Igloo Crate!"


__all__ = ["QueryEngine", "QueryResult", "Catalog", "MemoryCatalog", "MemoryTable", "TableSource", "Field", "Column",
           "Batch", "IglooError", "SqlParseError", "PlanError", "TableNotFound", "NotSupported", "ExecutionError",
           "IoError", "CommError", "DeviceError", "hello", "print_batches", "pretty_format"]
