"""Error hierarchy.

Parity: reference crates/common/src/error.rs:6-21 defines
``enum Error { Unknown(String), SqlParser(ParserError) }`` and the engine
panics on every SQL/execution error (crates/engine/src/lib.rs:55-56). Here
every failure is a typed exception instead ("fix: return
error"), and the Flight service maps them to gRPC status codes.
"""
from __future__ import annotations


class IglooError(Exception):
    """Base class (reference ``Error::Unknown``)."""

    code = "UNKNOWN"

    @classmethod
    def new(cls, msg: str) -> "IglooError":  # reference Error::new(&str)
        return cls(msg)


class SqlParseError(IglooError, SyntaxError):
    """SQL text could not be parsed (reference ``Error::SqlParser``)."""

    code = "SQL_PARSE"


class PlanError(IglooError):
    """Name resolution / typing / planning failure."""

    code = "PLAN"


class TableNotFound(PlanError):
    code = "NOT_FOUND"


class NotSupported(IglooError, NotImplementedError):
    code = "NOT_IMPLEMENTED"


class ExecutionError(IglooError):
    code = "EXECUTION"


class IoError(IglooError, OSError):
    code = "IO"


class CommError(IglooError):
    """Collective / RPC failure between coordinator, workers or ranks."""

    code = "COMM"


class DeviceError(IglooError):
    """GPU-side failure, or the native extension is missing on a GPU box."""

    code = "DEVICE"


class CancelledError(IglooError):
    code = "CANCELLED"
