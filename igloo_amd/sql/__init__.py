"""SQL frontend: native parser (csrc/sql) -> binder -> optimizer."""
from __future__ import annotations

from typing import List

from ..utils.errors import SqlParseError


def parse(sql: str) -> List[dict]:
    """Parse SQL text into statement ASTs with the native recursive-descent parser.

    Parity: reference crates/engine/src/parser.rs:7-12 ``parse_sql`` returns the
    LAST statement and panics on empty input; here all statements are returned and
    errors raise ``SqlParseError``."""
    from ..ops._lib import native
    try:
        return native().parse_sql(sql)
    except SyntaxError as e:
        raise SqlParseError(str(e)) from None


def parse_sql(sql: str) -> dict:
    """Reference-compatible: the last statement of ``sql``."""
    stmts = parse(sql)
    if not stmts:
        raise SqlParseError("empty SQL statement")
    return stmts[-1]
