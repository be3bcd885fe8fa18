"""Order-independent digest of a query result.

Used by ``bench.py`` to check every run against the first (and against the
CPU engine) and by the query-graph layer (exec/graphs.py) to check a graph's
first replay against the eager execution it replaces. Row order is ignored
(hash-built groups come out in any order); float sums are rounded to 9
significant digits (atomic accumulation order varies between runs).
"""
from __future__ import annotations

import decimal
import hashlib


def digest(table) -> str:
    """Row count, exact sums of integer / decimal columns, rounded float sums,
    hashed multiset of the other values."""
    import pyarrow as pa
    import pyarrow.compute as pc
    parts = [str(table.num_rows)]
    for name in table.column_names:
        col = table.column(name)
        t = col.type
        parts.append(f"{name}:{col.null_count}")
        if pa.types.is_integer(t) or pa.types.is_decimal(t):
            s = pc.sum(col).as_py() if table.num_rows else 0
            parts.append(str(decimal.Decimal(s or 0).normalize()))
        elif pa.types.is_floating(t):
            s = pc.sum(col).as_py() if table.num_rows else 0.0
            parts.append(f"{(s or 0.0):.9g}")
        else:
            vals = sorted(str(v) for v in col.to_pylist())
            parts.append(hashlib.sha1("\x1f".join(vals).encode()).hexdigest()[:16])
    return "|".join(parts)
