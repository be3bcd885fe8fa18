"""sqlite3 oracle for TPC-H results (CPU-side correctness reference).

DataFusion is not installable in this environment, so expected results come
from Python's built-in sqlite3 over the same generated data. The TPC-H text is
rewritten to sqlite's dialect (date arithmetic folded to literals, EXTRACT ->
strftime, SUBSTRING ... FROM ... FOR -> substr). Decimals are compared with a
tolerance (sqlite sums doubles).
"""
from __future__ import annotations

import datetime
import math
import re
import sqlite3
from decimal import Decimal
from typing import Dict, List

import pyarrow as pa

from .queries import QUERIES

_INTERVAL = re.compile(r"date\s+'(\d{4}-\d{2}-\d{2})'\s*([+-])\s*interval\s+'(\d+)'\s+(day|month|year)s?(\s*\(\d+\))?",
                       re.I)


def _shift(d: str, sign: str, n: int, unit: str) -> str:
    dt = datetime.date.fromisoformat(d)
    n = n if sign == "+" else -n
    unit = unit.lower()
    if unit == "day":
        dt = dt + datetime.timedelta(days=n)
    else:
        months = n * (12 if unit == "year" else 1)
        y, m = divmod(dt.month - 1 + months, 12)
        dt = dt.replace(year=dt.year + y, month=m + 1)
    return dt.isoformat()


def to_sqlite(sql: str) -> str:
    s = _INTERVAL.sub(lambda m: f"'{_shift(m.group(1), m.group(2), int(m.group(3)), m.group(4))}'", sql)
    s = re.sub(r"date\s+'(\d{4}-\d{2}-\d{2})'", r"'\1'", s, flags=re.I)
    s = re.sub(r"extract\s*\(\s*year\s+from\s+([\w.]+)\s*\)", r"cast(strftime('%Y', \1) as integer)", s, flags=re.I)
    s = re.sub(r"substring\s*\(\s*([\w.]+)\s+from\s+(\d+)\s+for\s+(\d+)\s*\)", r"substr(\1, \2, \3)", s, flags=re.I)
    # fold decimal constant arithmetic exactly (sqlite would do it in binary floating point)
    s = re.sub(r"(?<![\w.])(\d+\.\d+)\s*([+-])\s*(\d+\.\d+)(?![\w.])",
               lambda m: str(Decimal(m.group(1)) + (Decimal(m.group(3)) if m.group(2) == "+" else -Decimal(m.group(3)))), s)
    return s


INDEXES = [
    "create index i_l_ok on lineitem(l_orderkey)", "create index i_l_pk on lineitem(l_partkey, l_suppkey)",
    "create index i_o_ok on orders(o_orderkey)", "create index i_o_ck on orders(o_custkey)",
    "create index i_ps on partsupp(ps_partkey, ps_suppkey)", "create index i_p on part(p_partkey)",
    "create index i_s on supplier(s_suppkey)", "create index i_c on customer(c_custkey)",
]


def load_sqlite(tables: Dict[str, pa.Table]) -> sqlite3.Connection:
    con = sqlite3.connect(":memory:")
    for name, t in tables.items():
        cols = t.column_names
        con.execute(f"create table {name} ({', '.join(cols)})")
        rows = []
        pyl = [_col_py(t.column(c)) for c in cols]
        rows = list(zip(*pyl)) if pyl else []
        con.executemany(f"insert into {name} values ({', '.join('?' * len(cols))})", rows)
    for ix in INDEXES:
        try:
            con.execute(ix)
        except sqlite3.OperationalError:
            pass
    return con


def _col_py(col) -> list:
    t = col.type
    vals = col.to_pylist()
    if pa.types.is_decimal(t):
        return [None if v is None else float(v) for v in vals]
    if pa.types.is_date(t):
        return [None if v is None else v.isoformat() for v in vals]
    return vals


def run_sqlite(con: sqlite3.Connection, q: int) -> List[tuple]:
    return con.execute(to_sqlite(QUERIES[q])).fetchall()


def normalize(v):
    if isinstance(v, Decimal):
        return float(v)
    if isinstance(v, (datetime.date, datetime.datetime)):
        return v.isoformat()
    return v


def rows_match(a: List[tuple], b: List[tuple], ordered: bool = False, rel: float = 1e-6, abs_: float = 1e-2) -> str:
    """'' if equal (numerics with tolerance), else a description of the first difference."""
    a = [tuple(normalize(x) for x in r) for r in a]
    b = [tuple(normalize(x) for x in r) for r in b]
    if len(a) != len(b):
        return f"row count {len(a)} != {len(b)}"
    if not ordered:
        key = lambda r: tuple((0, round(x, 2)) if isinstance(x, float) else (1, str(x)) for x in r)
        a, b = sorted(a, key=key), sorted(b, key=key)
    for i, (ra, rb) in enumerate(zip(a, b)):
        if len(ra) != len(rb):
            return f"row {i}: width {len(ra)} != {len(rb)}"
        for x, y in zip(ra, rb):
            if isinstance(x, (int, float)) and isinstance(y, (int, float)) and not isinstance(x, bool):
                if not math.isclose(float(x), float(y), rel_tol=rel, abs_tol=abs_):
                    return f"row {i}: {ra} != {rb}"
            elif x != y:
                return f"row {i}: {ra} != {rb}"
    return ""
