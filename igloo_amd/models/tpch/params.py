"""TPC-H substitution parameters (spec §2.4, the rules qgen follows).

``QUERIES`` holds each query with its *validation* parameters. A TPC-H run
substitutes fresh parameters into every query, so a benchmark that only ever
replays the validation text measures a repeated-identical-query workload.
``query(q, rng)`` returns query ``q`` with parameters drawn by the spec's
rules (seeded ``random.Random``), by textual substitution of the validation
literals; ``rng=None`` returns the validation text.

The reference publishes no benchmark and ships no generator (its data/ is a
placeholder, reference data/sample.parquet); this feeds bench.py
``--vary-params`` (ad-hoc execution: every statement new SQL text).
"""
from __future__ import annotations

import datetime
import random
from typing import Callable, Dict, List, Optional, Tuple

from . import schema as S
from .queries import QUERIES

REGIONS = ["AFRICA", "AMERICA", "ASIA", "EUROPE", "MIDDLE EAST"]
SEGMENTS = ["AUTOMOBILE", "BUILDING", "FURNITURE", "MACHINERY", "HOUSEHOLD"]
TYPE1 = ["STANDARD", "SMALL", "MEDIUM", "LARGE", "ECONOMY", "PROMO"]
TYPE2 = ["ANODIZED", "BURNISHED", "PLATED", "POLISHED", "BRUSHED"]
TYPE3 = ["TIN", "NICKEL", "BRASS", "STEEL", "COPPER"]
CONT1 = ["SM", "LG", "MED", "JUMBO", "WRAP"]
CONT2 = ["CASE", "BOX", "BAG", "JAR", "PKG", "PACK", "CAN", "DRUM"]
MODES = ["REG AIR", "AIR", "RAIL", "SHIP", "TRUCK", "MAIL", "FOB"]
WORD1 = ["special", "pending", "unusual", "express"]
WORD2 = ["packages", "requests", "accounts", "deposits"]


def _nations() -> List[Tuple[str, int]]:
    return list(S.NATIONS)


def _month(rng, y0, m0, y1, m1) -> str:
    """First day of a month drawn uniformly from [y0-m0, y1-m1]."""
    a, b = y0 * 12 + m0 - 1, y1 * 12 + m1 - 1
    k = rng.randint(a, b)
    return f"{k // 12:04d}-{k % 12 + 1:02d}-01"


def _year(rng, y0=1993, y1=1997) -> str:
    return f"{rng.randint(y0, y1)}-01-01"


def _brand(rng) -> str:
    return f"Brand#{rng.randint(1, 5)}{rng.randint(1, 5)}"


def _colors(rng, k: int) -> List[str]:
    return rng.sample(list(S.COLORS), k)


def _subs(q: int, rng: random.Random, sf: float) -> List[Tuple[str, str]]:
    """(validation literal, substituted literal) pairs for query ``q``."""
    nat = _nations()
    if q == 1:
        return [("interval '90' day", f"interval '{rng.randint(60, 120)}' day")]
    if q == 2:
        return [("p_size = 15", f"p_size = {rng.randint(1, 50)}"), ("'%BRASS'", f"'%{rng.choice(TYPE3)}'"),
                ("'EUROPE'", f"'{rng.choice(REGIONS)}'")]
    if q == 3:
        d = datetime.date(1995, 3, rng.randint(1, 31)).isoformat()
        return [("'BUILDING'", f"'{rng.choice(SEGMENTS)}'"), ("'1995-03-15'", f"'{d}'")]
    if q == 4:
        return [("'1993-07-01'", f"'{_month(rng, 1993, 1, 1997, 10)}'")]
    if q == 5:
        return [("'ASIA'", f"'{rng.choice(REGIONS)}'"), ("'1994-01-01'", f"'{_year(rng)}'")]
    if q == 6:
        return [("'1994-01-01'", f"'{_year(rng)}'"), ("0.06 - 0.01", f"0.0{rng.randint(2, 9)} - 0.01"),
                ("0.06 + 0.01", None), ("l_quantity < 24", f"l_quantity < {rng.randint(24, 25)}")]
    if q == 7:
        a, b = rng.sample([n for n, _ in nat], 2)
        return [("'FRANCE'", f"'{a}'"), ("'GERMANY'", f"'{b}'")]
    if q == 8:
        n, r = rng.choice(nat)
        t = f"{rng.choice(TYPE1)} {rng.choice(TYPE2)} {rng.choice(TYPE3)}"
        return [("'BRAZIL'", f"'{n}'"), ("'AMERICA'", f"'{REGIONS[r]}'"), ("'ECONOMY ANODIZED STEEL'", f"'{t}'")]
    if q == 9:
        return [("'%green%'", f"'%{_colors(rng, 1)[0]}%'")]
    if q == 10:
        return [("'1993-10-01'", f"'{_month(rng, 1993, 2, 1995, 1)}'")]
    if q == 11:
        # FRACTION = 0.0001 / SF, written with its significant digits only
        frac = f"{0.0001 / max(sf, 1e-9):.10f}".rstrip("0")
        return [("'GERMANY'", f"'{rng.choice(nat)[0]}'"), ("* 0.0001", f"* {frac}")]
    if q == 12:
        a, b = rng.sample(MODES, 2)
        return [("('MAIL', 'SHIP')", f"('{a}', '{b}')"), ("'1994-01-01'", f"'{_year(rng)}'")]
    if q == 13:
        return [("'%special%requests%'", f"'%{rng.choice(WORD1)}%{rng.choice(WORD2)}%'")]
    if q == 14:
        return [("'1995-09-01'", f"'{_month(rng, 1993, 1, 1997, 12)}'")]
    if q == 15:
        return [("'1996-01-01'", f"'{_month(rng, 1993, 1, 1997, 10)}'")]
    if q == 16:
        sizes = rng.sample(range(1, 51), 8)
        return [("'Brand#45'", f"'{_brand(rng)}'"),
                ("'MEDIUM POLISHED%'", f"'{rng.choice(TYPE1)} {rng.choice(TYPE2)}%'"),
                ("(49, 14, 23, 45, 19, 3, 36, 9)", "(" + ", ".join(map(str, sizes)) + ")")]
    if q == 17:
        return [("'Brand#23'", f"'{_brand(rng)}'"), ("'MED BOX'", f"'{rng.choice(CONT1)} {rng.choice(CONT2)}'")]
    if q == 18:
        return [("> 300", f"> {rng.randint(312, 315)}")]
    if q == 19:
        q1, q2, q3 = rng.randint(1, 10), rng.randint(10, 20), rng.randint(20, 30)
        return [("'Brand#12'", f"'{_brand(rng)}'"), ("'Brand#23'", f"'{_brand(rng)}'"),
                ("'Brand#34'", f"'{_brand(rng)}'"),
                ("l_quantity >= 1 and l_quantity <= 1 + 10", f"l_quantity >= {q1} and l_quantity <= {q1} + 10"),
                ("l_quantity >= 10 and l_quantity <= 10 + 10", f"l_quantity >= {q2} and l_quantity <= {q2} + 10"),
                ("l_quantity >= 20 and l_quantity <= 20 + 10", f"l_quantity >= {q3} and l_quantity <= {q3} + 10")]
    if q == 20:
        return [("'forest%'", f"'{_colors(rng, 1)[0]}%'"), ("'1994-01-01'", f"'{_year(rng)}'"),
                ("'CANADA'", f"'{rng.choice(nat)[0]}'")]
    if q == 21:
        return [("'SAUDI ARABIA'", f"'{rng.choice(nat)[0]}'")]
    if q == 22:
        codes = rng.sample(range(10, 35), 7)
        return [("('13', '31', '23', '29', '30', '18', '17')", "(" + ", ".join(f"'{c}'" for c in codes) + ")")]
    return []


def query(q: int, rng: Optional[random.Random] = None, sf: float = 1.0) -> str:
    """Query ``q`` with substitution parameters drawn from ``rng`` (spec
    §2.4 rules); the validation text when ``rng`` is None."""
    sql = QUERIES[q]
    if rng is None:
        return sql
    subs = _subs(q, rng, sf)
    if q == 6:
        # DISCOUNT +- 0.01: both bounds move together
        lo = subs[1][1].split(" - ")[0]
        subs[2] = ("0.06 + 0.01", f"{lo} + 0.01")
    for old, new in subs:
        if old not in sql:
            raise KeyError(f"Q{q}: validation literal {old!r} not found")
        sql = sql.replace(old, new)
    return sql


def validation(q: int, sf: float = 1.0) -> str:
    """Query ``q`` with the spec's validation parameters at scale factor
    ``sf``: Q11's FRACTION is 0.0001 / SF (the validation text's 0.0001 is
    the SF1 value; at SF100 it would select no rows)."""
    from .queries import QUERIES
    sql = QUERIES[q]
    if q == 11 and sf != 1.0:
        frac = f"{0.0001 / max(sf, 1e-9):.10f}".rstrip("0")
        sql = sql.replace("* 0.0001", f"* {frac}")
    return sql


def stream(qs, seed: int, sf: float = 1.0) -> Dict[int, str]:
    """One query stream: every query of ``qs`` with its own parameters."""
    rng = random.Random(seed)
    return {q: query(q, rng, sf) for q in qs}
