"""Bound (typed, name-resolved) expressions.

Columns are referenced by globally unique integer ids (``cid``) assigned by
the binder, so plans can be rewritten (pushdown, decorrelation, join
reordering) without name clashes. Parity: replaces the DataFusion ``Expr`` /
``PhysicalExpr`` trees the reference evaluates per batch
(reference crates/engine/src/operators/filter.rs:47, projection.rs:60-64).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, List, Optional, Sequence, Set, Tuple

from ..types import BOOL, DataType


class Expr:
    dtype: DataType
    nullable: bool = True

    def children(self) -> List["Expr"]:
        return []

    def with_children(self, kids: List["Expr"]) -> "Expr":
        return self

    def __repr__(self) -> str:
        return self.sql()

    def sql(self) -> str:  # pragma: no cover - overridden
        return type(self).__name__


@dataclass(eq=False)
class ColRef(Expr):
    cid: int
    name: str
    dtype: DataType
    nullable: bool = True

    def sql(self) -> str:
        return f"{self.name}#{self.cid}"


@dataclass(eq=False)
class Lit(Expr):
    """Literal. Decimals hold the unscaled int, dates days since epoch."""
    value: Any
    dtype: DataType

    @property
    def nullable(self) -> bool:  # type: ignore[override]
        return self.value is None

    def sql(self) -> str:
        if self.value is None:
            return "NULL"
        if self.dtype.is_decimal:
            s = self.dtype.scale
            v = self.value
            sign = "-" if v < 0 else ""
            v = abs(v)
            return f"{sign}{v // 10**s}.{str(v % 10**s).zfill(s)}" if s else f"{sign}{v}"
        if self.dtype.kind == "date32":
            import datetime
            return f"DATE '{datetime.date(1970, 1, 1) + datetime.timedelta(days=self.value)}'"
        if isinstance(self.value, str):
            return "'" + self.value.replace("'", "''") + "'"
        return str(self.value)


@dataclass(eq=False)
class BinOp(Expr):
    op: str  # + - * / % = <> < <= > >= and or ||
    left: Expr
    right: Expr
    dtype: DataType

    @property
    def nullable(self) -> bool:  # type: ignore[override]
        return self.left.nullable or self.right.nullable or self.op in ("/", "%")

    def children(self):
        return [self.left, self.right]

    def with_children(self, kids):
        return BinOp(self.op, kids[0], kids[1], self.dtype)

    def sql(self):
        return f"({self.left.sql()} {self.op.upper() if self.op in ('and', 'or') else self.op} {self.right.sql()})"


@dataclass(eq=False)
class Not(Expr):
    x: Expr
    dtype: DataType = BOOL

    @property
    def nullable(self):  # type: ignore[override]
        return self.x.nullable

    def children(self):
        return [self.x]

    def with_children(self, kids):
        return Not(kids[0])

    def sql(self):
        return f"NOT {self.x.sql()}"


@dataclass(eq=False)
class Neg(Expr):
    x: Expr
    dtype: DataType

    @property
    def nullable(self):  # type: ignore[override]
        return self.x.nullable

    def children(self):
        return [self.x]

    def with_children(self, kids):
        return Neg(kids[0], self.dtype)

    def sql(self):
        return f"(-{self.x.sql()})"


@dataclass(eq=False)
class IsNull(Expr):
    x: Expr
    negated: bool = False
    dtype: DataType = BOOL
    nullable: bool = False

    def children(self):
        return [self.x]

    def with_children(self, kids):
        return IsNull(kids[0], self.negated)

    def sql(self):
        return f"{self.x.sql()} IS {'NOT ' if self.negated else ''}NULL"


@dataclass(eq=False)
class Cast(Expr):
    x: Expr
    dtype: DataType

    @property
    def nullable(self):  # type: ignore[override]
        return self.x.nullable

    def children(self):
        return [self.x]

    def with_children(self, kids):
        return Cast(kids[0], self.dtype)

    def sql(self):
        return f"CAST({self.x.sql()} AS {self.dtype})"


@dataclass(eq=False)
class Case(Expr):
    whens: List[Tuple[Expr, Expr]]
    else_: Optional[Expr]
    dtype: DataType

    def children(self):
        out = []
        for c, v in self.whens:
            out += [c, v]
        if self.else_ is not None:
            out.append(self.else_)
        return out

    def with_children(self, kids):
        n = len(self.whens)
        whens = [(kids[2 * i], kids[2 * i + 1]) for i in range(n)]
        return Case(whens, kids[2 * n] if self.else_ is not None else None, self.dtype)

    def sql(self):
        w = " ".join(f"WHEN {c.sql()} THEN {v.sql()}" for c, v in self.whens)
        e = f" ELSE {self.else_.sql()}" if self.else_ is not None else ""
        return f"CASE {w}{e} END"


@dataclass(eq=False)
class InList(Expr):
    x: Expr
    values: List[Expr]
    negated: bool = False
    dtype: DataType = BOOL

    @property
    def nullable(self):  # type: ignore[override]
        return self.x.nullable

    def children(self):
        return [self.x] + list(self.values)

    def with_children(self, kids):
        return InList(kids[0], kids[1:], self.negated)

    def sql(self):
        return f"{self.x.sql()} {'NOT ' if self.negated else ''}IN ({', '.join(v.sql() for v in self.values)})"


@dataclass(eq=False)
class Like(Expr):
    x: Expr
    pattern: str
    negated: bool = False
    case_insensitive: bool = False
    escape: Optional[str] = "\\"
    dtype: DataType = BOOL

    @property
    def nullable(self):  # type: ignore[override]
        return self.x.nullable

    def children(self):
        return [self.x]

    def with_children(self, kids):
        return Like(kids[0], self.pattern, self.negated, self.case_insensitive, self.escape)

    def sql(self):
        op = "ILIKE" if self.case_insensitive else "LIKE"
        return f"{self.x.sql()} {'NOT ' if self.negated else ''}{op} '{self.pattern}'"


@dataclass(eq=False)
class Func(Expr):
    name: str
    args: List[Expr]
    dtype: DataType
    options: Tuple = ()

    def children(self):
        return list(self.args)

    def with_children(self, kids):
        return Func(self.name, kids, self.dtype, self.options)

    def sql(self):
        opt = f"[{','.join(map(str, self.options))}]" if self.options else ""
        return f"{self.name}{opt}({', '.join(a.sql() for a in self.args)})"


AGG_FUNCS = {"sum", "count", "avg", "min", "max", "mean", "stddev", "var", "bool_and", "bool_or", "first_value",
             "array_agg", "count_distinct"}


@dataclass(eq=False)
class AggCall(Expr):
    func: str           # sum count avg min max median percentile string_agg covar_* corr ...
    arg: Optional[Expr]  # None for COUNT(*)
    distinct: bool
    dtype: DataType
    filter: Optional[Expr] = None
    arg2: Optional[Expr] = None   # second argument (covar / corr)
    param: Any = None             # constant parameter (percentile fraction, string_agg separator)
    #: ordered aggregates (array_agg / string_agg ... ORDER BY): (expr, ascending, nulls_first)
    order: Tuple = ()

    def children(self):
        out = [] if self.arg is None else [self.arg]
        if self.arg2 is not None:
            out.append(self.arg2)
        out += [e for e, _, _ in self.order]
        if self.filter is not None:
            out.append(self.filter)
        return out

    def with_children(self, kids):
        k = 0
        arg = arg2 = None
        if self.arg is not None:
            arg, k = kids[0], 1
        if self.arg2 is not None:
            arg2, k = kids[k], k + 1
        order = tuple((kids[k + i], a, nf) for i, (_, a, nf) in enumerate(self.order))
        flt = kids[-1] if self.filter is not None else None
        return AggCall(self.func, arg, self.distinct, self.dtype, flt, arg2, self.param, order)

    def sql(self):
        a = "*" if self.arg is None else (("DISTINCT " if self.distinct else "") + self.arg.sql())
        if self.arg2 is not None:
            a += ", " + self.arg2.sql()
        if self.param is not None:
            a += f", {self.param!r}"
        if self.order:
            a += " ORDER BY " + ", ".join(f"{e.sql()} {'ASC' if asc else 'DESC'} NULLS {'FIRST' if nf else 'LAST'}"
                                          for e, asc, nf in self.order)
        return f"{self.func.upper()}({a})"


#: window-function frame bound kinds (sql order: a frame's start never comes after its end)
FRAME_KINDS = ("unbounded_preceding", "preceding", "current", "following", "unbounded_following")
RANKING_FUNCS = ("row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile")
VALUE_FUNCS = ("lag", "lead", "first_value", "last_value", "nth_value")


@dataclass(eq=False)
class WindowFrame:
    """ROWS / RANGE / GROUPS frame: bound kinds (FRAME_KINDS) and offsets
    (``Lit`` in the ORDER BY key's representation for RANGE, int otherwise)."""
    unit: str
    start: str
    end: str
    start_off: Any = None
    end_off: Any = None

    def sql(self) -> str:
        def b(kind, off):
            if kind in ("preceding", "following"):
                v = off.sql() if isinstance(off, Lit) else str(off)
                return f"{v} {kind.upper()}"
            return kind.replace("_", " ").upper().replace("CURRENT", "CURRENT ROW")
        return f"{self.unit.upper()} BETWEEN {b(self.start, self.start_off)} AND {b(self.end, self.end_off)}"


@dataclass(eq=False)
class WindowCall(Expr):
    """``func(args) [FILTER (WHERE f)] OVER (PARTITION BY .. ORDER BY .. frame)``.
    Aggregates (sum/count/avg/min/max/stddev/var/bool_*), ranking functions
    and value functions; ``options`` holds constant arguments (ntile buckets,
    lag/lead offset, nth_value position)."""
    func: str
    args: List[Expr]
    partition: List[Expr]
    order: List[Tuple[Expr, bool, bool]]   # (expr, ascending, nulls_first)
    frame: WindowFrame
    dtype: DataType
    filter: Optional[Expr] = None
    options: Tuple = ()

    @property
    def nullable(self) -> bool:  # type: ignore[override]
        return self.func not in ("row_number", "rank", "dense_rank", "percent_rank", "cume_dist", "ntile", "count")

    def children(self):
        out = list(self.args) + list(self.partition) + [e for e, _, _ in self.order]
        if self.filter is not None:
            out.append(self.filter)
        return out

    def with_children(self, kids):
        na, np_ = len(self.args), len(self.partition)
        no = len(self.order)
        args = kids[:na]
        part = kids[na:na + np_]
        order = [(k, a, nf) for k, (_, a, nf) in zip(kids[na + np_:na + np_ + no], self.order)]
        flt = kids[na + np_ + no] if self.filter is not None else None
        return WindowCall(self.func, list(args), list(part), order, self.frame, self.dtype, flt, self.options)

    def spec_sql(self) -> str:
        p = ", ".join(e.sql() for e in self.partition)
        o = ", ".join(f"{e.sql()} {'ASC' if a else 'DESC'} NULLS {'FIRST' if nf else 'LAST'}" for e, a, nf in self.order)
        return (f"PARTITION BY {p} " if p else "") + (f"ORDER BY {o}" if o else "")

    def sql(self):
        opt = f"[{','.join(map(str, self.options))}]" if self.options else ""
        f = f" FILTER (WHERE {self.filter.sql()})" if self.filter is not None else ""
        return (f"{self.func}{opt}({', '.join(a.sql() for a in self.args)}){f} OVER "
                f"({self.spec_sql()} {self.frame.sql()})")


@dataclass(eq=False)
class SubqueryExpr(Expr):
    """Unresolved subquery in an expression: kind in {scalar, exists, in}."""
    kind: str
    plan: Any  # logical Plan
    x: Optional[Expr] = None
    negated: bool = False
    dtype: DataType = BOOL
    outer_refs: Set[int] = field(default_factory=set)

    def children(self):
        return [self.x] if self.x is not None else []

    def with_children(self, kids):
        return SubqueryExpr(self.kind, self.plan, kids[0] if kids else None, self.negated, self.dtype, self.outer_refs)

    def sql(self):
        inner = f"<subquery#{id(self.plan) % 10000}>"
        if self.kind == "exists":
            return f"{'NOT ' if self.negated else ''}EXISTS {inner}"
        if self.kind == "in":
            return f"{self.x.sql()} {'NOT ' if self.negated else ''}IN {inner}"
        return inner


# ---------------------------------------------------------------------- helpers
def walk(e: Expr) -> Iterable[Expr]:
    stack = [e]
    while stack:
        x = stack.pop()
        yield x
        stack.extend(x.children())


def transform(e: Expr, fn: Callable[[Expr], Optional[Expr]]) -> Expr:
    """Bottom-up rewrite: fn returns a replacement or None to keep."""
    kids = e.children()
    if kids:
        new = [transform(k, fn) for k in kids]
        if any(a is not b for a, b in zip(new, kids)):
            e = e.with_children(new)
    r = fn(e)
    return e if r is None else r


def col_refs(e: Expr) -> Set[int]:
    """Column ids ``e`` reads. Remembered on the expression object (bound
    expressions are not mutated: rewrites build new nodes), since a cached
    plan's operators ask again on every execution (join edges, prefetch
    lists): a frozenset, callers do not modify it."""
    r = e.__dict__.get("_igloo_refs") if hasattr(e, "__dict__") else None
    if r is None:
        r = frozenset(x.cid for x in walk(e) if isinstance(x, ColRef))
        try:
            e._igloo_refs = r
        except AttributeError:
            pass
    return r


def has_subquery(e: Expr) -> bool:
    return any(isinstance(x, SubqueryExpr) for x in walk(e))


def has_agg(e: Expr) -> bool:
    return any(isinstance(x, AggCall) for x in walk(e))


def has_window(e: Expr) -> bool:
    return any(isinstance(x, WindowCall) for x in walk(e))


def conjuncts(e: Optional[Expr]) -> List[Expr]:
    if e is None:
        return []
    if isinstance(e, BinOp) and e.op == "and":
        return conjuncts(e.left) + conjuncts(e.right)
    return [e]


def and_all(es: Sequence[Expr]) -> Optional[Expr]:
    out = None
    for x in es:
        out = x if out is None else BinOp("and", out, x, BOOL)
    return out


def replace_cols(e: Expr, mapping: dict) -> Expr:
    """Replace ColRef(cid) by mapping[cid] (an Expr)."""
    def fn(x):
        if isinstance(x, ColRef) and x.cid in mapping:
            return mapping[x.cid]
        return None
    return transform(e, fn)


def same_expr(a: Expr, b: Expr) -> bool:
    return a.sql() == b.sql()
