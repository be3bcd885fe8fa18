"""Logical plan IR.

The reference removed its own logical plan (reference
crates/engine/src/logical_plan.rs:1 is one comment) and relies on DataFusion's
``LogicalPlan``; its physical planner only understands TableScan, Projection,
Filter and Join (reference crates/engine/src/physical_planner.rs:28-138).
This IR covers the full SELECT surface: scans with pushed filters, projection,
filter, n-ary inner join groups (ordered adaptively at run time), outer /
semi / anti joins, hash aggregation, sort, limit, union, values.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ..types import DataType
from .expr import AggCall, ColRef, Expr, WindowCall


@dataclass
class ColInfo:
    cid: int
    name: str
    dtype: DataType
    nullable: bool = True
    qualifier: Optional[str] = None

    def ref(self) -> ColRef:
        return ColRef(self.cid, self.name, self.dtype, self.nullable)


class Plan:
    schema: List[ColInfo]

    @property
    def inputs(self) -> List["Plan"]:
        return []

    def with_inputs(self, inputs: List["Plan"]) -> "Plan":
        return self

    def cids(self) -> List[int]:
        return [c.cid for c in self.schema]

    def col(self, cid: int) -> ColInfo:
        for c in self.schema:
            if c.cid == cid:
                return c
        raise KeyError(cid)

    def label(self) -> str:
        return type(self).__name__

    def explain(self, indent: int = 0) -> str:
        lines = ["  " * indent + self.label()]
        for i in self.inputs:
            lines.append(i.explain(indent + 1))
        return "\n".join(lines)


@dataclass(eq=False)
class Scan(Plan):
    table: str
    source: Any                 # catalog TableSource
    schema: List[ColInfo]       # projected columns (cid, name = source column name)
    filters: List[Expr] = field(default_factory=list)

    def label(self):
        f = f" filters=[{', '.join(x.sql() for x in self.filters)}]" if self.filters else ""
        return f"Scan: {self.table} projection=[{', '.join(c.name for c in self.schema)}]{f}"


@dataclass(eq=False)
class Values(Plan):
    rows: List[List[Expr]]
    schema: List[ColInfo]

    def label(self):
        body = "; ".join(", ".join(e.sql() for e in r) for r in self.rows[:4])
        more = f" +{len(self.rows) - 4}" if len(self.rows) > 4 else ""
        return f"Values: {len(self.rows)} rows [{body}{more}]"


@dataclass(eq=False)
class TableFunction(Plan):
    """A table-valued function in FROM: ``generate_series(a, b [, step])``
    (inclusive), ``range(a, b [, step])`` (exclusive) with constant integer
    arguments, or ``unnest(list)`` of a constant list expression (DataFusion's
    datafusion-functions-table, reference Cargo.lock:1146)."""
    name: str
    args: List[Any]
    schema: List[ColInfo]

    def label(self):
        return f"TableFunction: {self.name}({', '.join(a.sql() if hasattr(a, 'sql') else repr(a) for a in self.args)})"


@dataclass(eq=False)
class Unnest(Plan):
    """``SELECT unnest(list_expr), ...``: one row per element of the list
    column ``list_col`` (NULL / empty lists give none); every input column is
    repeated, the element is ``out``."""
    input: Plan
    list_col: ColInfo
    out: ColInfo

    @property
    def schema(self):  # type: ignore[override]
        return self.input.schema + [self.out]

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Unnest(inputs[0], self.list_col, self.out)

    def label(self):
        return f"Unnest: {self.list_col.name}#{self.list_col.cid} -> {self.out.name}#{self.out.cid}"


@dataclass(eq=False)
class Filter(Plan):
    input: Plan
    pred: Expr

    @property
    def schema(self):  # type: ignore[override]
        return self.input.schema

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Filter(inputs[0], self.pred)

    def label(self):
        return f"Filter: {self.pred.sql()}"


@dataclass(eq=False)
class Project(Plan):
    input: Plan
    exprs: List[Tuple[ColInfo, Expr]]

    @property
    def schema(self):  # type: ignore[override]
        return [c for c, _ in self.exprs]

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Project(inputs[0], self.exprs)

    def label(self):
        return "Projection: " + ", ".join(
            e.sql() if isinstance(e, ColRef) and e.cid == c.cid else f"{e.sql()} AS {c.name}#{c.cid}"
            for c, e in self.exprs)


JOIN_KINDS = ("inner", "left", "right", "full", "semi", "anti", "cross")


@dataclass(eq=False)
class Join(Plan):
    left: Plan
    right: Plan
    kind: str
    on: List[Tuple[Expr, Expr]] = field(default_factory=list)   # equi keys (left expr, right expr)
    residual: Optional[Expr] = None                              # extra ON condition
    null_aware: bool = False                                     # NOT IN semantics for anti joins

    @property
    def schema(self):  # type: ignore[override]
        if self.kind in ("semi", "anti"):
            return self.left.schema
        ls = self.left.schema
        rs = self.right.schema
        if self.kind in ("right", "full"):
            ls = [ColInfo(c.cid, c.name, c.dtype, True, c.qualifier) for c in ls]
        if self.kind in ("left", "full"):
            rs = [ColInfo(c.cid, c.name, c.dtype, True, c.qualifier) for c in rs]
        return ls + rs

    @property
    def inputs(self):
        return [self.left, self.right]

    def with_inputs(self, inputs):
        return Join(inputs[0], inputs[1], self.kind, self.on, self.residual, self.null_aware)

    def label(self):
        on = ", ".join(f"{a.sql()} = {b.sql()}" for a, b in self.on)
        r = f" filter={self.residual.sql()}" if self.residual is not None else ""
        return f"Join({self.kind}): on=[{on}]{r}"


@dataclass(eq=False)
class SemiSpec:
    """A semi/anti join whose probe keys all come from ONE MultiJoin input
    (``child``): the executor may apply it to that input before joining (when
    the subquery side is small) or to the joined result."""
    child: int
    right: Plan
    kind: str
    on: List[Tuple[Expr, Expr]]
    residual: Optional[Expr] = None
    null_aware: bool = False

    def sql(self) -> str:
        on = ", ".join(f"{a.sql()} = {b.sql()}" for a, b in self.on)
        r = f" filter={self.residual.sql()}" if self.residual is not None else ""
        return f"{self.kind}@{self.child} on=[{on}]{r}"


@dataclass(eq=False)
class MultiJoin(Plan):
    """N-ary inner join; the executor picks the join order from actual sizes."""
    children: List[Plan]
    conds: List[Expr]  # conjuncts: equi predicates a = b across inputs + residuals
    semis: List[SemiSpec] = field(default_factory=list)

    @property
    def schema(self):  # type: ignore[override]
        out = []
        for c in self.children:
            out += c.schema
        return out

    @property
    def inputs(self):
        return list(self.children) + [s.right for s in self.semis]

    def with_inputs(self, inputs):
        n = len(self.children)
        semis = [SemiSpec(s.child, r, s.kind, s.on, s.residual, s.null_aware) for s, r in zip(self.semis, inputs[n:])]
        return MultiJoin(list(inputs[:n]), self.conds, semis)

    def label(self):
        extra = f", semi=[{'; '.join(s.sql() for s in self.semis)}]" if self.semis else ""
        return f"MultiJoin: {len(self.children)} inputs, conds=[{', '.join(c.sql() for c in self.conds)}]{extra}"


@dataclass(eq=False)
class FragmentRef(Plan):
    """Leaf standing for the materialized output of another query fragment
    (igloo_amd.parallel.fragments)."""
    fragment_id: str
    schema: List[ColInfo]

    def label(self):
        return f"FragmentRef: {self.fragment_id[:8]}"


@dataclass(eq=False)
class Aggregate(Plan):
    input: Plan
    groups: List[Tuple[ColInfo, Expr]]
    aggs: List[Tuple[ColInfo, AggCall]]

    @property
    def schema(self):  # type: ignore[override]
        return [c for c, _ in self.groups] + [c for c, _ in self.aggs]

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Aggregate(inputs[0], self.groups, self.aggs)

    def label(self):
        g = ", ".join(e.sql() for _, e in self.groups)
        a = ", ".join(f"{e.sql()} AS {c.name}#{c.cid}" for c, e in self.aggs)
        return f"Aggregate: groupBy=[{g}], aggr=[{a}]"


@dataclass(eq=False)
class Sort(Plan):
    input: Plan
    keys: List[Tuple[Expr, bool, bool]]  # (expr, ascending, nulls_first)
    fetch: Optional[int] = None          # top-k when a LIMIT sits above

    @property
    def schema(self):  # type: ignore[override]
        return self.input.schema

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Sort(inputs[0], self.keys, self.fetch)

    def label(self):
        k = ", ".join(f"{e.sql()} {'ASC' if a else 'DESC'} NULLS {'FIRST' if nf else 'LAST'}" for e, a, nf in self.keys)
        f = f", fetch={self.fetch}" if self.fetch is not None else ""
        return f"Sort: {k}{f}"


@dataclass(eq=False)
class Limit(Plan):
    input: Plan
    limit: Optional[int]
    offset: int = 0

    @property
    def schema(self):  # type: ignore[override]
        return self.input.schema

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Limit(inputs[0], self.limit, self.offset)

    def label(self):
        return f"Limit: skip={self.offset}, fetch={self.limit}"


@dataclass(eq=False)
class Union(Plan):
    children: List[Plan]
    schema: List[ColInfo]

    @property
    def inputs(self):
        return list(self.children)

    def with_inputs(self, inputs):
        return Union(list(inputs), self.schema)

    def label(self):
        return "Union"


@dataclass(eq=False)
class Window(Plan):
    """Window functions over ``input``: the input's columns plus one column per
    window call (SURVEY E4 "Window"; DataFusion WindowAggExec)."""
    input: Plan
    wexprs: List[Tuple[ColInfo, WindowCall]]

    @property
    def schema(self):  # type: ignore[override]
        return self.input.schema + [c for c, _ in self.wexprs]

    @property
    def inputs(self):
        return [self.input]

    def with_inputs(self, inputs):
        return Window(inputs[0], self.wexprs)

    def label(self):
        return "Window: " + ", ".join(f"{w.sql()} AS {c.name}#{c.cid}" for c, w in self.wexprs)


@dataclass(eq=False)
class WorkTableScan(Plan):
    """The rows of the previous iteration of a recursive CTE (``table_id``)."""
    table_id: int
    schema: List[ColInfo]

    def label(self):
        return f"WorkTable: #{self.table_id} subquery"


@dataclass(eq=False)
class RecursiveCTE(Plan):
    """WITH RECURSIVE: ``anchor`` once, then ``recursive`` over the previous
    iteration's rows (``WorkTableScan(table_id)``) until it yields none;
    ``distinct`` (UNION) drops rows already produced."""
    anchor: Plan
    recursive: Plan
    table_id: int
    schema: List[ColInfo]
    distinct: bool = False
    max_iterations: int = 1000

    @property
    def inputs(self):
        return [self.anchor, self.recursive]

    def with_inputs(self, inputs):
        return RecursiveCTE(inputs[0], inputs[1], self.table_id, self.schema, self.distinct, self.max_iterations)

    def label(self):
        return f"RecursiveCTE: #{self.table_id}{' distinct' if self.distinct else ''} subquery"


def transform_plan(p: Plan, fn) -> Plan:
    """Bottom-up plan rewrite."""
    ins = p.inputs
    if ins:
        new = [transform_plan(i, fn) for i in ins]
        if any(a is not b for a, b in zip(new, ins)):
            p = p.with_inputs(new)
    r = fn(p)
    return p if r is None else r


def walk_plan(p: Plan):
    yield p
    for i in p.inputs:
        yield from walk_plan(i)


def produced_cids(p: Plan) -> set:
    """All column ids defined anywhere inside ``p`` (for correlation analysis)."""
    out = set()
    for n in walk_plan(p):
        out.update(c.cid for c in n.schema)
        if isinstance(n, Project):
            out.update(c.cid for c, _ in n.exprs)
    return out
