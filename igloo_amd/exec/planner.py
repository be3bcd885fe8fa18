"""Physical planner: optimized logical plan -> tree of ExecNodes.

Parity: reference crates/engine/src/physical_planner.rs:13-141 maps only
TableScan / Projection / Filter / Join and returns NotImplemented for
everything else (incl. the EmptyRelation behind ``SELECT 42``); this planner
covers every logical node.
"""
from __future__ import annotations

from ..columnar import Batch
from ..sql import logical as L
from ..sql.expr import col_refs, has_subquery
from ..utils.errors import NotSupported
from .context import ExecContext, ExecNode
from .scan import FilterExec, FragmentInputExec, ProjectExec, ScanExec, ValuesExec
from .aggregate import HashAggExec
from .joins import HashJoinExec, MultiJoinExec
from .sorting import LimitExec, SortExec, UnionExec


def _require(child: ExecNode, exprs) -> None:
    """Tell a multi-way join which of its columns the parent reads, so index
    parts no remaining condition or output needs stop being carried."""
    if isinstance(child, MultiJoinExec) and not any(has_subquery(e) for e in exprs):
        child.required = set().union(*[col_refs(e) for e in exprs]) if exprs else set()


def create_physical_plan(p: L.Plan) -> ExecNode:
    if isinstance(p, L.Scan):
        return ScanExec(p)
    if isinstance(p, L.Values):
        return ValuesExec(p)
    if isinstance(p, L.Unnest):
        from .scan import UnnestExec
        return UnnestExec(p, create_physical_plan(p.input))
    if isinstance(p, L.TableFunction):
        from .scan import TableFunctionExec
        return TableFunctionExec(p)
    if isinstance(p, L.Filter):
        return FilterExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Project):
        node = ProjectExec(p, create_physical_plan(p.input))
        _require(node.children[0], [e for _, e in p.exprs])
        return node
    if isinstance(p, L.Join):
        return HashJoinExec(p, create_physical_plan(p.left), create_physical_plan(p.right))
    if isinstance(p, L.MultiJoin):
        return MultiJoinExec(p, [create_physical_plan(c) for c in p.inputs])
    if isinstance(p, L.Aggregate):
        node = HashAggExec(p, create_physical_plan(p.input))
        _require(node.children[0], [e for _, e in p.groups] + [a for _, a in p.aggs])
        return node
    if isinstance(p, L.Sort):
        return SortExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Limit):
        return LimitExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Union):
        return UnionExec(p, [create_physical_plan(c) for c in p.children])
    if isinstance(p, L.FragmentRef):
        return FragmentInputExec(p)
    if isinstance(p, L.Window):
        from .window import WindowExec
        node = WindowExec(p, create_physical_plan(p.input))
        _require(node.children[0], [w for _, w in p.wexprs] + [c.ref() for c in p.input.schema])
        return node
    if isinstance(p, L.RecursiveCTE):
        from .window import RecursiveCTEExec
        return RecursiveCTEExec(p, create_physical_plan(p.anchor), create_physical_plan(p.recursive))
    if isinstance(p, L.WorkTableScan):
        from .window import WorkTableExec
        return WorkTableExec(p)
    raise NotSupported(f"no physical operator for {type(p).__name__}")


def execute_plan(p: L.Plan, ctx: ExecContext) -> Batch:
    return create_physical_plan(p).execute(ctx)
