"""Physical planner: optimized logical plan -> tree of ExecNodes.

Parity: reference crates/engine/src/physical_planner.rs:13-141 maps only
TableScan / Projection / Filter / Join and returns NotImplemented for
everything else (incl. the EmptyRelation behind ``SELECT 42``); this planner
covers every logical node.
"""
from __future__ import annotations

from ..columnar import Batch
from ..sql import logical as L
from ..utils.errors import NotSupported
from .operators import (ExecContext, ExecNode, FilterExec, FragmentInputExec, HashAggExec, HashJoinExec, LimitExec,
                        MultiJoinExec, ProjectExec, ScanExec, SortExec, UnionExec, ValuesExec)


def create_physical_plan(p: L.Plan) -> ExecNode:
    if isinstance(p, L.Scan):
        return ScanExec(p)
    if isinstance(p, L.Values):
        return ValuesExec(p)
    if isinstance(p, L.Filter):
        return FilterExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Project):
        return ProjectExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Join):
        return HashJoinExec(p, create_physical_plan(p.left), create_physical_plan(p.right))
    if isinstance(p, L.MultiJoin):
        return MultiJoinExec(p, [create_physical_plan(c) for c in p.inputs])
    if isinstance(p, L.Aggregate):
        return HashAggExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Sort):
        return SortExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Limit):
        return LimitExec(p, create_physical_plan(p.input))
    if isinstance(p, L.Union):
        return UnionExec(p, [create_physical_plan(c) for c in p.children])
    if isinstance(p, L.FragmentRef):
        return FragmentInputExec(p)
    raise NotSupported(f"no physical operator for {type(p).__name__}")


def execute_plan(p: L.Plan, ctx: ExecContext) -> Batch:
    return create_physical_plan(p).execute(ctx)
