"""Logical optimizer.

Rules (in order):
1. decorrelation: EXISTS / IN subqueries become semi/anti joins, correlated
   scalar aggregate subqueries become a grouped aggregate + left join,
   uncorrelated scalar subqueries stay as run-once expressions;
2. predicate pushdown: filters move into scans (fused scan+filter), through
   projections/aggregates/sorts, and into join inputs; trees of inner/cross
   joins are flattened into one ``MultiJoin`` whose order the executor picks
   from actual input sizes at run time;
3. equi-key extraction for outer/semi/anti joins;
4. column pruning: scans load only referenced columns.

The reference delegates all of this to DataFusion's optimizer (reference
crates/engine/src/lib.rs:55; crates/engine/tests/integration_test.rs:82 calls
``into_optimized_plan``).
"""
from __future__ import annotations

from typing import List, Optional, Set, Tuple

from ..types import BOOL
from ..utils.errors import NotSupported, PlanError
from .template import eq_sql, quiet_sql
from .expr import (AggCall, BinOp, ColRef, Expr, Not, SubqueryExpr, and_all, col_refs, conjuncts, has_subquery,
                   replace_cols, transform, walk)
from .logical import (Aggregate, ColInfo, Filter, Join, Limit, MultiJoin, Plan, Project, RecursiveCTE, Scan, SemiSpec,
                      Sort, Union, Values, Window, WorkTableScan, produced_cids, transform_plan, walk_plan)


def optimize(plan: Plan) -> Plan:
    plan = decorrelate(plan)
    plan = push_filters(plan, [])
    plan = transform_plan(plan, _extract_join_keys)
    plan = transform_plan(plan, _attach_semi_joins)
    plan = prune(plan, set(plan.cids()))
    return plan


# =============================================================== decorrelation
def decorrelate(plan: Plan) -> Plan:
    def fn(p: Plan):
        if isinstance(p, Filter) and has_subquery(p.pred):
            return _rewrite_filter(p)
        if isinstance(p, Project) and any(has_subquery(e) for _, e in p.exprs):
            return _rewrite_project(p)
        if isinstance(p, Aggregate) and any(has_subquery(e) for _, e in p.groups):
            raise NotSupported("subqueries in GROUP BY")
        return None
    return transform_plan(plan, fn)


def _normalize_not(c: Expr) -> Expr:
    if isinstance(c, Not) and isinstance(c.x, SubqueryExpr) and c.x.kind in ("exists", "in"):
        s = c.x
        return SubqueryExpr(s.kind, s.plan, s.x, not s.negated, s.dtype, s.outer_refs)
    return c


def _is_correlated(sub: SubqueryExpr) -> bool:
    inner = produced_cids(sub.plan)
    for p in walk_plan(sub.plan):
        for e in _plan_exprs(p):
            if col_refs(e) - inner:
                return True
    return False


def _plan_exprs(p: Plan) -> List[Expr]:
    if isinstance(p, Filter):
        return [p.pred]
    if isinstance(p, Project):
        return [e for _, e in p.exprs]
    if isinstance(p, Aggregate):
        return [e for _, e in p.groups] + [e for _, e in p.aggs]
    if isinstance(p, Join):
        return [x for ab in p.on for x in ab] + ([p.residual] if p.residual is not None else [])
    if isinstance(p, MultiJoin):
        return list(p.conds)
    if isinstance(p, Sort):
        return [e for e, _, _ in p.keys]
    if isinstance(p, Scan):
        return list(p.filters)
    if isinstance(p, Window):
        return [w for _, w in p.wexprs]
    return []


def _rewrite_filter(p: Filter) -> Plan:
    inp = p.input
    remaining: List[Expr] = []
    for c in conjuncts(p.pred):
        c = _normalize_not(c)
        if isinstance(c, SubqueryExpr) and c.kind in ("exists", "in"):
            sub = decorrelate(c.plan)
            inner = produced_cids(sub)
            sub2, corr = _pull_correlated(sub, inner)
            keys, resid = _split_keys(corr, inner)
            if c.kind == "in":
                keys.append((c.x, sub2.schema[0].ref()))
            inp = Join(inp, sub2, "anti" if c.negated else "semi", keys, and_all(resid),
                       null_aware=(c.kind == "in" and c.negated))
            continue
        if has_subquery(c):
            c, inp = _rewrite_scalar_subqueries(c, inp)
        remaining.append(c)
    return Filter(inp, and_all(remaining)) if remaining else inp


def _rewrite_project(p: Project) -> Plan:
    inp = p.input
    exprs = []
    for ci, e in p.exprs:
        if has_subquery(e):
            e, inp = _rewrite_scalar_subqueries(e, inp)
        exprs.append((ci, e))
    return Project(inp, exprs)


def _rewrite_scalar_subqueries(e: Expr, inp: Plan) -> Tuple[Expr, Plan]:
    """Replace correlated scalar subqueries in ``e`` by a column of a left join."""
    state = {"inp": inp}

    def fn(x):
        if not isinstance(x, SubqueryExpr):
            return None
        if x.kind != "scalar":
            raise NotSupported("EXISTS / IN subqueries are only supported as WHERE conjuncts")
        sub = decorrelate(x.plan)
        if not _is_correlated(SubqueryExpr("scalar", sub)):
            # run-once subquery: fully optimise its plan on its own
            return SubqueryExpr("scalar", optimize(sub), None, False, x.dtype, set())
        inner = produced_cids(sub)
        sub2, corr = _pull_correlated(sub, inner, under_agg_ok=True)
        keys, resid = _split_keys(corr, inner)
        if resid:
            raise NotSupported("correlated scalar subquery with non-equality correlation")
        val = sub2.schema[0]
        state["inp"] = Join(state["inp"], sub2, "left", keys)
        return ColRef(val.cid, val.name, val.dtype, True)
    out = transform(e, fn)
    return out, state["inp"]


def _split_keys(corr: List[Expr], inner: Set[int]):
    keys, resid = [], []
    for c in corr:
        if isinstance(c, BinOp) and c.op == "=":
            lr, rr = col_refs(c.left), col_refs(c.right)
            if lr and lr <= inner and not (rr & inner):
                keys.append((c.right, c.left))
                continue
            if rr and rr <= inner and not (lr & inner):
                keys.append((c.left, c.right))
                continue
        resid.append(c)
    return keys, resid


def _pull_correlated(p: Plan, inner: Set[int], under_agg_ok: bool = False) -> Tuple[Plan, List[Expr]]:
    """Remove conjuncts referencing outer columns from ``p``; return them."""
    def is_corr(e):
        return bool(col_refs(e) - inner)

    if isinstance(p, Filter):
        ni, corr = _pull_correlated(p.input, inner, under_agg_ok)
        keep, out = [], []
        for c in conjuncts(p.pred):
            (out if is_corr(c) else keep).append(c)
        np_ = Filter(ni, and_all(keep)) if keep else ni
        return np_, corr + out
    if isinstance(p, Project):
        ni, corr = _pull_correlated(p.input, inner, under_agg_ok)
        if not corr:
            return (p if ni is p.input else Project(ni, p.exprs)), []
        have = {c.cid for c, _ in p.exprs}
        extra = []
        avail = {c.cid: c for c in ni.schema}
        for c in corr:
            for cid in col_refs(c) & inner:
                if cid not in have and cid in avail:
                    ci = avail[cid]
                    extra.append((ci, ci.ref()))
                    have.add(cid)
        return Project(ni, p.exprs + extra), corr
    if isinstance(p, Aggregate):
        ni, corr = _pull_correlated(p.input, inner, under_agg_ok)
        if not corr:
            return (p if ni is p.input else Aggregate(ni, p.groups, p.aggs)), []
        groups = list(p.groups)
        have = {e.cid for _, e in groups if isinstance(e, ColRef)}
        avail = {c.cid: c for c in ni.schema}
        for c in corr:
            if not (isinstance(c, BinOp) and c.op == "="):
                raise NotSupported("non-equality correlation below an aggregate")
            for cid in col_refs(c) & inner:
                if cid not in have:
                    if cid not in avail:
                        raise NotSupported("correlated column not available at aggregate input")
                    ci = avail[cid]
                    groups.append((ColInfo(ci.cid, ci.name, ci.dtype, ci.nullable), ci.ref()))
                    have.add(cid)
        # the pulled predicate now refers to the group output (same cid)
        return Aggregate(ni, groups, p.aggs), corr
    if isinstance(p, Join):
        if p.kind in ("inner", "cross"):
            nl, cl = _pull_correlated(p.left, inner, under_agg_ok)
            nr, cr = _pull_correlated(p.right, inner, under_agg_ok)
            resid = []
            if p.residual is not None:
                for c in conjuncts(p.residual):
                    (cl if is_corr(c) else resid).append(c)
            return Join(nl, nr, p.kind, p.on, and_all(resid)), cl + cr
        nl, cl = _pull_correlated(p.left, inner, under_agg_ok)
        return Join(nl, p.right, p.kind, p.on, p.residual, p.null_aware), cl
    if isinstance(p, MultiJoin):
        kids, corr = [], []
        for ch in p.children:
            n, c = _pull_correlated(ch, inner, under_agg_ok)
            kids.append(n)
            corr += c
        keep = []
        for c in p.conds:
            (corr if is_corr(c) else keep).append(c)
        return MultiJoin(kids, keep), corr
    if isinstance(p, Sort):
        ni, corr = _pull_correlated(p.input, inner, under_agg_ok)
        return Sort(ni, p.keys, p.fetch), corr
    if isinstance(p, Limit):
        ni, corr = _pull_correlated(p.input, inner, under_agg_ok)
        if corr:
            raise NotSupported("correlated subquery with LIMIT")
        return p, []
    return p, []


# ============================================================ filter pushdown
def _wrap(p: Plan, preds: List[Expr]) -> Plan:
    return Filter(p, and_all(preds)) if preds else p


def _flatten_inner(p: Plan, inputs: List[Plan], conds: List[Expr]):
    if isinstance(p, Join) and p.kind in ("inner", "cross"):
        _flatten_inner(p.left, inputs, conds)
        _flatten_inner(p.right, inputs, conds)
        conds += [BinOp("=", a, b, BOOL) for a, b in p.on]
        conds += conjuncts(p.residual)
    elif isinstance(p, MultiJoin):
        for ch in p.children:
            _flatten_inner(ch, inputs, conds)
        conds += p.conds
    else:
        inputs.append(p)


def factor_or(e: Expr) -> List[Expr]:
    """(A and B) or (A and C) -> A and (B or C); returns conjuncts."""
    if not (isinstance(e, BinOp) and e.op == "or"):
        return [e]
    branches = _disjuncts(e)
    conj = [conjuncts(b) for b in branches]
    texts = [[quiet_sql(c) for c in cs] for cs in conj]
    common = [i for i, t in enumerate(texts[0]) if all(t in ts for ts in texts[1:])]
    if not common:
        return [e]      # (for any literal values: leaving the OR as is stays correct)
    keys = {texts[0][i] for i in common}
    # what is factored out must stay equal in every instance of a statement
    # template (sql/template.py eq_sql); other coincidences do not matter
    for cs, ts in zip(conj, texts):
        for c, t in zip(cs, ts):
            if t in keys:
                eq_sql(c)
    rest = [[c for c, t in zip(cs, ts) if t not in keys] for cs, ts in zip(conj, texts)]
    common = [conj[0][i] for i in common]
    if any(not r for r in rest):
        return common  # one branch is exactly the common part: the OR is implied
    ors = and_all(rest[0])
    for r in rest[1:]:
        ors = BinOp("or", ors, and_all(r), ors.dtype)
    return common + [ors]


def _disjuncts(e: Expr) -> List[Expr]:
    if isinstance(e, BinOp) and e.op == "or":
        return _disjuncts(e.left) + _disjuncts(e.right)
    return [e]


def implied_filters(c: Expr, cids: Set[int]) -> Optional[Expr]:
    """From an OR spanning several inputs derive a filter on one input that every
    qualifying row satisfies: OR over branches of each branch's local conjuncts."""
    if not (isinstance(c, BinOp) and c.op == "or"):
        return None
    parts = []
    for b in _disjuncts(c):
        local = [x for x in conjuncts(b) if col_refs(x) and col_refs(x) <= cids]
        if not local:
            return None
        parts.append(and_all(local))
    out = parts[0]
    for x in parts[1:]:
        out = BinOp("or", out, x, out.dtype)
    return out


def push_filters(p: Plan, preds: List[Expr]) -> Plan:
    if preds:
        preds = [x for c in preds for x in factor_or(c)]
    if isinstance(p, Filter):
        return push_filters(p.input, preds + conjuncts(p.pred))
    if isinstance(p, (Join, MultiJoin)) and (isinstance(p, MultiJoin) or p.kind in ("inner", "cross")):
        inputs: List[Plan] = []
        conds: List[Expr] = []
        _flatten_inner(p, inputs, conds)
        conds = conds + preds
        per_child: List[List[Expr]] = [[] for _ in inputs]
        cids = [set(ch.cids()) for ch in inputs]
        multi = []
        for c in conds:
            refs = col_refs(c)
            owners = [i for i, s in enumerate(cids) if refs & s]
            if len(owners) == 1 and refs <= cids[owners[0]] and not _has_outer_only(c):
                per_child[owners[0]].append(c)
            else:
                multi.append(c)
                if len(owners) > 1:
                    for i in owners:
                        imp = implied_filters(c, cids[i])
                        if imp is not None:
                            per_child[i].append(imp)
        kids = [push_filters(ch, per_child[i]) for i, ch in enumerate(inputs)]
        return MultiJoin(kids, multi)
    if isinstance(p, Join):
        lc, rc = set(p.left.cids()), set(p.right.cids())
        lp, rp, above = [], [], []
        for c in preds:
            refs = col_refs(c)
            if refs and refs <= lc and p.kind in ("left", "semi", "anti"):
                lp.append(c)
            elif refs and refs <= rc and p.kind == "right":
                rp.append(c)
            else:
                above.append(c)
        resid = []
        for c in conjuncts(p.residual):
            refs = col_refs(c)
            if refs and refs <= rc and p.kind in ("left", "semi", "anti"):
                rp.append(c)          # ON-only predicate on the non-preserved side
            elif refs and refs <= lc and p.kind == "right":
                lp.append(c)
            else:
                resid.append(c)
        nj = Join(push_filters(p.left, lp), push_filters(p.right, rp), p.kind, p.on, and_all(resid), p.null_aware)
        return _wrap(nj, above)
    if isinstance(p, Project):
        mapping = {ci.cid: e for ci, e in p.exprs}
        down, above = [], []
        for c in preds:
            refs = col_refs(c)
            if refs <= set(mapping) and not any(has_subquery(mapping[r]) or _has_agg(mapping[r]) for r in refs):
                down.append(replace_cols(c, mapping))
            else:
                above.append(c)
        return _wrap(Project(push_filters(p.input, down), p.exprs), above)
    if isinstance(p, Aggregate):
        gmap = {ci.cid: e for ci, e in p.groups}
        down, above = [], []
        for c in preds:
            refs = col_refs(c)
            if refs and refs <= set(gmap):
                down.append(replace_cols(c, gmap))
            else:
                above.append(c)
        return _wrap(Aggregate(push_filters(p.input, down), p.groups, p.aggs), above)
    if isinstance(p, Sort):
        return Sort(push_filters(p.input, preds), p.keys, p.fetch)
    if isinstance(p, Scan):
        pushable = [c for c in preds if not has_subquery(c)]
        rest = [c for c in preds if has_subquery(c)]
        return _wrap(Scan(p.table, p.source, p.schema, p.filters + pushable), rest)
    if isinstance(p, Limit):
        return _wrap(Limit(push_filters(p.input, []), p.limit, p.offset), preds)
    if isinstance(p, Union):
        return _wrap(Union([push_filters(ch, []) for ch in p.children], p.schema), preds)
    if isinstance(p, Window):
        # a predicate on keys every window call partitions by keeps whole
        # partitions: it may run before the window functions
        common = None
        for _, w in p.wexprs:
            ks = {e.cid for e in w.partition if isinstance(e, ColRef)}
            common = ks if common is None else common & ks
        down, above = [], []
        for c in preds:
            refs = col_refs(c)
            (down if refs and common and refs <= common and not has_subquery(c) else above).append(c)
        return _wrap(Window(push_filters(p.input, down), p.wexprs), above)
    if isinstance(p, RecursiveCTE):
        return _wrap(RecursiveCTE(push_filters(p.anchor, []), push_filters(p.recursive, []), p.table_id, p.schema,
                                  p.distinct, p.max_iterations), preds)
    return _wrap(p, preds)


def _has_outer_only(c: Expr) -> bool:
    return False


def _has_agg(e: Expr) -> bool:
    return any(isinstance(x, AggCall) for x in walk(e))


# ============================================================ join keys
def _extract_join_keys(p: Plan):
    if not isinstance(p, Join) or p.kind in ("inner", "cross") or p.residual is None:
        return None
    lc, rc = set(p.left.cids()), set(p.right.cids())
    keys = list(p.on)
    resid = []
    for c in conjuncts(p.residual):
        if isinstance(c, BinOp) and c.op == "=":
            a, b = col_refs(c.left), col_refs(c.right)
            if a and b and a <= lc and b <= rc:
                keys.append((c.left, c.right))
                continue
            if a and b and a <= rc and b <= lc:
                keys.append((c.right, c.left))
                continue
        resid.append(c)
    return Join(p.left, p.right, p.kind, keys, and_all(resid), p.null_aware)


# ============================================================ semi-join placement
def _attach_semi_joins(p: Plan):
    """Semi/anti join over a MultiJoin whose probe side only needs one input:
    record it on the MultiJoin so the executor can filter that input first
    (e.g. TPC-H Q18: ``o_orderkey IN (<57 keys>)`` shrinks orders before the
    600M-row lineitem join) or, when the subquery side is large, after the join."""
    if not (isinstance(p, Join) and p.kind in ("semi", "anti") and isinstance(p.left, MultiJoin)):
        return None
    mj = p.left
    rc = set(p.right.cids())
    need = _refs([a for a, _ in p.on]) | (_refs([p.residual]) - rc)
    if not need:
        return None
    for i, ch in enumerate(mj.children):
        if need <= set(ch.cids()):
            spec = SemiSpec(i, p.right, p.kind, list(p.on), p.residual, p.null_aware)
            return MultiJoin(mj.children, mj.conds, mj.semis + [spec])
    return None


# ============================================================ column pruning
def _refs(exprs) -> Set[int]:
    out: Set[int] = set()
    for e in exprs:
        if e is not None:
            out |= col_refs(e)
    return out


def prune(p: Plan, required: Set[int]) -> Plan:
    if isinstance(p, Scan):
        keep = [c for c in p.schema if c.cid in required]
        s = Scan(p.table, p.source, keep, p.filters)
        s.table_cols = getattr(p, "table_cols", p.schema)  # type: ignore[attr-defined]
        return s
    if isinstance(p, Values):
        return p
    if isinstance(p, Filter):
        return Filter(prune(p.input, required | col_refs(p.pred)), p.pred)
    if isinstance(p, Project):
        exprs = [(c, e) for c, e in p.exprs if c.cid in required]
        return Project(prune(p.input, _refs(e for _, e in exprs)), exprs)
    if isinstance(p, Join):
        need = required | _refs([x for ab in p.on for x in ab] + [p.residual])
        return Join(prune(p.left, need & set(p.left.cids())), prune(p.right, need & set(p.right.cids())),
                    p.kind, p.on, p.residual, p.null_aware)
    if isinstance(p, MultiJoin):
        need = required | _refs(p.conds)
        semis = []
        for sp in p.semis:
            rc = set(sp.right.cids())
            sneed = _refs([x for ab in sp.on for x in ab] + [sp.residual])
            need |= sneed - rc
            semis.append(SemiSpec(sp.child, prune(sp.right, sneed & rc), sp.kind, sp.on, sp.residual, sp.null_aware))
        return MultiJoin([prune(ch, need & set(ch.cids())) for ch in p.children], p.conds, semis)
    if isinstance(p, Aggregate):
        aggs = [(c, a) for c, a in p.aggs if c.cid in required]
        need = _refs([e for _, e in p.groups]) | _refs(a for _, a in aggs)
        return Aggregate(prune(p.input, need), p.groups, aggs)
    if isinstance(p, Sort):
        return Sort(prune(p.input, required | _refs(e for e, _, _ in p.keys)), p.keys, p.fetch)
    if isinstance(p, Limit):
        return Limit(prune(p.input, required), p.limit, p.offset)
    if isinstance(p, Union):
        return Union([prune(ch, set(ch.cids())) for ch in p.children], p.schema)
    if isinstance(p, Window):
        wexprs = [(c, w) for c, w in p.wexprs if c.cid in required]
        in_cids = set(p.input.cids())
        need = (required & in_cids) | _refs(w for _, w in wexprs)
        if not wexprs:
            return prune(p.input, need)
        return Window(prune(p.input, need), wexprs)
    if isinstance(p, RecursiveCTE):
        return RecursiveCTE(prune(p.anchor, set(p.anchor.cids())), prune(p.recursive, set(p.recursive.cids())),
                            p.table_id, p.schema, p.distinct, p.max_iterations)
    return p
