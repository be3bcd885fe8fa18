"""Binder: native AST -> typed logical plan.

Resolves names against the catalog and enclosing scopes (correlated
subqueries), types and coerces expressions (DataFusion-compatible rules for
the TPC-H surface: exact decimals, DATE/INTERVAL arithmetic, string/date
literal coercion), and analyses aggregation (GROUP BY / HAVING / ORDER BY on
aggregates, DISTINCT). Parity: this is the SqlToRel stage the reference gets
from DataFusion via ``ctx.sql()`` (reference crates/engine/src/lib.rs:55).
"""
from __future__ import annotations

import datetime
import itertools
from decimal import Decimal
from typing import Any, Dict, List, Optional, Sequence, Tuple

from .. import types as T
from . import template as TPL
from ..types import BOOL, DATE32, FLOAT64, INT32, INT64, UTF8, DataType
from ..utils.errors import NotSupported, PlanError, TableNotFound
from .expr import (AGG_FUNCS, FRAME_KINDS, RANKING_FUNCS, VALUE_FUNCS, AggCall, BinOp, Case, Cast, ColRef, Expr,
                   Func, InList, IsNull, Like, Lit, Neg, Not, SubqueryExpr, WindowCall, WindowFrame, and_all, col_refs,
                   transform, walk)
from .logical import (Aggregate, ColInfo, Filter, Join, Limit, Plan, Project, RecursiveCTE, Scan, Sort, Union, Values,
                      TableFunction, Unnest, Window, WorkTableScan)

EPOCH = datetime.date(1970, 1, 1)

import contextvars as _cv

#: values of ``$n`` parameters while an EXECUTE binds its prepared statement
PARAMS: "_cv.ContextVar[Optional[List[Lit]]]" = _cv.ContextVar("igloo_params", default=None)
INTERVAL = DataType("interval")


def date_to_days(s: str) -> int:
    try:
        return (datetime.date.fromisoformat(s.strip()[:10]) - EPOCH).days
    except ValueError as e:
        raise PlanError(f"invalid date literal '{s}'") from e


def days_to_date(d: int) -> datetime.date:
    return EPOCH + datetime.timedelta(days=int(d))


def add_months(days: int, months: int) -> int:
    d = days_to_date(days)
    y, m = divmod(d.month - 1 + months, 12)
    y += d.year
    m += 1
    import calendar
    day = min(d.day, calendar.monthrange(y, m)[1])
    return (datetime.date(y, m, day) - EPOCH).days


class IdGen:
    def __init__(self, start: int = 1):
        self._it = itertools.count(start)

    def __call__(self) -> int:
        return next(self._it)


# ------------------------------------------------------------------------ scopes
class Relation:
    def __init__(self, qualifier: Optional[str], cols: List[ColInfo]):
        self.qualifier = qualifier
        self.cols = cols


class Scope:
    def __init__(self, rels: List[Relation], parent: Optional["Scope"] = None):
        self.rels = rels
        self.parent = parent
        self.aliases: Dict[str, ColRef] = {}  # select-list aliases visible to ORDER BY / HAVING
        self.outer_refs: set = set()          # cids of outer columns referenced from this scope

    def lookup_local(self, parts: List[str]) -> List[ColInfo]:
        name = parts[-1]
        qual = ".".join(parts[:-1]) if len(parts) > 1 else None
        found = []
        for r in self.rels:
            if qual is not None:
                rq = r.qualifier or ""
                if rq != qual and rq.split(".")[-1] != qual.split(".")[-1]:
                    continue
            for c in r.cols:
                if c.name == name:
                    found.append(c)
        return found

    def resolve(self, parts: List[str]) -> Tuple[ColInfo, int]:
        scope, depth = self, 0
        while scope is not None:
            found = scope.lookup_local(parts)
            if len(found) > 1:
                # same cid visible twice (USING / NATURAL joins) is fine
                if len({c.cid for c in found}) > 1:
                    raise PlanError(f"ambiguous column reference '{'.'.join(parts)}'")
            if found:
                return found[0], depth
            scope, depth = scope.parent, depth + 1
        raise PlanError(f"column '{'.'.join(parts)}' not found")


# ------------------------------------------------------------------- statements
class BoundQuery:
    def __init__(self, plan: Plan, names: List[str]):
        self.plan = plan
        self.names = names


def _lst(node) -> list:
    return node["c"] if node else []


class Binder:
    def __init__(self, catalog, ids: Optional[IdGen] = None, session: Optional[dict] = None):
        self.catalog = catalog
        self.ids = ids or IdGen()
        self.session = session or {}

    # =================================================================== query
    def bind_query(self, q: dict, outer: Optional[Scope] = None, ctes: Optional[dict] = None) -> BoundQuery:
        ctes = dict(ctes or {})
        for c in _lst(q.get("with")):
            rec = bool(q.get("recursive")) and _is_recursive_cte(c)
            ctes[c["s"]] = (c, dict(ctes), rec)
        prev = getattr(self, "_ctes", None)
        self._ctes = ctes
        try:
            return self._bind_query_inner(q, outer, ctes)
        finally:
            self._ctes = prev

    def _bind_query_inner(self, q: dict, outer: Optional[Scope], ctes: dict) -> BoundQuery:
        order = _lst(q.get("order"))
        limit = self._const_int(q.get("limit")) if q.get("limit") else None
        offset = self._const_int(q.get("offset")) if q.get("offset") else 0
        body = q["body"]
        if body["k"] == "select":
            bq = self._bind_select(body, outer, ctes, order)
        else:
            bq = self._bind_setop(body, outer, ctes)
            if order:
                bq = self._order_over_output(bq, order)
        plan = bq.plan
        if limit is not None or offset:
            if isinstance(plan, Sort) and limit is not None:
                plan = Sort(plan.input, plan.keys, fetch=limit + offset)
            elif isinstance(plan, Project) and isinstance(plan.input, Sort) and limit is not None:
                s = plan.input
                plan = Project(Sort(s.input, s.keys, fetch=limit + offset), plan.exprs)
            plan = Limit(plan, limit, offset)
        return BoundQuery(plan, bq.names)

    def _const_int(self, node) -> int:
        e = self.bind_expr(node, Scope([]))
        if not isinstance(e, Lit) or not isinstance(e.value, int):
            raise PlanError("LIMIT/OFFSET must be an integer literal")
        return int(e.value)

    def _bind_setop(self, node, outer, ctes) -> BoundQuery:
        k = node["k"]
        if k == "select":
            return self._bind_select(node, outer, ctes, [])
        if k == "subquery_body":
            return self.bind_query(node["query"], outer, ctes)
        if k == "values":
            return self._bind_values(node, outer)
        if k != "setop":
            raise NotSupported(f"set operand {k}")
        op = node["s"]
        a = self._bind_setop(node["c"][0], outer, ctes)
        b = self._bind_setop(node["c"][1], outer, ctes)
        if len(a.names) != len(b.names):
            raise PlanError("UNION inputs have different numbers of columns")
        if op.startswith("union"):
            schema, kids = [], []
            cast_a, cast_b = [], []
            for ca, cb in zip(a.plan.schema, b.plan.schema):
                t = T.common_numeric(ca.dtype, cb.dtype) if ca.dtype != cb.dtype else ca.dtype
                schema.append(ColInfo(self.ids(), ca.name, t, ca.nullable or cb.nullable))
            pa_ = Project(a.plan, [(ColInfo(s.cid, s.name, s.dtype, s.nullable), self._coerce(c.ref(), s.dtype))
                                    for s, c in zip(schema, a.plan.schema)])
            schema_b = [ColInfo(self.ids(), s.name, s.dtype, s.nullable) for s in schema]
            pb_ = Project(b.plan, [(sb, self._coerce(c.ref(), sb.dtype)) for sb, c in zip(schema_b, b.plan.schema)])
            # union output reuses the first input's cids
            plan: Plan = Union([pa_, _rename(pb_, schema)], schema)
            if op == "union":
                plan = self._distinct(plan)
            return BoundQuery(plan, a.names)
        if op.startswith("intersect") or op.startswith("except"):
            kind = "semi" if op.startswith("intersect") else "anti"
            if op.endswith("_all"):
                # bag semantics: the k-th copy of a row matches the k-th copy
                # on the other side (row_number over all columns)
                la, lrn = self._numbered(a.plan)
                rb, rrn = self._numbered(b.plan)
                on = self._null_safe_keys(la.schema[:-1], rb.schema[:-1]) + [(lrn.ref(), rrn.ref())]
                j = Join(la, rb, kind, on)
                keep = [(ColInfo(self.ids(), c.name, c.dtype, c.nullable), c.ref()) for c in la.schema[:-1]]
                return BoundQuery(Project(j, keep), a.names)
            left = self._distinct(a.plan)
            on = self._null_safe_keys(left.schema, b.plan.schema)
            return BoundQuery(Join(left, b.plan, kind, on), a.names)
        raise NotSupported(op)

    def _numbered(self, plan: Plan) -> Tuple[Plan, ColInfo]:
        """``plan`` plus row_number() over (partition by every column)."""
        part = [c.ref() for c in plan.schema]
        w = WindowCall("row_number", [], part, [], WindowFrame("rows", "unbounded_preceding", "unbounded_following"),
                       INT64)
        ci = ColInfo(self.ids(), "__rn", INT64, False)
        return Window(plan, [(ci, w)]), ci

    def _null_safe_keys(self, ls: List[ColInfo], rs: List[ColInfo]) -> List[Tuple[Expr, Expr]]:
        """Equi-join keys under which NULL equals NULL (set operations): a
        nullable column contributes (is-null flag, value-or-default)."""
        on = []
        for ca, cb in zip(ls, rs):
            a, b = ca.ref(), cb.ref()
            if a.dtype != b.dtype:
                t = T.common_numeric(a.dtype, b.dtype) if (a.dtype.is_numeric and b.dtype.is_numeric) else a.dtype
                a, b = self._coerce(a, t), self._coerce(b, t)
            if not (ca.nullable or cb.nullable):
                on.append((a, b))
                continue
            d = _default_lit(a.dtype)
            on.append((Cast(IsNull(a), INT32), Cast(IsNull(b), INT32)))
            on.append((Func("coalesce", [a, d], a.dtype), Func("coalesce", [b, d], b.dtype)))
        return on

    def _distinct(self, plan: Plan) -> Plan:
        groups = [(ColInfo(self.ids(), c.name, c.dtype, c.nullable), c.ref()) for c in plan.schema]
        return Aggregate(plan, groups, [])

    def _bind_values(self, node, outer) -> BoundQuery:
        rows = [[self.bind_expr(e, Scope([], outer)) for e in r["c"]] for r in node["c"]]
        width = len(rows[0])
        schema = []
        for j in range(width):
            t = rows[0][j].dtype
            for r in rows[1:]:
                t = T.common_numeric(t, r[j].dtype) if t != r[j].dtype else t
            schema.append(ColInfo(self.ids(), f"column{j + 1}", t, any(r[j].nullable for r in rows)))
        rows = [[self._coerce(e, s.dtype) for e, s in zip(r, schema)] for r in rows]
        return BoundQuery(Values(rows, schema), [s.name for s in schema])

    def _order_over_output(self, bq: BoundQuery, order) -> BoundQuery:
        scope = Scope([Relation(None, [ColInfo(c.cid, n, c.dtype, c.nullable) for c, n in zip(bq.plan.schema, bq.names)])])
        keys = []
        for o in order:
            e = o["c"][0]
            if e["k"] == "lit" and e.get("type") == "int":
                idx = int(e["s"]) - 1
                c = bq.plan.schema[idx]
                bound: Expr = c.ref()
            else:
                bound = self.bind_expr(e, scope)
            asc = not o.get("desc")
            nf = o.get("nulls", "last" if asc else "first") == "first"
            keys.append((bound, asc, nf))
        return BoundQuery(Sort(bq.plan, keys), bq.names)

    # ================================================================== select
    def _bind_select(self, s: dict, outer: Optional[Scope], ctes: dict, order: list) -> BoundQuery:
        prev_w = getattr(self, "_win_defs", None)
        self._win_defs = {d["s"]: d["spec"] for d in _lst(s.get("windows"))}
        try:
            return self._bind_select_inner(s, outer, ctes, order)
        finally:
            self._win_defs = prev_w

    def _bind_select_inner(self, s: dict, outer: Optional[Scope], ctes: dict, order: list) -> BoundQuery:
        # ---- FROM
        if s.get("from"):
            plan, rels = None, []
            for item in _lst(s["from"]):
                p, r = self._bind_from(item, outer, ctes)
                plan = p if plan is None else Join(plan, p, "cross")
                rels += r
        else:
            plan, rels = Values([[]], []), []
        scope = Scope(rels, outer)
        # ---- WHERE
        if s.get("where"):
            pred = self.bind_expr(s["where"], scope)
            self._require_bool(pred, "WHERE")
            plan = Filter(plan, pred)
        # ---- SELECT list (stars expanded)
        items: List[Tuple[Expr, str]] = []
        for it in _lst(s["items"]):
            if it["k"] == "star":
                qual = it["s"] or None
                for r in rels:
                    if qual is None or r.qualifier == qual or (r.qualifier or "").split(".")[-1] == qual:
                        for c in r.cols:
                            items.append((c.ref(), c.name))
                if qual and not any(r.qualifier == qual or (r.qualifier or "").split(".")[-1] == qual for r in rels):
                    raise PlanError(f"unknown table '{qual}' in {qual}.*")
                continue
            e = self.bind_expr(it["c"][0], scope, allow_agg=True)
            items.append((e, it.get("alias") or self._display_name(it["c"][0], e)))
        # ---- GROUP BY (plain keys, or ROLLUP / CUBE / GROUPING SETS)
        group_nodes, set_nodes = _expand_group_by(_lst(s.get("group")))
        group_exprs: List[Expr] = []
        for g in group_nodes:
            group_exprs.append(self._bind_group_key(g, scope, items))
        sets = None
        if set_nodes is not None:
            keyidx: Dict[str, int] = {}
            uniq: List[Expr] = []
            for g in group_exprs:
                if g.sql() not in keyidx:
                    keyidx[g.sql()] = len(uniq)
                    uniq.append(g)
            sets = []
            for gs in set_nodes:
                ids = sorted({keyidx[group_exprs[k].sql()] for k in gs})
                sets.append(ids)
            group_exprs = uniq
        having = self.bind_expr(s["having"], scope, allow_agg=True) if s.get("having") else None
        qualify = self.bind_expr(s["qualify"], scope, allow_agg=True) if s.get("qualify") else None
        # DISTINCT ON (exprs): the first row of each key group in ORDER BY order
        distinct_on = [self._bind_group_key(g, scope, items) for g in _lst(s.get("distinct_on"))]
        # ORDER BY expressions bound against input scope + aliases (resolved later)
        aliases = {a: e for e, a in items}
        order_bound = []
        for o in order:
            e = o["c"][0]
            asc = not o.get("desc")
            nf = o.get("nulls", "last" if asc else "first") == "first"
            if e["k"] == "lit" and e.get("type") == "int":
                idx = int(e["s"]) - 1
                if not 0 <= idx < len(items):
                    raise PlanError(f"ORDER BY position {idx + 1} out of range")
                order_bound.append(("item", idx, asc, nf))
                continue
            if e["k"] == "col" and len(e["c"]) == 1 and e["s"] in aliases:
                idx = [a for _, a in items].index(e["s"])
                order_bound.append(("item", idx, asc, nf))
                continue
            bound = self.bind_expr(e, scope, allow_agg=True)
            # an ORDER BY expression identical to a select item uses that item
            hit = [i for i, (ie, _) in enumerate(items) if ie.sql() == bound.sql()]
            if hit:
                order_bound.append(("item", hit[0], asc, nf))
            else:
                order_bound.append(("expr", bound, asc, nf))
        # ---- aggregation
        extra = ([having] if having is not None else []) + ([qualify] if qualify is not None else []) + distinct_on
        has_aggs = any(_contains_agg(e) for e, _ in items) or any(_contains_agg(x) for x in extra) or \
            any(k == "expr" and _contains_agg(x) for k, x, _, _ in order_bound) or \
            any(_contains_grouping(e) for e, _ in items)
        if group_exprs or has_aggs or sets is not None:
            plan, rewrite = self._aggregate(plan, group_exprs, [e for e, _ in items] + extra
                                            + [x for k, x, _, _ in order_bound if k == "expr"], sets)
            items = [(rewrite(e), a) for e, a in items]
            if having is not None:
                having = rewrite(having)
            if qualify is not None:
                qualify = rewrite(qualify)
            distinct_on = [rewrite(x) for x in distinct_on]
            order_bound = [(k, rewrite(x) if k == "expr" else x, a, nf) for k, x, a, nf in order_bound]
        if having is not None:
            self._require_bool(having, "HAVING")
            plan = Filter(plan, having)
        # ---- window functions (after GROUP BY / HAVING, before DISTINCT / ORDER BY)
        wsrc = [e for e, _ in items] + ([qualify] if qualify is not None else []) + \
            [x for k, x, _, _ in order_bound if k == "expr"]
        wmap: Dict[str, ColRef] = {}
        wexprs: List[Tuple[ColInfo, WindowCall]] = []
        for e in wsrc:
            for x in walk(e):
                if isinstance(x, WindowCall) and x.sql() not in wmap:
                    if any(isinstance(y, WindowCall) for k in x.children() for y in walk(k)):
                        raise PlanError("window function calls cannot be nested")
                    ci = ColInfo(self.ids(), x.func, x.dtype, x.nullable)
                    wexprs.append((ci, x))
                    wmap[x.sql()] = ci.ref()
        if wexprs:
            plan = Window(plan, wexprs)

            def wrw(e: Expr) -> Expr:
                return _transform_top_down(e, lambda x: wmap.get(x.sql()) if isinstance(x, WindowCall) else None)
            items = [(wrw(e), a) for e, a in items]
            if qualify is not None:
                qualify = wrw(qualify)
            distinct_on = [wrw(x) for x in distinct_on]
            order_bound = [(k, wrw(x) if k == "expr" else x, a, nf) for k, x, a, nf in order_bound]
        if qualify is not None:
            self._require_bool(qualify, "QUALIFY")
            plan = Filter(plan, qualify)
        if distinct_on:
            okeys = [(items[x][0] if k == "item" else x, a, nf) for k, x, a, nf in order_bound]
            rn = WindowCall("row_number", [], list(distinct_on), okeys, self._frame(None, okeys), INT64)
            rci = ColInfo(self.ids(), "__distinct_on", INT64, False)
            plan = Filter(Window(plan, [(rci, rn)]), BinOp("=", rci.ref(), Lit(1, INT64), BOOL))
        # ---- SELECT unnest(list): one row per element, the other items repeated
        unn = {}
        for e, _ in items:
            for x in walk(e):
                if isinstance(x, Func) and x.name == "unnest":
                    unn.setdefault(x.args[0].sql(), x)
        if len(unn) > 1:
            raise NotSupported("more than one distinct unnest() in a SELECT list")
        if unn:
            u = next(iter(unn.values()))
            lci = ColInfo(self.ids(), "__unnest_list", u.args[0].dtype, True)
            plan = Project(plan, [(c, c.ref()) for c in plan.schema] + [(lci, u.args[0])])
            oci = ColInfo(self.ids(), "__unnest", u.dtype, True)
            plan = Unnest(plan, lci, oci)
            key = u.sql()

            def urw(e: Expr) -> Expr:
                return _transform_top_down(e, lambda x: oci.ref() if x.sql() == key else None)
            items = [(urw(e), a) for e, a in items]
            order_bound = [(k, urw(x) if k == "expr" else x, a, nf) for k, x, a, nf in order_bound]
        # ---- projection (+ hidden ORDER BY columns)
        proj = [(ColInfo(self.ids(), a, e.dtype, e.nullable), e) for e, a in items]
        hidden = []
        sort_keys = []
        for k, x, asc, nf in order_bound:
            if k == "item":
                sort_keys.append((proj[x][0].ref(), asc, nf))
            else:
                ci = ColInfo(self.ids(), f"__order{len(hidden)}", x.dtype, x.nullable)
                hidden.append((ci, x))
                sort_keys.append((ci.ref(), asc, nf))
        distinct = bool(s.get("distinct"))
        if distinct and hidden:
            raise PlanError("for SELECT DISTINCT, ORDER BY expressions must appear in select list")
        plan = Project(plan, proj + hidden)
        if distinct:
            plan = self._distinct_keep(plan)
        if sort_keys:
            plan = Sort(plan, sort_keys)
            if hidden:
                plan = Project(plan, [(c, c.ref()) for c, _ in proj])
        names = [c.name for c, _ in proj]
        return BoundQuery(plan, names)

    def _bind_group_key(self, g: dict, scope: Scope, items) -> Expr:
        if g["k"] == "lit" and g.get("type") == "int":
            idx = int(g["s"]) - 1
            if not 0 <= idx < len(items):
                raise PlanError(f"GROUP BY position {idx + 1} out of range")
            return items[idx][0]
        if g["k"] == "col" and len(g["c"]) == 1:
            # a select alias may be used in GROUP BY (when it is not also an input column)
            nm = g["s"]
            try:
                scope.resolve([nm])
            except PlanError:
                hit = [e for e, a in items if a == nm]
                if hit:
                    return hit[0]
        return self.bind_expr(g, scope)

    def _distinct_keep(self, plan: Project) -> Plan:
        # DISTINCT keeps the projected cids so ORDER BY references stay valid
        groups = [(c, c.ref()) for c in plan.schema]
        return Aggregate(plan, [(ColInfo(c.cid, c.name, c.dtype, c.nullable), _Passthrough(c)) for c, _ in groups], [])

    def _aggregate(self, plan: Plan, group_exprs: List[Expr], exprs: List[Expr], sets=None):
        """One Aggregate over ``plan`` (``sets`` None), or for GROUPING SETS /
        ROLLUP / CUBE a UNION ALL of one Aggregate per grouping set, each
        padded with NULL for the keys it does not group by and tagged with a
        grouping-id column (bit k-1-i set when key i is aggregated away) that
        ``grouping(...)`` reads."""
        groups: List[Tuple[ColInfo, Expr]] = []
        gmap: Dict[str, ColRef] = {}
        for g in group_exprs:
            key = TPL.eq_sql(g)
            if key in gmap:
                continue
            name = g.name if isinstance(g, ColRef) else key
            ci = ColInfo(self.ids(), name, g.dtype, g.nullable or sets is not None)
            groups.append((ci, g))
            gmap[key] = ci.ref()
        aggs: List[Tuple[ColInfo, AggCall]] = []
        amap: Dict[str, ColRef] = {}
        for e in exprs:
            for x in walk(e):
                if isinstance(x, AggCall):
                    key = TPL.eq_sql(x) + (f" FILTER {TPL.eq_sql(x.filter)}" if x.filter is not None else "")
                    if key not in amap:
                        if x.arg is not None and _contains_agg(x.arg):
                            raise PlanError("aggregate function calls cannot be nested")
                        ci = ColInfo(self.ids(), TPL.eq_sql(x), x.dtype, x.func not in ("count", "approx_distinct"))
                        aggs.append((ci, x))
                        amap[key] = ci.ref()
        gid_ref: Optional[ColRef] = None
        if sets is None:
            agg: Plan = Aggregate(plan, groups, aggs)
        else:
            k = len(groups)
            gid_ci = ColInfo(self.ids(), "__grouping_id", INT64, False)
            gid_ref = gid_ci.ref()
            schema = [c for c, _ in groups] + [gid_ci] + [c for c, _ in aggs]
            branches = []
            for st in sets:
                gi = [(ColInfo(self.ids(), groups[i][0].name, groups[i][1].dtype, groups[i][1].nullable), groups[i][1])
                      for i in st]
                ai = [(ColInfo(self.ids(), c.name, c.dtype, c.nullable), a) for c, a in aggs]
                a_plan = Aggregate(plan, gi, ai)
                pos = {i: gi[n][0] for n, i in enumerate(st)}
                bits = sum(1 << (k - 1 - i) for i in range(k) if i not in pos)
                pe: List[Tuple[ColInfo, Expr]] = []
                for i, (c, _) in enumerate(groups):
                    e = pos[i].ref() if i in pos else Lit(None, c.dtype)
                    pe.append((ColInfo(self.ids(), c.name, c.dtype, True), e))
                pe.append((ColInfo(self.ids(), "__grouping_id", INT64, False), Lit(bits, INT64)))
                for (c, _), (cc, _) in zip(aggs, ai):
                    pe.append((ColInfo(self.ids(), c.name, c.dtype, c.nullable), cc.ref()))
                branches.append(Project(a_plan, pe))
            agg = Union(branches, schema)
        group_cids = {ci.cid for ci, _ in groups}
        ginfo = [g for _, g in groups]

        def grouping_expr(f: Func) -> Expr:
            out: Expr = Lit(0, INT64)
            m = len(f.args)
            for j, a in enumerate(f.args):
                idx = next((i for i, g in enumerate(ginfo) if g.sql() == a.sql()), None)
                if idx is None:
                    raise PlanError(f"grouping() argument {a.sql()} is not a GROUP BY expression")
                if gid_ref is None:
                    continue
                bit = BinOp("%", BinOp("/", gid_ref, Lit(1 << (len(ginfo) - 1 - idx), INT64), INT64),
                            Lit(2, INT64), INT64)
                term = BinOp("*", bit, Lit(1 << (m - 1 - j), INT64), INT64)
                out = term if isinstance(out, Lit) and out.value == 0 else BinOp("+", out, term, INT64)
            return Cast(out, INT32) if not isinstance(out, Lit) else Lit(0, INT32)

        def rewrite(e: Expr) -> Expr:
            def fn(x):
                k_ = TPL.eq_sql(x)
                if isinstance(x, AggCall):
                    return amap[k_ + (f" FILTER {TPL.eq_sql(x.filter)}" if x.filter is not None else "")]
                if isinstance(x, Func) and x.name == "grouping":
                    return grouping_expr(x)
                if k_ in gmap:
                    return gmap[k_]
                return None
            out = _transform_top_down(e, fn)
            for x in walk(out):
                if isinstance(x, ColRef) and x.cid not in group_cids and x.cid not in {c.cid for c, _ in aggs} \
                        and (gid_ref is None or x.cid != gid_ref.cid):
                    if isinstance(x, ColRef) and not getattr(x, "_outer", False):
                        raise PlanError(f"column '{x.name}' must appear in the GROUP BY clause or be used in an aggregate function")
            return out
        return agg, rewrite

    # =================================================================== FROM
    def _bind_from(self, item: dict, outer, ctes) -> Tuple[Plan, List[Relation]]:
        k = item["k"]
        if k == "table":
            name = item["s"]
            alias = item.get("alias")
            if name in ctes:
                ent = ctes[name]
                if ent[0] == "__work":
                    # the recursive term's reference to its own CTE: last iteration's rows
                    _, tid, wschema = ent
                    sch = [ColInfo(self.ids(), c.name, c.dtype, c.nullable, alias or name) for c in wschema]
                    return WorkTableScan(tid, sch), [Relation(alias or name, sch)]
                cnode, cenv = ent[0], ent[1]
                if len(ent) > 2 and ent[2]:
                    bq = self._bind_recursive_cte(cnode, outer, cenv)
                else:
                    bq = self.bind_query(cnode["query"], outer, cenv)
                cols = [c["s"] for c in _lst(cnode.get("columns"))] or bq.names
                return self._derived(bq, alias or name, cols, item)
            view = self.catalog.get_view(name) if hasattr(self.catalog, "get_view") else None
            if view is not None:
                from ..sql import parse
                q = view if isinstance(view, dict) else parse(view)[0]
                bq = self.bind_query(q, outer, {})
                return self._derived(bq, alias or name, q.get("__columns") or bq.names, item)
            src = self.catalog.get_table(name)
            if src is None:
                raise TableNotFound(f"table '{name}' not found")
            schema = [ColInfo(self.ids(), f.name, f.dtype, f.nullable, alias or name) for f in src.schema()]
            qual = alias or name
            rel = Relation(qual, schema)
            if item.get("columns"):
                new = [c["s"] for c in _lst(item["columns"])]
                rel = Relation(qual, [ColInfo(c.cid, n, c.dtype, c.nullable, qual) for c, n in zip(schema, new)] + schema[len(new):])
            return Scan(name, src, schema), [rel]
        if k == "subquery":
            bq = self.bind_query(item["query"], outer, ctes)
            cols = [c["s"] for c in _lst(item.get("columns"))] or bq.names
            return self._derived(bq, item.get("alias"), cols, item)
        if k == "table_func":
            return self._table_func(item, outer)
        if k == "join":
            lp, lr = self._bind_from(item["c"][0], outer, ctes)
            rp, rr = self._bind_from(item["c"][1], outer, ctes)
            kind = item["s"]
            kind = {"left_semi": "semi", "left_anti": "anti"}.get(kind, kind)
            if kind in ("right_semi", "right_anti"):
                lp, rp, lr, rr = rp, lp, rr, lr
                kind = kind.split("_")[1]
            scope = Scope(lr + rr, outer)
            residual = None
            if item.get("on"):
                residual = self.bind_expr(item["on"], scope)
            names = None
            if item.get("using"):
                names = [c["s"] for c in _lst(item["using"])]
            elif item.get("natural"):
                ln = {c.name for r in lr for c in r.cols}
                names = [c.name for r in rr for c in r.cols if c.name in ln]
            if names:
                conds = []
                for n in names:
                    a = Scope(lr).resolve([n])[0]
                    b = Scope(rr).resolve([n])[0]
                    conds.append(self._cmp("=", a.ref(), b.ref()))
                residual = and_all(conds + ([residual] if residual is not None else []))
                # the USING column is visible once (from the left input)
                rr = [Relation(r.qualifier, [c for c in r.cols if c.name not in names]) for r in rr]
            if kind == "cross":
                return Join(lp, rp, "cross"), lr + rr
            return Join(lp, rp, kind, [], residual), (lr + rr if kind not in ("semi", "anti") else lr)
        raise NotSupported(f"FROM item {k}")

    def _table_func(self, item: dict, outer) -> Tuple[Plan, List[Relation]]:
        """generate_series / range / unnest in FROM (constant arguments)."""
        name = item["s"].lower()
        alias = item.get("alias") or name
        names = [c["s"] for c in _lst(item.get("columns"))]
        args = [self.bind_expr(a, Scope([], outer)) for a in item["c"]]
        if name in ("generate_series", "range"):
            if not 1 <= len(args) <= 3:
                raise PlanError(f"{name}() takes 1 to 3 arguments")
            vals = []
            for a in args:
                a = _fold(a)
                if not isinstance(a, Lit) or a.value is None or not a.dtype.is_integer:
                    raise NotSupported(f"{name}(): arguments must be integer constants")
                vals.append(int(a.value))
            if len(vals) == 1:
                vals = [0, vals[0]]
            if len(vals) == 2:
                vals.append(1)
            ci = ColInfo(self.ids(), names[0] if names else "value", INT64, False, alias)
            return TableFunction(name, vals, [ci]), [Relation(alias, [ci])]
        if name == "unnest":
            _nargs(name, args, 1)
            lt = args[0].dtype
            if lt.kind != "list":
                raise PlanError(f"unnest() needs a list argument, got {lt}")
            if col_refs(args[0]):
                raise NotSupported("unnest() in FROM of a column: use SELECT unnest(col) FROM t")
            cname = names[0] if names else f"UNNEST({args[0].sql()})"
            ci = ColInfo(self.ids(), cname, lt.child, True, alias)
            return TableFunction("unnest", [args[0]], [ci]), [Relation(alias, [ci])]
        raise NotSupported(f"table function {name}()")

    def _bind_recursive_cte(self, cnode: dict, outer, cenv: dict) -> BoundQuery:
        """WITH RECURSIVE name AS (anchor UNION [ALL] recursive-term)."""
        q = cnode["query"]
        body = q["body"]
        if body["k"] != "setop" or not body["s"].startswith("union"):
            raise PlanError(f"recursive CTE '{cnode['s']}' must be <anchor> UNION [ALL] <recursive term>")
        if q.get("order") or q.get("limit"):
            raise NotSupported("ORDER BY / LIMIT on a recursive CTE body")
        env = dict(cenv)
        env.update(getattr(self, "_ctes", None) or {})
        env.pop(cnode["s"], None)
        anchor = self._bind_setop(body["c"][0], outer, env)
        names = [c["s"] for c in _lst(cnode.get("columns"))] or anchor.names
        if len(names) != len(anchor.plan.schema):
            raise PlanError(f"recursive CTE '{cnode['s']}' has {len(names)} column names for "
                            f"{len(anchor.plan.schema)} columns")
        tid = self.ids()
        wschema = [ColInfo(self.ids(), n, c.dtype, True) for n, c in zip(names, anchor.plan.schema)]
        env[cnode["s"]] = ("__work", tid, wschema)
        rec = self._bind_setop(body["c"][1], outer, env)
        if len(rec.plan.schema) != len(wschema):
            raise PlanError("recursive term returns a different number of columns than the anchor")
        out = [ColInfo(self.ids(), w.name, w.dtype, True) for w in wschema]
        ap = Project(anchor.plan, [(ColInfo(self.ids(), o.name, o.dtype, True), self._coerce(c.ref(), o.dtype))
                                   for o, c in zip(out, anchor.plan.schema)])
        rp = Project(rec.plan, [(ColInfo(self.ids(), o.name, o.dtype, True), self._coerce(c.ref(), o.dtype))
                                for o, c in zip(out, rec.plan.schema)])
        limit = int(self.session.get("max_recursion", 1000) or 1000)
        return BoundQuery(RecursiveCTE(ap, rp, tid, out, body["s"] == "union", limit), names)

    def _derived(self, bq: BoundQuery, alias, names, item) -> Tuple[Plan, List[Relation]]:
        cols = [ColInfo(c.cid, n, c.dtype, c.nullable, alias) for c, n in zip(bq.plan.schema, names)]
        return bq.plan, [Relation(alias, cols)]

    # ============================================================ expressions
    def bind_expr(self, node: dict, scope: Scope, allow_agg: bool = False) -> Expr:
        k = node["k"]
        if k == "paren":
            return self.bind_expr(node["c"][0], scope, allow_agg)
        if k == "col":
            parts = [p["s"] for p in node["c"]]
            if len(parts) == 1 and parts[0] in scope.aliases:
                return scope.aliases[parts[0]]
            try:
                ci, depth = scope.resolve(parts)
            except PlanError:
                if len(parts) == 1 and parts[0] in ("current_date", "current_timestamp", "localtimestamp"):
                    return self._func_library(parts[0].replace("localtimestamp", "current_timestamp"), [])
                raise
            r = ci.ref()
            if depth > 0:
                r._outer = True  # type: ignore[attr-defined]
                s = scope
                for _ in range(depth):
                    s.outer_refs.add(ci.cid)
                    s = s.parent
            return r
        if k == "lit":
            return self._literal(node)
        if k == "bin":
            op = node["s"]
            l = self.bind_expr(node["c"][0], scope, allow_agg)
            r = self.bind_expr(node["c"][1], scope, allow_agg)
            if op in ("and", "or"):
                self._require_bool(l, op.upper())
                self._require_bool(r, op.upper())
                return _fold(BinOp(op, l, r, BOOL))
            if op in ("=", "<>", "<", "<=", ">", ">=", "is_distinct_from", "is_not_distinct_from"):
                return self._cmp(op, l, r)
            if op == "||":
                return Func("concat", [self._coerce(l, UTF8), self._coerce(r, UTF8)], UTF8)
            if op in ("~", "~*", "!~", "!~*"):
                # POSIX regex match operators: regexp_like, '*' = case-insensitive
                if not isinstance(r, Lit) or not isinstance(TPL.peek(r), str):
                    raise NotSupported(f"{op}: the pattern must be a string literal")
                e = self._func_library("regexp_like", [l, r, Lit("i" if op.endswith("*") else "", UTF8)])
                return Not(e) if op.startswith("!") else e
            return self._arith(op, l, r)
        if k == "un":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            if node["s"] == "not":
                self._require_bool(x, "NOT")
                if isinstance(x, Lit):
                    return TPL.derive(lambda a: Lit(None if a.value is None else (not a.value), BOOL), x)
                return Not(x)
            if isinstance(x, Lit) and TPL.peek(x) is not None:
                return TPL.derive(lambda a: Lit(-a.value, a.dtype), x)
            return Neg(x, x.dtype)
        if k == "between":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            lo = self.bind_expr(node["c"][1], scope, allow_agg)
            hi = self.bind_expr(node["c"][2], scope, allow_agg)
            e = BinOp("and", self._cmp(">=", x, lo), self._cmp("<=", x, hi), BOOL)
            return Not(e) if node.get("neg") else e
        if k == "inlist":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            vals = [self.bind_expr(v, scope, allow_agg) for v in node["c"][1:]]
            if not all(isinstance(v, Lit) for v in vals):
                ors = [self._cmp("=", x, v) for v in vals]
                e = ors[0]
                for o in ors[1:]:
                    e = BinOp("or", e, o, BOOL)
                return Not(e) if node.get("neg") else e
            t = x.dtype
            vals = [self._coerce_lit(v, t) for v in vals]
            return InList(x, vals, bool(node.get("neg")))
        if k == "like":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            p = self.bind_expr(node["c"][1], scope, allow_agg)
            if not isinstance(p, Lit) or not isinstance(TPL.peek(p), str):
                raise NotSupported("LIKE pattern must be a string literal")
            esc = "\\"
            if node.get("escape"):
                esc = self.bind_expr(node["escape"], scope).value
            e = Like(self._coerce(x, UTF8), TPL.peek(p), bool(node.get("neg")), bool(node.get("ilike")), esc)
            TPL.raw(e, "pattern", lambda a: a.value, p)      # (a template re-reads the pattern)
            return e
        if k == "similar":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            p = self.bind_expr(node["c"][1], scope, allow_agg)
            if not isinstance(p, Lit) or not isinstance(p.value, str):
                raise NotSupported("SIMILAR TO pattern must be a string literal")
            esc = self.bind_expr(node["escape"], scope).value if node.get("escape") else "\\"
            e = self._func_library("regexp_like", [x, Lit(similar_to_regex(p.value, esc), UTF8), Lit("", UTF8)])
            return Not(e) if node.get("neg") else e
        if k == "param":
            params = PARAMS.get() or []
            i = int(node["s"]) - 1
            if not 0 <= i < len(params):
                raise PlanError(f"no value for parameter ${i + 1} ({len(params)} given)")
            return params[i]
        if k == "isnull":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            return IsNull(x, bool(node.get("neg")))
        if k == "istruth":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            want = node["s"] == "true"
            e = BinOp("and", IsNull(x, True), x if want else Not(x), BOOL)
            return Not(e) if node.get("neg") else e
        if k == "cast":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            t = T.parse_type_name(node["type"])
            return self._cast(x, t)
        if k == "case":
            return self._case(node, scope, allow_agg)
        if k == "extract":
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            return self._date_part(node["s"].lower(), x)
        if k == "func":
            return self._func(node, scope, allow_agg)
        if k in ("subq", "exists", "insub"):
            sub_scope = Scope([], scope)
            bq = self.bind_query(node["query"], sub_scope, getattr(self, "_ctes", None))
            outer = set(sub_scope.outer_refs)
            if k == "exists":
                return SubqueryExpr("exists", bq.plan, None, bool(node.get("neg")), BOOL, outer)
            if k == "subq":
                if len(bq.plan.schema) != 1:
                    raise PlanError("scalar subquery must return exactly one column")
                c = bq.plan.schema[0]
                return SubqueryExpr("scalar", bq.plan, None, False, c.dtype, outer)
            x = self.bind_expr(node["c"][0], scope, allow_agg)
            if len(bq.plan.schema) != 1:
                raise PlanError("IN subquery must return exactly one column")
            return SubqueryExpr("in", bq.plan, x, bool(node.get("neg")), BOOL, outer)
        if k == "row":
            raise NotSupported("row constructors")
        raise NotSupported(f"expression kind {k}")

    # ------------------------------------------------------------ literals
    def _literal(self, node) -> Lit:
        x = self.literal_of(node)
        slot = node.get("__slot")
        if slot is not None and TPL.active():
            # a literal token of a statement being recorded as a template (sql/template.py)
            return TPL.SlotLit(x.value, x.dtype, slot)
        return x

    @staticmethod
    def literal_of(node) -> Lit:
        """The literal an AST literal node denotes."""
        t = node["type"]
        s = node["s"]
        if t == "int":
            v = int(s)
            return Lit(v, INT64)
        if t == "dec":
            d = Decimal(s)
            sign, digits, exp = d.as_tuple()
            scale = max(-exp, 0)
            unscaled = int(d.scaleb(scale))
            prec = max(len(str(abs(unscaled))), scale + 1)
            return Lit(unscaled, T.DECIMAL(prec, scale))
        if t == "float":
            return Lit(float(s), FLOAT64)
        if t == "str":
            return Lit(s, UTF8)
        if t == "bool":
            return Lit(s == "true", BOOL)
        if t == "null":
            return Lit(None, T.NULL)
        if t == "date":
            return Lit(date_to_days(s), DATE32)
        if t == "timestamp":
            dt = datetime.datetime.fromisoformat(s)
            return Lit(int((dt - datetime.datetime(1970, 1, 1)).total_seconds() * 1_000_000), T.TIMESTAMP)
        if t == "interval":
            return Lit(_parse_interval(s, node.get("unit")), INTERVAL)
        raise NotSupported(f"literal type {t}")

    # ------------------------------------------------------------ typing
    @staticmethod
    def _require_bool(e: Expr, where: str):
        if e.dtype not in (BOOL, T.NULL):
            raise PlanError(f"{where} requires a boolean expression, got {e.dtype}")

    def _cast(self, x: Expr, t: DataType) -> Expr:
        if x.dtype == t:
            return x
        if isinstance(x, Lit):
            return _fold_cast(x, t)
        return Cast(x, t)

    def _coerce_lit(self, v: Lit, t: DataType) -> Lit:
        if TPL.tracking(v):
            return TPL.derive(lambda a, t=t: self._coerce_lit(a, t), v)
        if v.dtype == t or v.value is None:
            return Lit(v.value, t) if v.value is None else v
        if t.is_string:
            return v if v.dtype.is_string else _fold_cast(v, UTF8)
        if t.kind == "date32" and v.dtype.is_string:
            return Lit(date_to_days(v.value), DATE32)
        if t.is_numeric and v.dtype.is_numeric:
            ct = T.common_numeric(t, v.dtype)
            return _fold_cast(v, ct)
        return _fold_cast(v, t)

    def _coerce(self, e: Expr, t: DataType) -> Expr:
        if e.dtype == t:
            return e
        if isinstance(e, Lit):
            return self._coerce_lit(e, t) if TPL.peek(e) is not None else Lit(None, t)
        return Cast(e, t)

    def _cmp(self, op: str, l: Expr, r: Expr) -> Expr:
        lt, rt = l.dtype, r.dtype
        # literal coercion towards the column type
        if lt != rt:
            if isinstance(r, Lit) and not isinstance(l, Lit):
                if lt.kind == "timestamp" and (rt.is_string or rt.kind == "date32"):
                    r = _fold_cast(r, T.TIMESTAMP)
                elif rt.kind == "timestamp" and lt.kind == "date32":
                    l = self._to_ts(l)
                elif lt.kind == "date32" and rt.is_string:
                    r = TPL.derive(lambda a: Lit(date_to_days(a.value), DATE32), r)
                elif lt.is_string and not rt.is_string and TPL.peek(r) is not None:
                    r = _fold_cast(r, UTF8)
            elif isinstance(l, Lit) and not isinstance(r, Lit):
                if rt.kind == "timestamp" and (lt.is_string or lt.kind == "date32"):
                    l = _fold_cast(l, T.TIMESTAMP)
                elif rt.kind == "date32" and lt.is_string:
                    l = TPL.derive(lambda a: Lit(date_to_days(a.value), DATE32), l)
                elif rt.is_string and not lt.is_string and TPL.peek(l) is not None:
                    l = _fold_cast(l, UTF8)
            lt, rt = l.dtype, r.dtype
        if lt != rt:
            ct = T.common_numeric(lt, rt)
            l, r = self._coerce(l, ct), self._coerce(r, ct)
        if op in ("is_distinct_from", "is_not_distinct_from"):
            return _distinct_from(op == "is_distinct_from", l, r)
        return _fold(BinOp(op, l, r, BOOL))

    def _arith(self, op: str, l: Expr, r: Expr) -> Expr:
        if isinstance(l, Lit) and isinstance(r, Lit) and TPL.tracking(l, r):
            # literal arithmetic (date +/- interval, folded numbers): re-derived per template instance
            return TPL.derive(lambda a, b, op=op: self._arith(op, a, b), l, r)
        lt, rt = l.dtype, r.dtype
        # ---- DATE / INTERVAL arithmetic
        if lt == INTERVAL or rt == INTERVAL:
            if rt == INTERVAL and op in ("+", "-") and lt.kind in ("date32", "timestamp"):
                months, days, us = r.value
                if op == "-":
                    months, days, us = -months, -days, -us
                if lt.kind == "date32" and not us:
                    if isinstance(l, Lit):
                        return Lit(add_months(l.value, months) + days if l.value is not None else None, DATE32)
                    if months:
                        return Func("add_months", [l], DATE32, (months, days))
                    return BinOp("+", l, Lit(days, INT32), DATE32)
                x = self._to_ts(l)
                if isinstance(x, Lit):
                    if x.value is None:
                        return Lit(None, T.TIMESTAMP)
                    dd, rem = divmod(x.value, 86_400_000_000)
                    return Lit((add_months(dd, months) + days) * 86_400_000_000 + rem + us, T.TIMESTAMP)
                return Func("ts_add", [x], T.TIMESTAMP, (months, days, us))
            if lt == INTERVAL and op == "+" and rt.kind in ("date32", "timestamp"):
                return self._arith("+", r, l)
            if lt == INTERVAL and rt == INTERVAL and op in ("+", "-"):
                sg = 1 if op == "+" else -1
                return Lit(tuple(a + sg * b for a, b in zip(l.value, r.value)), INTERVAL)
            raise NotSupported(f"interval arithmetic {lt} {op} {rt}")
        if lt.kind == "timestamp" or rt.kind == "timestamp":
            if op == "-" and lt.kind == "timestamp" and rt.kind in ("timestamp", "date32"):
                return BinOp("-", l, self._to_ts(r), INT64)
            raise PlanError(f"cannot apply {op} to {lt} and {rt}")
        if lt.kind == "date32" or rt.kind == "date32":
            if op == "-" and lt.kind == "date32" and rt.kind == "date32":
                return _fold(BinOp("-", l, r, INT64))
            if op in ("+", "-") and lt.kind == "date32" and rt.is_integer:
                return _fold(BinOp(op, l, r, DATE32))
            if op == "+" and rt.kind == "date32" and lt.is_integer:
                return _fold(BinOp(op, r, l, DATE32))
            raise PlanError(f"cannot apply {op} to {lt} and {rt}")
        if lt.is_string or rt.is_string:
            raise PlanError(f"cannot apply {op} to {lt} and {rt}")
        if lt.kind == "null" or rt.kind == "null":
            t = rt if lt.kind == "null" else lt
            return Lit(None, t if t.kind != "null" else INT64)
        if lt.kind == "bool" or rt.kind == "bool":
            raise PlanError(f"cannot apply {op} to boolean")
        # ---- numeric
        if lt.is_float or rt.is_float:
            t = FLOAT64
            return _fold(BinOp(op, self._coerce(l, t), self._coerce(r, t), t))
        if lt.is_decimal or rt.is_decimal:
            dl = lt if lt.is_decimal else _int_as_decimal(l)
            dr = rt if rt.is_decimal else _int_as_decimal(r)
            if op in ("+", "-"):
                s = max(dl.scale, dr.scale)
                p = min(38, max(dl.precision - dl.scale, dr.precision - dr.scale) + s + 1)
                t = T.DECIMAL(p, s)
                return _fold(BinOp(op, self._coerce(l, T.DECIMAL(dl.precision + s - dl.scale, s)),
                                   self._coerce(r, T.DECIMAL(dr.precision + s - dr.scale, s)), t))
            if op == "*":
                t = T.DECIMAL(min(38, dl.precision + dr.precision + 1), dl.scale + dr.scale)
                return _fold(BinOp("*", self._coerce(l, dl), self._coerce(r, dr), t))
            if op == "/":
                return _fold(BinOp("/", self._coerce(l, FLOAT64), self._coerce(r, FLOAT64), FLOAT64))
            if op == "%":
                s = max(dl.scale, dr.scale)
                t = T.DECIMAL(max(dl.precision, dr.precision), s)
                return _fold(BinOp("%", self._coerce(l, T.DECIMAL(dl.precision, s)), self._coerce(r, T.DECIMAL(dr.precision, s)), t))
        if lt.is_integer and rt.is_integer:
            return _fold(BinOp(op, self._coerce(l, INT64), self._coerce(r, INT64), INT64))
        raise PlanError(f"cannot apply {op} to {lt} and {rt}")

    def _case(self, node, scope, allow_agg) -> Expr:
        operand = self.bind_expr(node["operand"], scope, allow_agg) if node.get("operand") else None
        kids = node["c"]
        whens = []
        for i in range(0, len(kids), 2):
            c = self.bind_expr(kids[i], scope, allow_agg)
            v = self.bind_expr(kids[i + 1], scope, allow_agg)
            if operand is not None:
                c = self._cmp("=", operand, c)
            whens.append((c, v))
        els = self.bind_expr(node["else"], scope, allow_agg) if node.get("else") else None
        t = None
        for _, v in whens + ([(None, els)] if els is not None else []):
            if v.dtype.kind == "null":
                continue
            t = v.dtype if t is None else (t if t == v.dtype else T.common_numeric(t, v.dtype))
        t = t or T.NULL
        whens = [(c, self._coerce(v, t)) for c, v in whens]
        els = self._coerce(els, t) if els is not None else None
        return Case(whens, els, t)

    def _func(self, node, scope, allow_agg) -> Expr:
        name = node["s"].lower()
        if node.get("over") is not None:
            return self._window_call(name, node, scope, allow_agg)
        if name == "grouping":
            if not allow_agg:
                raise PlanError("grouping() is only allowed with GROUP BY")
            return Func("grouping", [self.bind_expr(a, scope) for a in node["c"]], INT32)
        if name in AGG_FUNCS or name in _EXTRA_AGGS:
            if not allow_agg:
                raise PlanError(f"aggregate function {name} not allowed here")
            distinct = bool(node.get("distinct"))
            arg2, param = None, None
            order = tuple(self._agg_order(node.get("order"), scope))
            if node.get("within_group") is not None:
                # ordered-set aggregate: percentile_cont(q) WITHIN GROUP (ORDER BY x [DESC])
                if name not in ("percentile_cont", "percentile_disc", "approx_percentile_cont", "median"):
                    raise PlanError(f"WITHIN GROUP is not valid for {name}()")
                wg = self._agg_order(node["within_group"], scope)
                if len(wg) != 1:
                    raise PlanError(f"{name}() WITHIN GROUP takes exactly one ORDER BY expression")
                x, asc, _ = wg[0]
                qs = [self.bind_expr(a, scope) for a in node["c"]]
                if name == "median":
                    q = 0.5
                else:
                    if len(qs) != 1 or not isinstance(qs[0], Lit) or qs[0].value is None:
                        raise PlanError(f"{name}() takes a constant fraction")
                    q = float(qs[0].value) / (10 ** qs[0].dtype.scale if qs[0].dtype.is_decimal else 1)
                if not 0.0 <= q <= 1.0:
                    raise PlanError("percentile must be between 0 and 1")
                if not asc:
                    q = 1.0 - q
                flt = self.bind_expr(node["filter"], scope) if node.get("filter") else None
                return _make_agg("percentile_disc" if name == "percentile_disc" else "percentile_cont", x, False,
                                 flt, None, q)
            if node.get("star"):
                arg = None
            else:
                args = [self.bind_expr(a, scope) for a in node["c"]]
                if not args:
                    raise PlanError(f"{name}() needs an argument")
                arg = args[0]
                if name in ("covar", "covar_samp", "covar_pop", "corr"):
                    if len(args) != 2:
                        raise PlanError(f"{name}() takes two arguments")
                    arg2 = args[1]
                elif name in ("percentile_cont", "percentile_disc"):
                    # percentile_cont(x, q): the DataFusion function-call spelling
                    if len(args) != 2 or not isinstance(args[1], Lit) or args[1].value is None:
                        raise PlanError(f"{name}() takes a constant fraction")
                    param = float(args[1].value) / (10 ** args[1].dtype.scale if args[1].dtype.is_decimal else 1)
                    if not 0.0 <= param <= 1.0:
                        raise PlanError("percentile must be between 0 and 1")
                elif name in ("string_agg", "approx_percentile_cont"):
                    if len(args) != 2 or not isinstance(args[1], Lit) or args[1].value is None:
                        raise PlanError(f"{name}() takes a constant second argument")
                    param = args[1].value
                    if name == "approx_percentile_cont":
                        param = float(args[1].value) / (10 ** args[1].dtype.scale if args[1].dtype.is_decimal else 1)
                        if not 0.0 <= param <= 1.0:
                            raise PlanError("percentile must be between 0 and 1")
                    else:
                        param = str(param)
                elif len(args) != 1:
                    raise NotSupported(f"{name} with {len(args)} arguments")
            flt = self.bind_expr(node["filter"], scope) if node.get("filter") else None
            if order and name not in ("array_agg", "string_agg", "first_value", "last_value"):
                order = ()      # ORDER BY does not change an order-insensitive aggregate
            return _make_agg(name, arg, distinct, flt, arg2, param, order)
        args = [self.bind_expr(a, scope, allow_agg) for a in node["c"]]
        if name in ("upper", "lower", "capitalize"):
            _nargs(name, args, 1)
            a = self._coerce(args[0], UTF8)
            fn = "upper" if name == "capitalize" else name
            if isinstance(a, Lit):
                return Lit(None if a.value is None else (a.value.upper() if fn == "upper" else a.value.lower()), UTF8)
            return Func(fn, [a], UTF8)
        if name in ("substr", "substring"):
            if len(args) not in (2, 3):
                raise PlanError("substr takes 2 or 3 arguments")
            a = self._coerce(args[0], UTF8)
            if not all(isinstance(x, Lit) for x in args[1:]):
                raise NotSupported("substr with non-literal positions")
            start = int(args[1].value)
            ln = int(args[2].value) if len(args) == 3 else None
            if isinstance(a, Lit):
                from ..ops.strings import _py_substr
                return Lit(None if a.value is None else _py_substr(a.value, start, ln), UTF8)
            return Func("substr", [a], UTF8, (start, ln))
        if name in ("length", "char_length", "character_length"):
            _nargs(name, args, 1)
            return Func("char_length", [self._coerce(args[0], UTF8)], INT32)
        if name == "abs":
            _nargs(name, args, 1)
            return Func("abs", args, args[0].dtype)
        if name == "round":
            d = int(args[1].value) if len(args) > 1 else 0
            t = args[0].dtype
            if t.is_decimal:
                return Func("round", [args[0]], T.DECIMAL(t.precision, min(t.scale, max(d, 0))), (d,))
            return Func("round", [self._coerce(args[0], FLOAT64) if not t.is_integer else args[0]],
                        FLOAT64 if not t.is_integer else t, (d,))
        if name in ("coalesce", "ifnull", "nvl"):
            t = None
            for a in args:
                if a.dtype.kind != "null":
                    t = a.dtype if t is None else (t if t == a.dtype else T.common_numeric(t, a.dtype))
            t = t or T.NULL
            return Func("coalesce", [self._coerce(a, t) for a in args], t)
        if name == "nullif":
            _nargs(name, args, 2)
            return Case([(self._cmp("=", args[0], args[1]), Lit(None, args[0].dtype))], args[0], args[0].dtype)
        if name in ("date_part", "datepart"):
            if not isinstance(args[0], Lit) or not isinstance(args[0].value, str):
                raise PlanError("date_part() field must be a string literal")
            return self._date_part(args[0].value.lower(), args[1])
        if name in ("year", "month", "day", "hour", "minute", "second", "quarter", "week"):
            return self._date_part(name, args[0])
        if name in ("concat",):
            # the concat() function reads NULL arguments as '' (the || operator propagates NULL)
            parts = [a for a in args if not (isinstance(a, Lit) and a.value is None)]
            parts = [Func("coalesce", [self._coerce(a, UTF8), Lit("", UTF8)], UTF8) if a.nullable
                     else self._coerce(a, UTF8) for a in parts] or [Lit("", UTF8)]
            out = parts[0]
            for a in parts[1:]:
                out = Func("concat", [out, a], UTF8)
            return out
        if name in ("sqrt", "ln", "log10", "exp", "floor", "ceil", "ceiling"):
            _nargs(name, args, 1)
            return Func(name.replace("ceiling", "ceil"), [self._coerce(args[0], FLOAT64)], FLOAT64)
        if name in ("power", "pow"):
            return Func("power", [self._coerce(a, FLOAT64) for a in args], FLOAT64)
        if name in ("to_date",):
            return self._coerce(args[0], DATE32)
        if name == "arrow_typeof":
            _nargs(name, args, 1)
            return Lit(arrow_type_name(args[0].dtype), UTF8)
        if name in _NESTED_FUNCS:
            return self._nested_func(name, args)
        if name in ("md5", "sha224", "sha256", "sha384", "sha512", "digest"):
            if name == "digest":
                if len(args) != 2 or not isinstance(args[1], Lit) or not isinstance(args[1].value, str):
                    raise PlanError("digest(value, algorithm): the algorithm must be a string constant")
                algo = args[1].value.lower()
                if algo not in ("md5", "sha224", "sha256", "sha384", "sha512"):
                    raise NotSupported(f"digest(): algorithm '{algo}'")
            else:
                _nargs(name, args, 1)
                algo = name
            a = self._coerce(args[0], UTF8)
            if isinstance(a, Lit):
                import hashlib
                return Lit(None if a.value is None else hashlib.new(algo, a.value.encode()).hexdigest(), UTF8)
            return Func("hex_digest", [a], UTF8, (algo,))
        if name in ("uuid", "gen_random_uuid"):
            return Func("uuid", [], UTF8)
        if name in ("to_char", "date_format"):
            _nargs(name, args, 2)
            if not isinstance(args[1], Lit) or not isinstance(args[1].value, str):
                raise NotSupported(f"{name}(): the format must be a string constant")
            x = args[0]
            if x.dtype.is_string:
                x = self._coerce(x, T.TIMESTAMP)
            if x.dtype.kind not in ("date32", "timestamp"):
                raise PlanError(f"{name}() formats dates and timestamps, got {x.dtype}")
            if isinstance(x, Lit):
                from ..ops.digest import py_strftime
                mult = 86_400_000_000 if x.dtype.kind == "date32" else 1
                return Lit(None if x.value is None else py_strftime(x.value * mult, args[1].value), UTF8)
            return Func("to_char", [x], UTF8, (args[1].value,))
        return self._func_library(name, args)

    def _nested_func(self, name: str, args: List[Expr]) -> Expr:
        """LIST / STRUCT functions (DataFusion's datafusion-functions-nested,
        reference Cargo.lock:1125); evaluated by ops/nested.py."""
        def lit(i, what, kind=None):
            if len(args) <= i or not isinstance(args[i], Lit) or args[i].value is None or \
                    (kind is not None and not isinstance(args[i].value, kind)):
                raise NotSupported(f"{name}(): {what} must be a constant")
            return args[i].value

        def need_list(i=0):
            if len(args) <= i or args[i].dtype.kind != "list":
                raise PlanError(f"{name}() needs a list argument, got "
                                f"{args[i].dtype if len(args) > i else 'nothing'}")
            return args[i]
        if name in ("make_array", "make_list", "array"):
            t = None
            for a in args:
                if a.dtype.kind != "null":
                    t = a.dtype if t is None else (t if t == a.dtype else T.common_numeric(t, a.dtype))
            t = t or INT64
            return Func("make_array", [self._coerce(a, t) for a in args], T.LIST(t))
        if name in ("array_length", "cardinality", "list_length", "array_size"):
            a = need_list()
            return Func("array_length", [a], INT64)
        if name in ("array_element", "list_element", "array_extract", "list_extract", "get_field"):
            _nargs(name, args, 2)
            a = args[0]
            if a.dtype.kind == "struct":
                f = lit(1, "field name", str)
                ft = dict(a.dtype.fields).get(f)
                if ft is None:
                    raise PlanError(f"struct {a.dtype} has no field '{f}'")
                return Func("get_field", [a], ft, (f,))
            need_list()
            i = args[1]
            if isinstance(i, Lit):
                if i.value is None:
                    return Lit(None, a.dtype.child)
                return Func("array_element", [a], a.dtype.child, (int(i.value),))
            return Func("array_element", [a, self._coerce(i, INT64)], a.dtype.child)
        if name == "struct":
            names = [f"c{i}" for i in range(len(args))]
            return Func("struct", args, T.STRUCT(list(zip(names, [a.dtype for a in args]))), tuple(names))
        if name == "named_struct":
            if len(args) % 2:
                raise PlanError("named_struct() takes name, value pairs")
            names = [lit(i, "field name", str) for i in range(0, len(args), 2)]
            vals = args[1::2]
            return Func("struct", list(vals), T.STRUCT(list(zip(names, [a.dtype for a in vals]))), tuple(names))
        if name in ("array_has", "array_contains", "list_has", "list_contains"):
            a = need_list()
            v = args[1] if len(args) > 1 else None
            if not isinstance(v, Lit):
                raise NotSupported(f"{name}(): the value must be a constant")
            v = self._coerce_lit(v, a.dtype.child) if v.value is not None else v
            return Func("array_has", [a], BOOL, (v.value,))
        if name in ("array_to_string", "list_to_string", "array_join", "list_join"):
            a = need_list()
            sep = lit(1, "separator", str)
            null_str = lit(2, "null string", str) if len(args) > 2 else None
            return Func("array_to_string", [a], UTF8, (sep, null_str))
        if name == "unnest":
            a = need_list()
            return Func("unnest", [a], a.dtype.child)
        if name == "regexp_match":
            a = self._coerce(args[0], UTF8)
            pat = lit(1, "pattern", str)
            flags = lit(2, "flags", str) if len(args) > 2 else ""
            return Func("regexp_match", [a], T.LIST(UTF8), (pat, flags))
        raise NotSupported(f"function {name}()")

    def _agg_order(self, node, scope) -> List[Tuple[Expr, bool, bool]]:
        out = []
        for o in _lst(node):
            asc = not o.get("desc")
            nf = o.get("nulls", "last" if asc else "first") == "first"
            out.append((self.bind_expr(o["c"][0], scope), asc, nf))
        return out

    def _date_part(self, field: str, x: Expr) -> Expr:
        field = {"years": "year", "months": "month", "days": "day", "dayofweek": "dow", "dayofyear": "doy",
                 "hours": "hour", "minutes": "minute", "seconds": "second", "weeks": "week"}.get(field, field)
        date_fields = ("year", "month", "day", "quarter", "dow", "doy", "week")
        time_fields = ("hour", "minute", "second", "millisecond", "microsecond", "epoch")
        if field not in date_fields + time_fields:
            raise NotSupported(f"EXTRACT({field})")
        if x.dtype.is_string:
            x = self._coerce(x, T.TIMESTAMP if field in time_fields else DATE32)
        if x.dtype.kind == "timestamp" or field in time_fields:
            x = self._to_ts(x)
            rt = FLOAT64 if field == "epoch" else INT32
            if isinstance(x, Lit):
                from ..exec.expr_eval import ts_part_py
                return Lit(None if x.value is None else ts_part_py(x.value, field), rt)
            return Func("ts_part", [x], rt, (field,))
        x = self._coerce(x, DATE32)
        if isinstance(x, Lit):
            return Lit(None if x.value is None else _date_part_py(x.value, field), INT32)
        return Func("date_part", [x], INT32, (field,))

    # ------------------------------------------------------ function library
    def _func_library(self, name: str, args: List[Expr]) -> Expr:
        """DataFusion built-ins beyond the TPC-H set (strings, math, dates)."""
        from ..ops import strfuncs as SF

        def lit_str(i, what):
            if len(args) <= i or not isinstance(args[i], Lit) or not isinstance(args[i].value, str):
                raise NotSupported(f"{name}(): {what} must be a string literal")
            return args[i].value

        def lit_int(i, what):
            if len(args) <= i or not isinstance(args[i], Lit) or not isinstance(args[i].value, int):
                raise NotSupported(f"{name}(): {what} must be an integer literal")
            return int(args[i].value)

        def strfn(fname, opts, rt=UTF8):
            a = self._coerce(args[0], UTF8)
            if isinstance(a, Lit):
                return Lit(None if a.value is None else SF.py_fn(fname, opts)(a.value), rt)
            return Func(fname, [a], rt, opts)
        if not args and name not in ("pi", "random", "now", "current_timestamp", "current_date", "today",
                                     "uuid", "current_time"):
            raise PlanError(f"{name}() needs arguments")
        # ---- strings
        if name in ("btrim", "trim", "ltrim", "rtrim"):
            chars = lit_str(1, "trim characters") if len(args) > 1 else " "
            return strfn("trim", ({"ltrim": 1, "rtrim": 2}.get(name, 3), chars))
        if name == "replace":
            return strfn("replace", (lit_str(1, "search string"), lit_str(2, "replacement")))
        if name in ("lpad", "rpad"):
            return strfn(name, (lit_int(1, "length"), lit_str(2, "fill") if len(args) > 2 else " "))
        if name in ("reverse", "initcap"):
            return strfn(name, ())
        if name == "repeat":
            return strfn("repeat", (lit_int(1, "count"),))
        if name in ("left", "right"):
            return strfn(name, (lit_int(1, "length"),))
        if name == "translate":
            return strfn("translate", (lit_str(1, "from"), lit_str(2, "to")))
        if name == "split_part":
            return strfn("split_part", (lit_str(1, "delimiter"), lit_int(2, "part")))
        if name in ("strpos", "instr"):
            return strfn("strpos", (lit_str(1, "substring"),), INT32)
        if name == "ascii":
            return strfn("ascii", (), INT32)
        if name in ("octet_length",):
            return strfn("octet_length", (), INT32)
        if name == "bit_length":
            return BinOp("*", Cast(strfn("octet_length", (), INT32), INT64), Lit(8, INT64), INT64)
        if name in ("starts_with", "ends_with"):
            p = _like_escape(lit_str(1, "prefix"))
            return Like(self._coerce(args[0], UTF8), p + "%" if name == "starts_with" else "%" + p)
        if name == "concat_ws":
            sep = lit_str(0, "separator")
            return self._concat_ws(sep, args[1:])
        if name in ("regexp_like", "regexp_replace", "regexp_count"):
            a = self._coerce(args[0], UTF8)
            pat = lit_str(1, "pattern")
            if name == "regexp_replace":
                rep = lit_str(2, "replacement")
                flags = lit_str(3, "flags") if len(args) > 3 else ""
                return Func(name, [a], UTF8, (pat, rep, flags))
            flags = lit_str(2, "flags") if len(args) > 2 else ""
            return Func(name, [a], BOOL if name == "regexp_like" else INT64, (pat, flags))
        if name == "chr":
            if isinstance(args[0], Lit):
                return Lit(None if args[0].value is None else chr(int(args[0].value)), UTF8)
            raise NotSupported("chr() of a column")
        if name == "to_hex":
            if isinstance(args[0], Lit):
                return Lit(None if args[0].value is None else format(int(args[0].value) & (2**64 - 1), "x"), UTF8)
            raise NotSupported("to_hex() of a column")
        # ---- math
        if name == "mod":
            return self._arith("%", args[0], args[1])
        if name in ("sign", "signum", "trunc", "log2", "cbrt", "degrees", "radians", "sin", "cos", "tan", "asin",
                    "acos", "atan", "sinh", "cosh", "tanh", "isnan", "iszero", "factorial"):
            x = self._coerce(args[0], FLOAT64) if name != "factorial" else self._coerce(args[0], INT64)
            if name == "trunc" and len(args) > 1:
                return Func("trunc", [x], FLOAT64, (lit_int(1, "precision"),))
            rt = BOOL if name in ("isnan", "iszero") else (INT64 if name == "factorial" else FLOAT64)
            return Func(name.replace("signum", "sign"), [x], rt)
        if name == "log":
            if len(args) == 1:
                return Func("log10", [self._coerce(args[0], FLOAT64)], FLOAT64)
            return Func("logb", [self._coerce(args[0], FLOAT64), self._coerce(args[1], FLOAT64)], FLOAT64)
        if name in ("atan2", "nanvl"):
            return Func(name, [self._coerce(a, FLOAT64) for a in args[:2]], FLOAT64)
        if name == "pi":
            return Lit(3.141592653589793, FLOAT64)
        if name == "random":
            return Func("random", [], FLOAT64)
        if name in ("greatest", "least"):
            t = None
            for a in args:
                if a.dtype.kind != "null":
                    t = a.dtype if t is None else (t if t == a.dtype else T.common_numeric(t, a.dtype))
            t = t or T.NULL
            if t.is_string:
                raise NotSupported(f"{name}() over strings")
            return Func(name, [self._coerce(a, t) for a in args], t)
        if name in ("gcd", "lcm"):
            return Func(name, [self._coerce(a, INT64) for a in args[:2]], INT64)
        if name == "nvl2":
            t = _common(args[1].dtype, args[2].dtype)
            return Case([(IsNull(args[0], True), self._coerce(args[1], t))], self._coerce(args[2], t), t)
        # ---- dates and timestamps
        if name in ("now", "current_timestamp"):
            return Lit(self._now_us(), T.TIMESTAMP)
        if name in ("current_date", "today"):
            return Lit(self._now_us() // 86_400_000_000, DATE32)
        if name == "date_trunc":
            unit = lit_str(0, "unit").lower()
            if unit not in _TRUNC_UNITS:
                raise PlanError(f"date_trunc unit '{unit}' is not supported")
            x = args[1]
            if x.dtype.is_string:
                x = self._coerce(x, T.TIMESTAMP)
            x = self._to_ts(x)
            if isinstance(x, Lit):
                from ..exec.expr_eval import trunc_ts_py
                return Lit(None if x.value is None else trunc_ts_py(x.value, unit), T.TIMESTAMP)
            return Func("date_trunc", [x], T.TIMESTAMP, (unit,))
        if name in ("to_timestamp", "to_timestamp_micros", "to_timestamp_millis", "to_timestamp_seconds",
                    "from_unixtime"):
            x = args[0]
            if x.dtype.is_string:
                if isinstance(x, Lit):
                    return _fold_cast(x, T.TIMESTAMP)
                return Cast(x, T.TIMESTAMP)
            scale = {"to_timestamp_micros": 1, "to_timestamp_millis": 1000}.get(name, 1_000_000)
            if name == "to_timestamp" and x.dtype.is_float:
                return Func("ts_from_float", [x], T.TIMESTAMP)
            return self._arith_ts_scale(self._coerce(x, INT64), scale)
        if name == "to_unixtime":
            return Func("to_unixtime", [self._to_ts(args[0])], INT64)
        if name == "make_date":
            return Func("make_date", [self._coerce(a, INT64) for a in args[:3]], DATE32)
        raise NotSupported(f"function {name}()")

    def _now_us(self) -> int:
        now = getattr(self, "_now", None)
        if now is None:
            import time as _t
            now = self._now = int(_t.time() * 1_000_000)
        return now

    def _to_ts(self, x: Expr) -> Expr:
        if x.dtype.kind == "timestamp":
            return x
        if x.dtype.kind == "date32":
            if isinstance(x, Lit):
                return Lit(None if x.value is None else x.value * 86_400_000_000, T.TIMESTAMP)
            return Cast(x, T.TIMESTAMP)
        return self._coerce(x, T.TIMESTAMP)

    def _arith_ts_scale(self, x: Expr, scale: int) -> Expr:
        if isinstance(x, Lit):
            return Lit(None if x.value is None else int(x.value) * scale, T.TIMESTAMP)
        return Cast(BinOp("*", x, Lit(scale, INT64), INT64), T.TIMESTAMP)

    def _concat_ws(self, sep: str, parts: List[Expr]) -> Expr:
        """concat_ws(sep, a, b, ...): the non-NULL arguments joined by sep."""
        out: Optional[Expr] = None
        seen: Optional[Expr] = None   # some earlier argument is not NULL
        for p in parts:
            p = self._coerce(p, UTF8)
            if isinstance(p, Lit) and p.value is None:
                continue
            if out is None:
                out = Func("coalesce", [p, Lit("", UTF8)], UTF8) if p.nullable else p
                seen = IsNull(p, True) if p.nullable else Lit(True, BOOL)
                continue
            piece: Expr = Func("concat", [Lit(sep, UTF8), p], UTF8)
            if p.nullable or not (isinstance(seen, Lit) and seen.value):
                piece = Case([(IsNull(p), Lit("", UTF8)), (seen, piece)], p, UTF8)
            out = Func("concat", [out, piece], UTF8)
            seen = Lit(True, BOOL) if not p.nullable else BinOp("or", seen, IsNull(p, True), BOOL)
        return out if out is not None else Lit("", UTF8)

    # ------------------------------------------------------------ windows
    def _window_call(self, name: str, node, scope, allow_agg) -> Expr:
        if not allow_agg:
            raise PlanError(f"window function {name}() is only allowed in SELECT, QUALIFY and ORDER BY")
        if node.get("distinct"):
            raise NotSupported("DISTINCT in a window aggregate")
        spec = self._window_spec(node["over"])
        part = [self.bind_expr(e, scope, allow_agg=True) for e in _lst(spec.get("partition"))]
        order = []
        for o in _lst(spec.get("order")):
            e = self.bind_expr(o["c"][0], scope, allow_agg=True)
            asc = not o.get("desc")
            order.append((e, asc, o.get("nulls", "last" if asc else "first") == "first"))
        args = [self.bind_expr(a, scope, allow_agg=True) for a in node["c"]]
        flt = self.bind_expr(node["filter"], scope, allow_agg=True) if node.get("filter") else None
        frame = self._frame(spec.get("frame"), order)
        if name in RANKING_FUNCS:
            opts: tuple = ()
            if name == "ntile":
                if len(args) != 1 or not isinstance(args[0], Lit) or not isinstance(args[0].value, int) \
                        or args[0].value <= 0:
                    raise PlanError("ntile() takes one positive integer literal")
                opts = (int(args[0].value),)
            elif args:
                raise PlanError(f"{name}() takes no arguments")
            dt = FLOAT64 if name in ("percent_rank", "cume_dist") else INT64
            return WindowCall(name, [], part, order, frame, dt, None, opts)
        if name in VALUE_FUNCS:
            if not args:
                raise PlanError(f"{name}() needs an argument")
            x = args[0]
            if name in ("lag", "lead"):
                if len(args) > 3:
                    raise PlanError(f"{name}() takes at most 3 arguments")
                k = 1
                if len(args) > 1:
                    if not isinstance(args[1], Lit) or not isinstance(args[1].value, int):
                        raise NotSupported(f"{name}() offset must be an integer literal")
                    k = int(args[1].value)
                wargs = [x]
                t = x.dtype
                if len(args) > 2 and not (isinstance(args[2], Lit) and args[2].value is None):
                    if not isinstance(args[2], Lit):
                        raise NotSupported(f"{name}() default must be a literal")
                    if t.kind == "null":
                        t = args[2].dtype
                    wargs.append(self._coerce(args[2], t))
                return WindowCall("lag", wargs, part, order, frame, t, None, (k if name == "lag" else -k,))
            if name == "nth_value":
                if len(args) != 2 or not isinstance(args[1], Lit) or not isinstance(args[1].value, int) \
                        or args[1].value < 1:
                    raise PlanError("nth_value(x, n) needs a positive integer literal n")
                return WindowCall(name, [x], part, order, frame, x.dtype, None, (int(args[1].value),))
            if len(args) != 1:
                raise PlanError(f"{name}() takes one argument")
            return WindowCall(name, [x], part, order, frame, x.dtype)
        if name in AGG_FUNCS or name in _EXTRA_AGGS:
            if node.get("star") or not args:
                arg = None
            elif len(args) == 1:
                arg = args[0]
            else:
                raise NotSupported(f"window aggregate {name} with {len(args)} arguments")
            a = _make_agg(name, arg, False, None)
            if a.func not in _WINDOW_AGGS:
                raise NotSupported(f"{name}() as a window function")
            return WindowCall(a.func, [arg] if arg is not None else [], part, order, frame, a.dtype, flt)
        raise NotSupported(f"window function {name}()")

    def _window_spec(self, w: dict) -> dict:
        """Named-window references merged with the inline spec."""
        out: dict = {}
        if w.get("s"):
            named = (getattr(self, "_win_defs", None) or {}).get(w["s"])
            if named is None:
                raise PlanError(f"window '{w['s']}' is not defined")
            out = dict(self._window_spec(named))
        for k in ("partition", "order", "frame"):
            if w.get(k):
                out[k] = w[k]
        return out

    def _frame(self, fr: Optional[dict], order) -> WindowFrame:
        if fr is None:
            if order:
                return WindowFrame("range", "unbounded_preceding", "current")
            return WindowFrame("rows", "unbounded_preceding", "unbounded_following")
        unit = fr["s"]
        (sb, eb) = fr["c"]
        sk, ek = sb["s"], eb["s"]
        if sk == "unbounded_following" or ek == "unbounded_preceding" or FRAME_KINDS.index(sk) > FRAME_KINDS.index(ek):
            raise PlanError("window frame start cannot be after its end")

        def off(b):
            if b["s"] not in ("preceding", "following"):
                return None
            v = self.bind_expr(b["c"][0], Scope([]))
            if not isinstance(v, Lit) or v.value is None:
                raise PlanError("window frame offset must be a constant")
            if unit in ("rows", "groups"):
                if not isinstance(v.value, int) or v.value < 0:
                    raise PlanError(f"{unit.upper()} frame offset must be a non-negative integer")
                return int(v.value)
            if len(order) != 1:
                raise PlanError("RANGE with an offset needs exactly one ORDER BY key")
            kt = order[0][0].dtype
            if v.dtype == INTERVAL:
                months, days, us = v.value
                if months:
                    raise NotSupported("RANGE offsets in months")
                if kt.kind == "timestamp":
                    return Lit(days * 86_400_000_000 + us, INT64)
                if us or kt.kind != "date32":
                    raise PlanError("RANGE interval offset over a non-temporal key")
                return Lit(days, INT64)
            if kt.kind == "date32":
                return Lit(int(v.value), INT64)
            if not kt.is_numeric:
                raise PlanError(f"RANGE offset over a {kt} key")
            lv = self._coerce_lit(v, kt) if v.dtype != kt else v
            if kt.is_decimal and lv.dtype.is_decimal and lv.dtype.scale != kt.scale:
                lv = _fold_cast(lv, kt)
            if (lv.value or 0) < 0:
                raise PlanError("RANGE offset must not be negative")
            return lv
        return WindowFrame(unit, sk, ek, off(sb), off(eb))

    def _display_name(self, ast: dict, e: Expr) -> str:
        if isinstance(e, ColRef) and ast["k"] == "col":
            return e.name
        return _ast_text(ast)


class _Passthrough(ColRef):
    """Group key that is the projected column itself (DISTINCT)."""

    def __init__(self, c: ColInfo):
        super().__init__(c.cid, c.name, c.dtype, c.nullable)


# ---------------------------------------------------------------------- helpers
#: aggregates computed by the window operator (exec/window.py)
_WINDOW_AGGS = ("sum", "count", "avg", "min", "max", "stddev", "stddev_samp", "stddev_pop", "var", "var_samp",
                "var_pop", "bool_and", "bool_or")
_EXTRA_AGGS = ("stddev_samp", "stddev_pop", "var_samp", "var_pop", "variance", "var_population", "stddev_population",
               "median", "approx_distinct", "approx_median", "string_agg", "array_agg", "bit_and", "bit_or",
               "bit_xor", "percentile_cont", "percentile_disc", "covar", "covar_samp", "covar_pop", "corr", "approx_percentile_cont", "first_value",
               "last_value", "every", "any", "some")


_TRUNC_UNITS = ("microsecond", "millisecond", "second", "minute", "hour", "day", "week", "month", "quarter", "year")


_NESTED_FUNCS = ("make_array", "make_list", "array", "array_length", "cardinality", "list_length", "array_size",
                 "array_element", "list_element", "array_extract", "list_extract", "get_field", "struct",
                 "named_struct", "array_has", "array_contains", "list_has", "list_contains", "array_to_string",
                 "list_to_string", "array_join", "list_join", "unnest", "regexp_match")


def similar_to_regex(pat: str, esc: str = "\\") -> str:
    """SQL ``SIMILAR TO`` pattern -> an anchored regular expression: ``%`` and
    ``_`` are the LIKE wildcards, ``| * + ? {m,n} ( ) [...]`` keep their regex
    meaning, everything else (``.`` included) is literal."""
    import re as _re
    out, i, n = [], 0, len(pat)
    while i < n:
        ch = pat[i]
        if esc and ch == esc and i + 1 < n:
            out.append(_re.escape(pat[i + 1]))
            i += 2
            continue
        if ch == "%":
            out.append(".*")
        elif ch == "_":
            out.append(".")
        elif ch in "|*+?(){},":
            out.append(ch)
        elif ch == "[":
            j = pat.find("]", i + 2 if i + 1 < n and pat[i + 1] in "^]" else i + 1)
            if j < 0:
                raise PlanError("SIMILAR TO: unterminated bracket expression")
            out.append(pat[i:j + 1])
            i = j + 1
            continue
        else:
            out.append(_re.escape(ch))
        i += 1
    return "^(?:" + "".join(out) + ")$"


def arrow_type_name(t: DataType) -> str:
    """DataFusion's ``arrow_typeof`` spelling of a type (Arrow DataType Display)."""
    k = t.kind
    if k == "decimal":
        return f"Decimal128({t.precision}, {t.scale})"
    if k == "timestamp":
        return "Timestamp(Microsecond, None)"
    if k == "list":
        return f"List(Field {{ name: \"item\", data_type: {arrow_type_name(t.child)}, nullable: true, dict_id: 0, " \
               f"dict_is_ordered: false, metadata: {{}} }})"
    if k == "struct":
        return "Struct(" + ", ".join(f"{n} {arrow_type_name(ft)}" for n, ft in t.fields) + ")"
    return str(t)


def _like_escape(s: str) -> str:
    return s.replace("\\", "\\\\").replace("%", "\\%").replace("_", "\\_")


def _common(a: DataType, b: DataType) -> DataType:
    if a.kind == "null":
        return b
    if b.kind == "null" or a == b:
        return a
    return T.common_numeric(a, b)


def _distinct_from(distinct: bool, l: Expr, r: Expr) -> Expr:
    """a IS [NOT] DISTINCT FROM b: NULL-safe (in)equality, never NULL."""
    eq = "<>" if distinct else "="
    if isinstance(l, Lit) and l.value is None:
        l, r = r, l
    if isinstance(r, Lit) and r.value is None:
        if isinstance(l, Lit):
            return Lit((l.value is not None) == distinct, BOOL)
        return IsNull(l, negated=distinct)
    if not l.nullable and not r.nullable:
        return _fold(BinOp(eq, l, r, BOOL))
    both = BinOp("and", IsNull(l), IsNull(r), BOOL)
    one = BinOp("or", IsNull(l), IsNull(r), BOOL)
    return Case([(both, Lit(not distinct, BOOL)), (one, Lit(distinct, BOOL))], BinOp(eq, l, r, BOOL), BOOL)


def _default_lit(t: DataType) -> Lit:
    if t.is_string:
        return Lit("", t)
    if t.kind == "bool":
        return Lit(False, t)
    if t.is_float:
        return Lit(0.0, t)
    return Lit(0, t)


def _is_recursive_cte(c: dict) -> bool:
    """A CTE body of the form anchor UNION [ALL] term, the term reading the CTE itself."""
    body = c["query"]["body"]
    if body["k"] != "setop" or not body["s"].startswith("union"):
        return False
    return _mentions_table(body["c"][1], c["s"])


def _mentions_table(n, name: str) -> bool:
    if isinstance(n, dict):
        if n.get("k") == "table" and n.get("s") == name:
            return True
        return any(_mentions_table(v, name) for k, v in n.items() if k not in ("k", "s", "pos"))
    if isinstance(n, list):
        return any(_mentions_table(v, name) for v in n)
    return False


def _expand_group_by(items: list):
    """GROUP BY items -> (key expression nodes, grouping sets as lists of
    positions into them, or None when no ROLLUP / CUBE / GROUPING SETS)."""
    if not any(it["k"] in ("rollup", "cube", "grouping_sets") for it in items):
        return items, None
    keys: list = []

    def pos(e):
        keys.append(e)
        return len(keys) - 1

    def elem(lst):  # a grouping element: list node of expressions
        return [pos(e) for e in lst["c"]]

    def item_sets(it):
        k = it["k"]
        if k == "rollup":
            els = [elem(x) for x in it["c"]]
            return [sum(els[:i], []) for i in range(len(els), -1, -1)]
        if k == "cube":
            els = [elem(x) for x in it["c"]]
            out = []
            for mask in range((1 << len(els)) - 1, -1, -1):
                out.append(sum((els[i] for i in range(len(els)) if mask >> (len(els) - 1 - i) & 1), []))
            return out
        if k == "grouping_sets":
            out = []
            for x in it["c"]:
                if x["k"] in ("rollup", "cube"):
                    out += item_sets(x)
                else:
                    out.append(elem(x))
            return out
        return [[pos(it)]]

    sets = [[]]
    for it in items:
        sets = [a + b for a in sets for b in item_sets(it)]
    if len(sets) > 4096:
        raise PlanError("too many grouping sets")
    return keys, sets


def _contains_grouping(e: Expr) -> bool:
    return any(isinstance(x, Func) and x.name == "grouping" for x in walk(e))


def _rename(p: Project, schema: List[ColInfo]) -> Project:
    return Project(p.input, [(s, e) for s, (_, e) in zip(schema, p.exprs)])


def _contains_agg(e: Expr) -> bool:
    for x in walk(e):
        if isinstance(x, AggCall):
            return True
    return False


def _transform_top_down(e: Expr, fn) -> Expr:
    r = fn(e)
    if r is not None:
        return r
    kids = e.children()
    if not kids:
        return e
    new = [_transform_top_down(k, fn) for k in kids]
    if any(a is not b for a, b in zip(new, kids)):
        # SubqueryExpr keeps its plan; other nodes rebuild from children
        return e.with_children(new)
    return e


def _nargs(name, args, n):
    if len(args) != n:
        raise PlanError(f"{name}() takes {n} argument(s)")


def _int_as_decimal(e: Expr) -> DataType:
    if isinstance(e, Lit) and isinstance(e.value, int):
        return T.DECIMAL(max(len(str(abs(e.value))), 1), 0)
    return T.DECIMAL(19 if e.dtype.kind == "int64" else 10, 0)


_AGG_ALIASES = {"mean": "avg", "variance": "var_samp", "var": "var_samp", "var_population": "var_pop",
                "stddev": "stddev_samp", "stddev_population": "stddev_pop", "approx_median": "median",
                "covar": "covar_samp", "every": "bool_and", "any": "bool_or", "some": "bool_or"}


def _make_agg(name: str, arg: Optional[Expr], distinct: bool, flt, arg2: Optional[Expr] = None,
              param=None, order: Tuple = ()) -> AggCall:
    name = _AGG_ALIASES.get(name, name)
    if name == "count":
        return AggCall("count", arg, distinct, INT64, flt)
    if name == "approx_distinct":
        # exact distinct count (a valid answer for the approximate function)
        if arg is None:
            raise PlanError("approx_distinct(*) is not valid")
        return AggCall("count", arg, True, INT64, flt)
    if arg is None:
        raise PlanError(f"{name}(*) is not valid")
    t = arg.dtype
    if name == "sum":
        if t.is_integer or t.kind == "bool":
            rt = INT64
        elif t.is_decimal:
            rt = T.DECIMAL(min(38, t.precision + 10), t.scale)
        elif t.is_float:
            rt = FLOAT64
        else:
            raise PlanError(f"sum({t}) is not supported")
        return AggCall("sum", arg, distinct, rt, flt)
    if name == "avg":
        if t.is_decimal:
            rt = T.DECIMAL(min(38, t.precision + 4), min(38, t.scale + 4))
        elif t.is_numeric:
            rt = FLOAT64
        else:
            raise PlanError(f"avg({t}) is not supported")
        return AggCall("avg", arg, distinct, rt, flt)
    if name in ("min", "max", "first_value", "last_value"):
        return AggCall(name if name not in ("first_value", "last_value") else
                       ("min" if name == "first_value" else "max"), arg, distinct, t, flt)
    if name in ("stddev_samp", "stddev_pop", "var_samp", "var_pop"):
        if not t.is_numeric:
            raise PlanError(f"{name}({t}) is not supported")
        return AggCall(name, arg, distinct, FLOAT64, flt)
    if name in ("bool_and", "bool_or"):
        return AggCall(name, arg, distinct, BOOL, flt)
    if name == "median":
        if not t.is_numeric:
            raise PlanError(f"median({t}) is not supported")
        return AggCall("median", arg, distinct, t, flt)
    if name in ("approx_percentile_cont", "percentile_cont"):
        if not t.is_numeric:
            raise PlanError(f"{name}({t}) is not supported")
        return AggCall("percentile", arg, False, FLOAT64, flt, None, param)
    if name == "percentile_disc":
        if not (t.is_numeric or t.is_temporal):
            raise PlanError(f"percentile_disc({t}) is not supported")
        return AggCall("percentile_disc", arg, False, t, flt, None, param)
    if name in ("bit_and", "bit_or", "bit_xor"):
        if not t.is_integer:
            raise PlanError(f"{name}({t}) needs an integer argument")
        return AggCall(name, arg, distinct, t, flt)
    if name == "string_agg":
        if not t.is_string:
            raise PlanError("string_agg() needs a string argument")
        return AggCall("string_agg", arg, distinct, UTF8, flt, None, param, order)
    if name in ("covar_samp", "covar_pop", "corr"):
        if not (t.is_numeric and arg2 is not None and arg2.dtype.is_numeric):
            raise PlanError(f"{name}() needs two numeric arguments")
        return AggCall(name, arg, False, FLOAT64, flt, arg2)
    if name == "array_agg":
        return AggCall("array_agg", arg, distinct, T.LIST(t), flt, None, None, order)
    raise NotSupported(f"aggregate {name}")


def _parse_interval(s: str, unit: Optional[str]) -> Tuple[int, int]:
    """'3' month / '1 year' / '90 days' -> (months, days)."""
    txt = s.strip().lower()
    parts = txt.split()
    if unit is None:
        if len(parts) == 2:
            txt, unit = parts
        else:
            unit = "day"
    d = Decimal(txt.split()[0])
    n = int(d)
    unit = unit.rstrip("s")
    if unit == "year":
        return (12 * n, 0, 0)
    if unit == "month":
        return (n, 0, 0)
    if unit == "week":
        return (0, 7 * n, 0)
    if unit == "day":
        return (0, n, 0)
    if unit == "hour":
        return (0, 0, int(d * 3_600_000_000))
    if unit == "minute":
        return (0, 0, int(d * 60_000_000))
    if unit == "second":
        return (0, 0, int(d * 1_000_000))
    if unit in ("millisecond", "milli"):
        return (0, 0, int(d * 1000))
    if unit in ("microsecond", "micro"):
        return (0, 0, n)
    raise NotSupported(f"interval unit {unit}")


def _date_part_py(days: int, field: str) -> int:
    d = days_to_date(days)
    return {"year": d.year, "month": d.month, "day": d.day, "quarter": (d.month - 1) // 3 + 1,
            "dow": (d.weekday() + 1) % 7, "doy": d.timetuple().tm_yday, "week": d.isocalendar()[1]}[field]


def _fold_cast(v: Lit, t: DataType) -> Lit:
    if TPL.tracking(v):
        return TPL.derive(lambda a, t=t: _fold_cast(a, t), v)
    x = v.value
    if x is None:
        return Lit(None, t)
    src = v.dtype
    try:
        if t.is_decimal:
            if src.is_decimal:
                ds = t.scale - src.scale
                return Lit(x * 10**ds if ds >= 0 else _round_div(x, 10**(-ds)), t)
            if src.is_integer:
                return Lit(int(x) * 10**t.scale, t)
            if src.is_float or src.is_string:
                return Lit(int((Decimal(str(x)) * (10**t.scale)).to_integral_value()), t)
        if t.is_integer:
            if src.is_decimal:
                return Lit(int(Decimal(x) / (10**src.scale)), t)
            return Lit(int(float(x)) if src.is_string else int(x), t)
        if t.is_float:
            if src.is_decimal:
                return Lit(x / 10**src.scale, t)
            return Lit(float(x), t)
        if t.is_string:
            if src.is_decimal:
                return Lit(Lit(x, src).sql(), t)
            if src.kind == "date32":
                return Lit(str(days_to_date(x)), t)
            if src.kind == "bool":
                return Lit("true" if x else "false", t)
            return Lit(str(x), t)
        if t.kind == "date32":
            if src.is_string:
                return Lit(date_to_days(x), t)
            if src.kind == "timestamp":
                return Lit(int(x) // 86_400_000_000, t)
            return Lit(int(x), t)
        if t.kind == "timestamp":
            if src.is_string:
                dt = datetime.datetime.fromisoformat(x.strip().replace("T", " ").rstrip("Z"))
                if dt.tzinfo is not None:
                    dt = dt.astimezone(datetime.timezone.utc).replace(tzinfo=None)
                return Lit((dt - datetime.datetime(1970, 1, 1)) // datetime.timedelta(microseconds=1), t)
            if src.kind == "date32":
                return Lit(int(x) * 86_400_000_000, t)
            return Lit(int(x), t)
        if t.kind == "bool":
            if src.is_string:
                return Lit(x.lower() in ("true", "t", "1", "yes"), t)
            return Lit(bool(x), t)
    except (ValueError, ArithmeticError) as e:
        raise PlanError(f"cannot cast {v.sql()} to {t}") from e
    return Lit(x, t)


def _round_div(a: int, b: int) -> int:
    q, r = divmod(abs(a), b)
    if 2 * r >= b:
        q += 1
    return q if a >= 0 else -q


def _fold(e: Expr) -> Expr:
    """Constant-fold binary operations on literals."""
    if not isinstance(e, BinOp) or not isinstance(e.left, Lit) or not isinstance(e.right, Lit):
        return e
    if TPL.tracking(e.left, e.right):
        return TPL.derive(lambda a, b, op=e.op, t=e.dtype: _fold(BinOp(op, a, b, t)), e.left, e.right)
    a, b = e.left.value, e.right.value
    op = e.op
    if op in ("and", "or"):
        if op == "and":
            if a is False or b is False:
                return Lit(False, BOOL)
            if a is None or b is None:
                return Lit(None, BOOL)
            return Lit(True, BOOL)
        if a is True or b is True:
            return Lit(True, BOOL)
        if a is None or b is None:
            return Lit(None, BOOL)
        return Lit(False, BOOL)
    if a is None or b is None:
        return Lit(None, e.dtype)
    lt, rt = e.left.dtype, e.right.dtype
    try:
        if op in ("=", "<>", "<", "<=", ">", ">="):
            import operator as o
            f = {"=": o.eq, "<>": o.ne, "<": o.lt, "<=": o.le, ">": o.gt, ">=": o.ge}[op]
            return Lit(bool(f(a, b)), BOOL)
        t = e.dtype
        if t.is_decimal:
            if op in ("+", "-"):
                return Lit(a + b if op == "+" else a - b, t)
            if op == "*":
                return Lit(a * b, t)
            if op == "%":
                return Lit(int(__import__("math").fmod(a, b)), t)
        if t.is_float:
            fa = a / 10**lt.scale if lt.is_decimal else float(a)
            fb = b / 10**rt.scale if rt.is_decimal else float(b)
            if op == "+":
                return Lit(fa + fb, t)
            if op == "-":
                return Lit(fa - fb, t)
            if op == "*":
                return Lit(fa * fb, t)
            if op == "/":
                return Lit(fa / fb if fb != 0 else None, t)
        if t.is_integer or t.kind == "date32":
            if op == "+":
                return Lit(a + b, t)
            if op == "-":
                return Lit(a - b, t)
            if op == "*":
                return Lit(a * b, t)
            if op == "/":
                return Lit(int(a / b) if b != 0 else None, t)
            if op == "%":
                return Lit(int(__import__("math").fmod(a, b)) if b != 0 else None, t)
    except (TypeError, ZeroDivisionError):
        return e
    return e


_OPS_TXT = {"and": "AND", "or": "OR"}


def _ast_text(n: dict) -> str:
    """Readable column name for an unaliased select expression (DataFusion-like)."""
    k = n["k"]
    if k == "col":
        return ".".join(p["s"] for p in n["c"])
    if k == "lit":
        t = n.get("type")
        if t == "str":
            return "Utf8(\"" + n["s"] + "\")"
        if t == "int":
            return f"Int64({n['s']})"
        if t == "date":
            return f"Date32(\"{n['s']}\")"
        return n["s"]
    if k == "bin":
        return f"{_ast_text(n['c'][0])} {_OPS_TXT.get(n['s'], n['s'])} {_ast_text(n['c'][1])}"
    if k == "paren":
        return _ast_text(n["c"][0])
    if k == "func":
        if n.get("star"):
            return f"{n['s']}(*)"
        d = "DISTINCT " if n.get("distinct") else ""
        return f"{n['s']}({d}{', '.join(_ast_text(c) for c in n['c'])})"
    if k == "un":
        return ("NOT " if n["s"] == "not" else "-") + _ast_text(n["c"][0])
    if k == "cast":
        return f"CAST({_ast_text(n['c'][0])} AS {n['type']})"
    if k == "case":
        return "CASE ... END"
    if k == "extract":
        return f"date_part(Utf8(\"{n['s']}\"),{_ast_text(n['c'][0])})"
    return k
