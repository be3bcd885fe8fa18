"""Statement templates: a query that differs from an earlier one only in its
literal values reuses that query's bound and optimized plan with the new
values put in, instead of being parsed, bound and optimized again.

TPC-H's power and throughput tests (and any serving workload) send the same
statements with fresh substitution parameters; planning them from scratch
costs ~1.2 ms per statement of host time in front of every execution (parse
0.2, bind 0.7, optimize 0.4). The reference plans every statement through
DataFusion's SQL planner (reference crates/engine/src/lib.rs:54-57); this
engine keys the planned statement on its *template* -- the SQL text with
every numeric / string literal token replaced by a typed marker -- and
records, while planning the first statement of a template, how each literal
reached the plan:

* passed through: the literal's own ``Lit`` object sits in the plan
  (``SlotLit``) and is swapped for the new value's;
* derived: constant folding, casts and coercions, date +/- interval,
  negation compute a literal from literal operands (``derive``): the
  derivation is kept with its result (``DerivedLit``) and re-run on the new
  operands;
* copied into a plan field (the LIKE pattern string, ``raw``): the field is
  recomputed from the new literal;
* read in any other way (``Lit.value`` read during binding or optimization:
  LIMIT counts, substring positions, function options, a value that
  decides the plan's shape): the template is keyed on that literal's exact
  text -- a different value plans afresh.

A recorded template is verified before it is used: the statement is planned
a second time with every literal perturbed (numbers +1, dates +1 day, the
last alphanumeric character of a string shifted) and the template
instantiated with the same perturbed values must serialize to the identical
plan (sql/serde.py). Only verified templates serve statements; an
instantiation whose derived literals change type or NULL-ness, or whose
re-derivation fails, plans afresh.
"""
from __future__ import annotations

import copy
import datetime
import re
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..utils import switches as _sw
from .expr import Lit

#: IGLOO_DEBUG=templates: print why a template was not recorded, not verified or not instantiated
DEBUG = _sw.debug("templates")


def why(msg: str) -> None:
    if DEBUG:
        print(f"[template] {msg}", flush=True)

# ------------------------------------------------------------------ lexing
# one alternation, leftmost first: comments, quoted identifiers and string
# literals are consumed whole (a digit inside them is not a number token)
_TOKEN = re.compile(r"""
    (?P<comment>--[^\n]*|/\*.*?\*/)
  | (?P<ident>"(?:[^"]|"")*"|`[^`]*`)
  | (?P<str>'(?:[^']|'')*')
  | (?P<num>(?<![\w$.])(?:\d+\.\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?(?![\w.]))
""", re.X | re.S)


@dataclass
class Lexed:
    """A statement split into its template text and its literal tokens."""
    key: str
    spans: List[Tuple[int, int]]        # [start, end) of each literal token in the SQL
    texts: List[str]                    # decoded text (string contents / number spelling)
    kinds: List[str]                    # 'str' | 'int' | 'dec' | 'float'


def _num_kind(s: str) -> str:
    if "e" in s or "E" in s:
        return "float"
    if "." in s:
        frac = s.split(".", 1)[1]
        digits = s.replace(".", "").lstrip("0") or "0"
        return f"dec{max(len(digits), len(frac) + 1)},{len(frac)}"
    return "int"


def lex(sql: str) -> Optional[Lexed]:
    out, spans, texts, kinds, last = [], [], [], [], 0
    for m in _TOKEN.finditer(sql):
        g = m.lastgroup
        if g in ("comment", "ident"):
            continue
        s, e = m.span()
        tok = m.group()
        if g == "str":
            texts.append(tok[1:-1].replace("''", "'"))
            kinds.append("str")
            marker = "'?'"
        else:
            texts.append(tok)
            k = _num_kind(tok)
            kinds.append(k)
            marker = "?" + k
        out.append(sql[last:s])
        out.append(marker)
        spans.append((s, e))
        last = e
    if not spans:
        return None
    out.append(sql[last:])
    return Lexed("".join(out), spans, texts, kinds)


def render(sql: str, lx: Lexed, texts: List[str]) -> str:
    """``sql`` with its literal tokens replaced by ``texts``."""
    out, last = [], 0
    for (s, e), k, t in zip(lx.spans, lx.kinds, texts):
        out.append(sql[last:s])
        out.append("'" + t.replace("'", "''") + "'" if k == "str" else t)
        last = e
    out.append(sql[last:])
    return "".join(out)


_SLOT_TYPES = {"int": False, "dec": False, "float": False, "str": True, "date": True, "timestamp": True,
               "interval": True}      # literal node type -> written as a quoted string


def annotate(ast: dict, lx: Lexed) -> Optional[List[dict]]:
    """Number the AST's literal nodes by the lexed token each one came
    from (``node["__slot"]``); returns per token the node's type fields
    (None: a token that is not a literal node -- the template keeps its
    text), or None when a literal node has no token."""
    lits = []
    stack = [ast]
    while stack:
        n = stack.pop()
        if isinstance(n, dict):
            if n.get("k") == "lit" and n.get("type") in _SLOT_TYPES:
                lits.append(n)
            stack.extend(v for v in n.values() if isinstance(v, (dict, list)))
        elif isinstance(n, list):
            stack.extend(n)
    lits.sort(key=lambda n: n.get("pos", -1))
    slots: List[Optional[dict]] = [None] * len(lx.spans)
    j = 0
    for n in lits:
        # the node's token: the next one at or after its position (a typed
        # literal's keyword comes first); tokens before it that no literal
        # node claims (an interval's precision, ``day (3)``) stay fixed text
        while j < len(lx.spans) and lx.spans[j][0] < n.get("pos", -1):
            j += 1
        if j >= len(lx.spans) or not _same(n, lx, j):
            return None
        n["__slot"] = j
        slots[j] = {k: v for k, v in n.items() if k in ("type", "unit")}
        j += 1
    return slots


def _same(n: dict, lx: Lexed, j: int) -> bool:
    quoted = _SLOT_TYPES[n["type"]]
    return (lx.kinds[j] == "str") == quoted and lx.texts[j] == n.get("s")


# -------------------------------------------------------------- recording
class _Rec:
    def __init__(self):
        self.reads: set = set()
        self.raws: List[tuple] = []     # (obj, field name, fn, operand lits)
        self.quiet = 0
        self.eq = 0                     # inside eq_sql(): reads compare values for equality only
        self.mask: Optional[list] = None  # eq_sql's masked rendering: the tracked literals met, in order
        # eq_sql calls: (text with tracked literals masked, those literals, full text)
        self.eq_calls: List[Tuple[str, tuple, str]] = []

    def read(self, lit) -> None:
        if not self.eq:
            self.reads.update(lit.leaves())


_TLS = threading.local()


def _rec() -> Optional[_Rec]:
    r = getattr(_TLS, "rec", None)
    return r if r is not None and not r.quiet else None


class SlotLit(Lit):
    """A literal token of the statement, by position (``slot``): reading
    its value while a template is recorded keys the template on it."""

    def __init__(self, value, dtype, slot: int):
        super().__init__(value, dtype)
        object.__setattr__(self, "slot", slot)

    def __getattribute__(self, name):
        if name == "value":
            r = getattr(_TLS, "rec", None)
            if r is not None and not r.quiet:
                r.read(self)
        return object.__getattribute__(self, name)

    @property
    def nullable(self) -> bool:  # a token is never NULL (NULL is a keyword)
        return False

    def sql(self) -> str:
        r = getattr(_TLS, "rec", None)
        if r is not None and r.mask is not None:
            r.mask.append(self)
            return "\x00?"
        return Lit.sql(self)

    def leaves(self):
        return (self.slot,)


class DerivedLit(Lit):
    """A literal computed from literal operands by ``fn(*args)``."""

    def __init__(self, value, dtype, fn, args):
        super().__init__(value, dtype)
        object.__setattr__(self, "fn", fn)
        object.__setattr__(self, "args", tuple(args))

    def __getattribute__(self, name):
        if name == "value":
            r = getattr(_TLS, "rec", None)
            if r is not None and not r.quiet:
                r.read(self)
        return object.__getattribute__(self, name)

    @property
    def nullable(self) -> bool:   # NULL-ness is re-checked per instantiation
        r = getattr(_TLS, "rec", None)
        if r is not None:
            r.quiet += 1
        try:
            return object.__getattribute__(self, "value") is None
        finally:
            if r is not None:
                r.quiet -= 1

    def sql(self) -> str:
        r = getattr(_TLS, "rec", None)
        if r is not None and r.mask is not None:
            r.mask.append(self)
            return "\x00?"
        return Lit.sql(self)

    def leaves(self):
        out = []
        for a in self.args:
            if isinstance(a, (SlotLit, DerivedLit)):
                out.extend(a.leaves())
        return tuple(out)


_TRACKED = (SlotLit, DerivedLit)


def tracking(*xs) -> bool:
    """True while a template is recorded and one of ``xs`` carries a slot."""
    return _rec() is not None and any(isinstance(x, _TRACKED) for x in xs)


def derive(fn: Callable[..., Any], *args):
    """``fn(*args)`` for literal operands: recorded as a re-runnable
    derivation (its value reads are the derivation's, not the plan's)."""
    r = _rec()
    if r is None or not any(isinstance(a, _TRACKED) for a in args):
        return fn(*args)
    r.quiet += 1
    try:
        out = fn(*args)
    finally:
        r.quiet -= 1
    if isinstance(out, _TRACKED):
        return out                       # an operand passed through
    if type(out) is Lit:
        return DerivedLit(out.value, out.dtype, fn, args)
    # not folded to a literal (a decision that may depend on the values):
    # the template is keyed on the operands
    for a in args:
        if isinstance(a, _TRACKED):
            r.reads.update(a.leaves())
    return out


def eq_sql(e) -> str:
    """``e.sql()`` for a lookup or de-duplication by expression text (equal
    texts share one column, one aggregate, one factored-out predicate): the
    template records which texts that differ only in literals were equal --
    an instance must keep them equal -- instead of keying on the values.
    (Names built from the text keep the recorded statement's literals:
    internal column names, not results.)"""
    r = _rec()
    if r is None:
        return e.sql()
    r.eq += 1
    try:
        real = e.sql()
        if r.mask is None:
            r.mask = []
            try:
                masked = e.sql()
                lits = tuple(r.mask)
            finally:
                r.mask = None
            if lits:
                r.eq_calls.append((masked, lits, real))
        return real
    finally:
        r.eq -= 1


def quiet_sql(e) -> str:
    """``e.sql()`` recording nothing: for decisions whose every outcome is
    correct for any literal values (the caller records what must hold with
    ``eq_sql``)."""
    r = getattr(_TLS, "rec", None)
    if r is None:
        return e.sql()
    r.quiet += 1
    try:
        return e.sql()
    finally:
        r.quiet -= 1


def _partition(keys: list) -> tuple:
    first: Dict[Any, int] = {}
    return tuple(first.setdefault(k, i) for i, k in enumerate(keys))


def peek(x):
    """A literal's value read without keying the template on it (the caller
    records the use with ``raw`` or only tests for NULL, which a token
    never is and a derivation re-checks)."""
    r = getattr(_TLS, "rec", None)
    if r is None or not isinstance(x, _TRACKED):
        return x.value
    r.quiet += 1
    try:
        return x.value
    finally:
        r.quiet -= 1


def raw(obj, name: str, fn: Callable[..., Any], *args) -> None:
    """Plan object ``obj`` holds ``fn(*args)`` in its field ``name``,
    computed from literal operands: recomputed on instantiation."""
    r = _rec()
    if r is not None and any(isinstance(a, _TRACKED) for a in args):
        r.raws.append((obj, name, fn, args))


class recording:
    """Context: literals of annotated AST nodes bind as ``SlotLit`` and value
    reads are collected."""

    def __enter__(self):
        self.prev = getattr(_TLS, "rec", None)
        self.rec = _TLS.rec = _Rec()
        return self.rec

    def __exit__(self, *exc):
        _TLS.rec = self.prev
        return False


def active() -> bool:
    return getattr(_TLS, "rec", None) is not None


# ------------------------------------------------------------- templates
_SCALARS = (type(None), bool, int, float, str, bytes, complex)


def _dirty_map(root, raws_objs) -> Tuple[set, Dict[int, Any]]:
    """ids of the objects under ``root`` that contain a tracked literal or a
    recorded raw field (only they are copied on instantiation)."""
    dirty, keep, seen = set(), {}, {}
    from . import expr as E, logical as L

    def visit(o) -> bool:
        i = id(o)
        if i in seen:
            return seen[i]
        seen[i] = False          # cycles: assume clean while visiting
        keep[i] = o
        if isinstance(o, _TRACKED):
            d = True
        elif isinstance(o, _SCALARS) or isinstance(o, type):
            d = False
        elif isinstance(o, (list, tuple)):
            d = any([visit(x) for x in o])
        elif isinstance(o, dict):
            d = any([visit(v) for v in o.values()])
        elif isinstance(o, (E.Expr, L.Plan, L.ColInfo)) or type(o).__module__.startswith("igloo_amd.sql"):
            d = any([visit(v) for v in vars(o).values()]) if hasattr(o, "__dict__") else False
            d = d or i in raws_objs
        else:
            d = False            # table sources, dtypes, ...: never copied
        seen[i] = d
        if d:
            dirty.add(i)
        return d
    visit(root)
    return dirty, keep


class Template:
    """A recorded statement: its plan with slot literals, how to key it and
    how to instantiate it with new literal texts."""

    def __init__(self, plan, names, lx: Lexed, slot_nodes: List[dict], rec: _Rec):
        self.plan = plan
        self.names = names
        self.kinds = lx.kinds
        self.nodes = slot_nodes              # AST literal node per slot (type, unit)
        self.keyed = {s: lx.texts[s] for s in sorted(set(rec.reads) | {i for i, n in enumerate(slot_nodes) if n is None})}
        self.raws = rec.raws
        raw_ids = {id(o) for o, _, _, _ in rec.raws}
        # texts compared by eq_sql that differ only in literals: which of them
        # were equal (every use shares, de-duplicates or factors equal texts)
        groups: Dict[str, Dict[tuple, str]] = {}
        for masked, lits, real in rec.eq_calls:
            groups.setdefault(masked, {})[tuple(id(o) for o in lits)] = (lits, real)
        self.eq_groups = []
        for recs in groups.values():
            if len(recs) > 1:
                rs = list(recs.values())
                self.eq_groups.append(([l for l, _ in rs], _partition([t for _, t in rs])))
        self.dirty, self._keep = _dirty_map((plan, names), raw_ids)
        self.verified = False

    def matches(self, texts: List[str]) -> bool:
        return all(texts[s] == t for s, t in self.keyed.items())

    def instantiate(self, texts: List[str], literal: Callable[[dict], Lit]):
        """(plan, names) with the literal texts ``texts``, or None when a
        derivation no longer holds (the caller plans afresh)."""
        base: Dict[int, Lit] = {}
        memo: Dict[int, Any] = {}
        raws: Dict[int, list] = {}
        for o, name, fn, args in self.raws:
            raws.setdefault(id(o), []).append((name, fn, args))

        class _Stale(Exception):
            pass

        def lit(x):
            i = id(x)
            if i in memo:
                return memo[i]
            if isinstance(x, SlotLit):
                s = x.slot
                if s not in base:
                    node = dict(self.nodes[s])
                    node["s"] = texts[s]
                    base[s] = literal(node)
                r = base[s]
                if r.dtype != x.dtype:
                    raise _Stale(f"slot {s} type {r.dtype} != {x.dtype}")
            elif isinstance(x, DerivedLit):
                r = x.fn(*[lit(a) if isinstance(a, _TRACKED) else a for a in x.args])
                if not isinstance(r, Lit) or r.dtype != x.dtype or \
                        (r.value is None) != (object.__getattribute__(x, "value") is None):
                    raise _Stale(f"derived {getattr(r, 'dtype', r)} != {x.dtype}")
                r = Lit(r.value, r.dtype) if type(r) is not Lit else r
            else:
                r = x
            memo[i] = r
            return r

        def sub(o):
            i = id(o)
            if i in memo:
                return memo[i]
            if isinstance(o, _TRACKED):
                return lit(o)
            if isinstance(o, list):
                r = [sub(x) if id(x) in self.dirty else x for x in o]
            elif isinstance(o, tuple):
                r = tuple(sub(x) if id(x) in self.dirty else x for x in o)
            elif isinstance(o, dict):
                r = {k: (sub(v) if id(v) in self.dirty else v) for k, v in o.items()}
            else:
                r = copy.copy(o)
                memo[i] = r       # (before the fields: shared sub-objects resolve to this copy)
                for k, v in vars(o).items():
                    if id(v) in self.dirty:
                        object.__setattr__(r, k, sub(v))
                for name, fn, args in raws.get(i, ()):
                    object.__setattr__(r, name, fn(*[lit(a) if isinstance(a, _TRACKED) else a for a in args]))
            memo[i] = r
            return r

        try:
            for lits_list, part in self.eq_groups:
                # texts that were equal (shared, de-duplicated, factored out)
                # must still be; texts that were distinct may coincide now --
                # the plan then computes an equal thing twice
                new = [tuple(lit(o).sql() for o in lits) for lits in lits_list]
                if any(new[i] != new[p] for i, p in enumerate(part)):
                    why(f"equal texts differ now: {new}")
                    return None
            plan, names = sub((self.plan, self.names))
        except _Stale as ex:
            why(f"stale derivation {ex}")
            return None
        except Exception as ex:       # noqa: BLE001 - a re-derivation failed: plan afresh
            why(f"re-derivation failed: {type(ex).__name__}: {ex}")
            return None
        return plan, names


def signature(plan) -> str:
    """The plan serialized (sql/serde.py) without column names: names built
    from expression text by ``eq_sql`` keep the recorded literals."""
    import json
    from . import serde

    def strip(o):
        if isinstance(o, dict):
            drop = o.get("__c") in ("ColInfo", "ColRef")
            return {k: strip(v) for k, v in o.items() if not (drop and k == "name")}
        if isinstance(o, list):
            return [strip(v) for v in o]
        return o
    return json.dumps(strip(serde.to_obj(plan)), separators=(",", ":"))


# -------------------------------------------------------------- perturbing
def perturb(texts: List[str], kinds: List[str], nodes: List[dict]) -> List[str]:
    """Every literal changed, within its token class (same number kind and
    decimal shape, valid dates, same string length and wildcards)."""
    out = []
    for t, k, n in zip(texts, kinds, nodes):
        if n is None:
            out.append(t)
            continue
        typ = n.get("type")
        if typ == "date" or (typ == "str" and re.fullmatch(r"\d{4}-\d{2}-\d{2}", t)):
            # (a date, or a string that spells one: it may be coerced to a date)
            try:
                d = datetime.date.fromisoformat(t.strip()) + datetime.timedelta(days=1)
                out.append(d.isoformat())
                continue
            except ValueError:
                out.append(t)
                continue
        if k == "str":
            j = max((i for i, c in enumerate(t) if c.isalnum()), default=-1)
            if j < 0 or typ in ("timestamp", "interval"):
                if typ == "interval" and t.strip().isdigit():
                    out.append(str(int(t) + 1))
                else:
                    out.append(t)
                continue
            c = t[j]
            # cyclic within the character's class: injective, so literals
            # equal before are equal after and distinct ones stay distinct
            nc = {"9": "0", "z": "a", "Z": "A"}.get(c, chr(ord(c) + 1)) if c.isascii() else c
            out.append(t[:j] + nc + t[j + 1:])
            continue
        if k == "int":
            out.append(str(int(t) + 1))
            continue
        if k.startswith("dec"):
            cand = _bump_decimal(t)
            out.append(cand if cand is not None and _num_kind(cand) == k else t)
            continue
        out.append(repr(float(t) + 1.0))
    return out


def _bump_decimal(t: str) -> Optional[str]:
    whole, frac = t.split(".", 1)
    digits = whole + frac
    for delta in (1, -1):
        v = int(digits or "0") + delta
        if v < 0:
            continue
        s = str(v).zfill(len(digits))
        cand = (s[:len(s) - len(frac)] or "0") + "." + s[len(s) - len(frac):] if frac else s + "."
        if _num_kind(cand) == _num_kind(t):
            return cand
    return None
