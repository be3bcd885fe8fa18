"""Regular expressions compiled to a byte DFA for the GPU (csrc/kernels/regex.hip).

Parity: DataFusion's regexp_like / ``~`` / ``~*`` / ``!~`` / ``SIMILAR TO``
(reference Cargo.lock:1062-1090: datafusion-functions with the Rust
``regex`` crate), reached through ``SessionContext::sql`` (reference
crates/engine/src/lib.rs:54-57).

A match test needs no capture positions, so the pattern becomes a
deterministic automaton over byte classes: parse -> Thompson NFA (byte-set
edges) -> subset construction with the search loop built in (the start
state is re-entered at every byte unless the pattern starts with ``^``).
The kernel keeps the transition table in LDS and walks one string per lane,
leaving early once an accepting (or dead) state is reached.

Supported: literals (UTF-8), ``.`` (one UTF-8 character, not ``\\n``),
classes ``[...]`` / ``[^...]`` with ranges and ``\\d \\w \\s`` (ASCII members;
a negated class also matches any non-ASCII character), the escapes
``\\d \\D \\w \\W \\s \\S`` and escaped punctuation, groups ``(..)`` /
``(?:..)``, ``|``, ``* + ?`` (lazy forms too) and ``{m}`` / ``{m,}`` /
``{m,n}``, ``^`` at the start and ``$`` at the end, and the ``i`` flag
(ASCII case folding). Anything else (back-references, look-around, word
boundaries, anchors elsewhere, non-ASCII class members, automata past the
LDS budget) raises ``Unsupported`` and the caller uses the host engine.
"""
from __future__ import annotations

from typing import Dict, FrozenSet, List, Optional, Tuple

#: LDS budget of the transition table (uint16 entries)
MAX_TABLE_ENTRIES = 16384
MAX_STATES = 4096


class Unsupported(Exception):
    pass


ALL = frozenset(range(256))
DIGIT = frozenset(range(48, 58))
WORD = frozenset(list(range(48, 58)) + list(range(65, 91)) + list(range(97, 123)) + [95])
SPACE = frozenset([9, 10, 11, 12, 13, 32])
CONT = frozenset(range(0x80, 0xC0))


# ------------------------------------------------------------------ parser
def _utf8_any(exclude_ascii: FrozenSet[int]) -> tuple:
    """One UTF-8 character: an ASCII byte not in ``exclude_ascii`` or a
    well-formed 2/3/4-byte sequence."""
    ascii_ok = frozenset(b for b in range(128) if b not in exclude_ascii)
    return ("alt", [("set", ascii_ok),
                    ("seq", [("set", frozenset(range(0xC2, 0xE0))), ("set", CONT)]),
                    ("seq", [("set", frozenset(range(0xE0, 0xF0))), ("set", CONT), ("set", CONT)]),
                    ("seq", [("set", frozenset(range(0xF0, 0xF5))), ("set", CONT), ("set", CONT), ("set", CONT)])])


class _Parser:
    def __init__(self, pat: str, icase: bool):
        self.p = pat
        self.i = 0
        self.icase = icase

    def peek(self) -> Optional[str]:
        return self.p[self.i] if self.i < len(self.p) else None

    def take(self) -> str:
        c = self.p[self.i]
        self.i += 1
        return c

    def fold(self, s: FrozenSet[int]) -> FrozenSet[int]:
        if not self.icase:
            return s
        out = set(s)
        for b in s:
            if 65 <= b <= 90:
                out.add(b + 32)
            elif 97 <= b <= 122:
                out.add(b - 32)
        return frozenset(out)

    def literal(self, ch: str) -> tuple:
        bs = ch.encode("utf-8")
        if len(bs) == 1:
            return ("set", self.fold(frozenset(bs)))
        return ("seq", [("set", frozenset([b])) for b in bs])

    def parse(self):
        node = self.alt()
        if self.i != len(self.p):
            raise Unsupported(f"unexpected '{self.p[self.i]}' at {self.i}")
        return node

    def alt(self):
        items = [self.concat()]
        while self.peek() == "|":
            self.take()
            items.append(self.concat())
        return items[0] if len(items) == 1 else ("alt", items)

    def concat(self):
        items = []
        while self.peek() is not None and self.peek() not in "|)":
            items.append(self.repeat())
        if not items:
            return ("empty",)
        return items[0] if len(items) == 1 else ("seq", items)

    def repeat(self):
        atom = self.atom()
        while True:
            c = self.peek()
            if c in ("*", "+", "?"):
                self.take()
                atom = {"*": ("star", atom), "+": ("plus", atom), "?": ("opt", atom)}[c]
            elif c == "{" and self._counted():
                lo, hi = self._counts()
                atom = _expand_count(atom, lo, hi)
            else:
                break
            if self.peek() == "?":      # lazy: same language
                self.take()
        return atom

    def _counted(self) -> bool:
        j = self.p.find("}", self.i)
        if j < 0:
            return False
        body = self.p[self.i + 1:j]
        parts = body.split(",")
        return 1 <= len(parts) <= 2 and parts[0].isdigit() and (len(parts) == 1 or parts[1] == "" or parts[1].isdigit())

    def _counts(self) -> Tuple[int, Optional[int]]:
        j = self.p.find("}", self.i)
        body = self.p[self.i + 1:j]
        self.i = j + 1
        parts = body.split(",")
        lo = int(parts[0])
        hi = lo if len(parts) == 1 else (None if parts[1] == "" else int(parts[1]))
        if (hi is not None and hi < lo) or lo > 64 or (hi or 0) > 64:
            raise Unsupported("repetition count")
        return lo, hi

    def atom(self):
        c = self.take()
        if c == "(":
            if self.p.startswith("?:", self.i):
                self.i += 2
            elif self.peek() == "?":
                raise Unsupported("group flags / look-around")
            node = self.alt()
            if self.peek() != ")":
                raise Unsupported("unbalanced parenthesis")
            self.take()
            return node
        if c == "[":
            return self.cls()
        if c == ".":
            return _utf8_any(frozenset([10]))
        if c == "\\":
            return self.escape(in_class=False)
        if c in "^$":
            raise Unsupported("anchor inside the pattern")
        if c in "*+?{":
            if c == "{":
                return self.literal(c)
            raise Unsupported("quantifier without an operand")
        return self.literal(c)

    def escape(self, in_class: bool):
        if self.peek() is None:
            raise Unsupported("trailing backslash")
        e = self.take()
        sets = {"d": DIGIT, "w": WORD, "s": SPACE}
        if e in sets:
            return ("set", sets[e])
        if e in "DWS":
            base = sets[e.lower()]
            if in_class:
                return ("set", frozenset(b for b in range(128) if b not in base), "neg")
            return _utf8_any(base)
        ctl = {"n": 10, "t": 9, "r": 13, "f": 12, "v": 11, "0": 0}
        if e in ctl:
            return ("set", frozenset([ctl[e]]))
        if e.isalnum():
            raise Unsupported(f"escape \\{e}")
        return self.literal(e)

    def cls(self):
        neg = False
        if self.peek() == "^":
            self.take()
            neg = True
        members = set()
        first = True
        while True:
            c = self.peek()
            if c is None:
                raise Unsupported("unterminated class")
            if c == "]" and not first:
                self.take()
                break
            first = False
            self.take()
            if c == "[" and self.peek() == ":":
                raise Unsupported("POSIX class")
            if c == "\\":
                r = self.escape(in_class=True)
                if len(r) == 3:      # \D \W \S inside a class
                    if neg:
                        raise Unsupported("negated class with a negated escape")
                    members |= r[1]
                    members |= {-1}      # marker: non-ASCII characters too
                    continue
                if r[0] != "set":
                    raise Unsupported("multi-byte class member")
                lo_set = r[1]
                if len(lo_set) == 1 and self.peek() == "-" and self.p[self.i + 1:self.i + 2] not in ("]", ""):
                    lo = next(iter(lo_set))
                    self.take()
                    hi = self._class_char()
                    members |= set(range(lo, hi + 1))
                else:
                    members |= lo_set
                continue
            b = c.encode("utf-8")
            if len(b) != 1:
                raise Unsupported("non-ASCII class member")
            lo = b[0]
            if self.peek() == "-" and self.p[self.i + 1:self.i + 2] not in ("]", ""):
                self.take()
                hi = self._class_char()
                if hi < lo:
                    raise Unsupported("class range")
                members |= set(range(lo, hi + 1))
            else:
                members.add(lo)
        nonascii = -1 in members
        members.discard(-1)
        ascii_members = self.fold(frozenset(members))
        if neg:
            return _utf8_any(ascii_members)
        if nonascii:
            return ("alt", [("set", ascii_members), _utf8_any(ALL)])
        return ("set", ascii_members)

    def _class_char(self) -> int:
        c = self.take()
        if c == "\\":
            r = self.escape(in_class=True)
            if r[0] != "set" or len(r[1]) != 1:
                raise Unsupported("class range end")
            return next(iter(r[1]))
        b = c.encode("utf-8")
        if len(b) != 1:
            raise Unsupported("non-ASCII class member")
        return b[0]


def _expand_count(atom, lo: int, hi: Optional[int]):
    parts = [atom] * lo
    if hi is None:
        parts.append(("star", atom))
    else:
        parts += [("opt", atom)] * (hi - lo)
    if not parts:
        return ("empty",)
    return parts[0] if len(parts) == 1 else ("seq", parts)


# ------------------------------------------------------------------ NFA
class _NFA:
    def __init__(self):
        self.eps: List[List[int]] = []
        self.edges: List[List[Tuple[FrozenSet[int], int]]] = []

    def new(self) -> int:
        self.eps.append([])
        self.edges.append([])
        if len(self.eps) > 20000:
            raise Unsupported("pattern too large")
        return len(self.eps) - 1

    def build(self, node) -> Tuple[int, int]:
        k = node[0]
        if k == "set":
            a, b = self.new(), self.new()
            self.edges[a].append((node[1], b))
            return a, b
        if k == "empty":
            a = self.new()
            return a, a
        if k == "seq":
            start, end = self.build(node[1][0])
            for x in node[1][1:]:
                s2, e2 = self.build(x)
                self.eps[end].append(s2)
                end = e2
            return start, end
        if k == "alt":
            a, b = self.new(), self.new()
            for x in node[1]:
                s, e = self.build(x)
                self.eps[a].append(s)
                self.eps[e].append(b)
            return a, b
        if k in ("star", "plus", "opt"):
            s, e = self.build(node[1])
            a, b = self.new(), self.new()
            self.eps[a].append(s)
            self.eps[e].append(b)
            if k in ("star", "opt"):
                self.eps[a].append(b)
            if k in ("star", "plus"):
                self.eps[e].append(s)
            return a, b
        raise Unsupported(f"node {k}")


def _closure(nfa: _NFA, states) -> FrozenSet[int]:
    out = set(states)
    stack = list(states)
    while stack:
        s = stack.pop()
        for t in nfa.eps[s]:
            if t not in out:
                out.add(t)
                stack.append(t)
    return frozenset(out)


class DFA:
    """Transition table [states x classes] (uint16), byte -> class map,
    per-state flags (1 accepting, 2 dead), start state, end anchoring."""

    def __init__(self, table: List[List[int]], cls: List[int], accept: List[int], start: int, anchored_end: bool):
        self.table, self.cls, self.accept, self.start, self.anchored_end = table, cls, accept, start, anchored_end

    @property
    def nstates(self) -> int:
        return len(self.table)

    @property
    def nclasses(self) -> int:
        return max(self.cls) + 1

    def match(self, data: bytes) -> bool:
        """Host walk of the same automaton (tests / CPU engine)."""
        s = self.start
        for b in data:
            if not self.anchored_end and self.accept[s] == 1:
                return True
            if self.accept[s] == 2:
                return False
            s = self.table[s][self.cls[b]]
        return self.accept[s] == 1


_CACHE: Dict[Tuple[str, bool], DFA] = {}


def compile_dfa(pattern: str, icase: bool = False) -> DFA:
    key = (pattern, icase)
    hit = _CACHE.get(key)
    if hit is not None:
        return hit
    pat = pattern
    anchored_start = pat.startswith("^")
    if anchored_start:
        pat = pat[1:]
    anchored_end = pat.endswith("$") and not pat.endswith("\\$")
    if anchored_end:
        pat = pat[:-1]
    node = _Parser(pat, icase).parse()
    nfa = _NFA()
    s0, final = nfa.build(node)
    # byte classes: bytes no byte-set edge distinguishes share a class
    sig: Dict[int, list] = {b: [] for b in range(256)}
    for i, edges in enumerate(nfa.edges):
        for j, (bs, _) in enumerate(edges):
            for b in bs:
                sig[b].append((i, j))
    classes: Dict[tuple, int] = {}
    cls = []
    for b in range(256):
        t = tuple(sig[b])
        if t not in classes:
            classes[t] = len(classes)
        cls.append(classes[t])
    ncls = len(classes)
    rep = {}
    for b in range(256):
        rep.setdefault(cls[b], b)
    start_cl = _closure(nfa, [s0])
    states: Dict[FrozenSet[int], int] = {start_cl: 0}
    order = [start_cl]
    table: List[List[int]] = []
    i = 0
    while i < len(order):
        cur = order[i]
        row = []
        for c in range(ncls):
            b = rep[c]
            nxt = set()
            for s in cur:
                for bs, t in nfa.edges[s]:
                    if b in bs:
                        nxt.add(t)
            if not anchored_start:
                nxt.add(s0)          # search: a match may start at every byte
            ncl = _closure(nfa, nxt) if nxt else frozenset()
            if ncl not in states:
                states[ncl] = len(order)
                order.append(ncl)
                if len(order) > MAX_STATES or len(order) * ncls > MAX_TABLE_ENTRIES:
                    raise Unsupported("automaton too large for LDS")
            row.append(states[ncl])
        table.append(row)
        i += 1
    accept = [1 if final in st else 0 for st in order]
    # dead states: no accepting state reachable (early exit with "no match")
    live = {k for k, a in enumerate(accept) if a}
    changed = True
    while changed:
        changed = False
        for k, row in enumerate(table):
            if k not in live and any(t in live for t in row):
                live.add(k)
                changed = True
    for k in range(len(order)):
        if k not in live:
            accept[k] = 2
    if not anchored_end:
        # accepting states are absorbing for a search: the kernel exits there
        pass
    d = DFA(table, cls, accept, 0, anchored_end)
    _CACHE[key] = d
    return d
