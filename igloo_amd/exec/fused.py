"""Planner for the fused scan kernels (csrc/kernels/fused.hip).

Turns a scan predicate into AND-ed range / code-set terms over integer
columns (decimals as scaled int64, dates as days, dictionary codes) and an
aggregate over a scan into a small-domain GROUP BY of sums of products of
affine terms — the shape of TPC-H's scan-heavy queries (Q1, Q6 and the
``price * (1 - discount)`` revenue expression nearly every query sums).

Semantics mirror ``expr_eval.Evaluator`` exactly: comparisons happen in the
common numeric type (bounds are adjusted with exact integer ceil/floor instead
of rescaling the column), products keep the scale sum, decimal products whose
static precision exceeds 18 digits are overflow-checked. A conjunct that does
not fit a term is evaluated node by node into a mask the kernel reads;
aggregates that do not fit return None so the caller keeps its generic path.

Role in the reference: DataFusion's FilterExec -> ProjectionExec ->
AggregateExec chain run by ``QueryEngine::execute`` (reference
crates/engine/src/lib.rs:55-56; operators/filter.rs:47).
"""
from __future__ import annotations

from ..utils import switches as _sw
import os
from typing import Dict, List, Optional, Tuple

import torch

from .. import types as T
from ..columnar import Batch, Column
from ..ops._lib import check_not_capturing, to_host_ints
from ..sql.expr import BinOp, Cast, ColRef, Expr, InList, Lit, conjuncts
from ..types import DataType
from ..utils.errors import ExecutionError

MAX_COLS, MAX_TERMS, MAX_AGGS, MAX_GROUPS, MAX_FACTORS = 8, 16, 8, 16, 3
MAX_OR_GROUPS = 31  # disjuncts of the one OR conjunct a launch can hold
# column-vs-column range terms (l_commitdate < l_receiptdate): with generated
# scan kernels the extra compare is free; SF100 A/B: Q12 6.1 -> 3.7 ms
COL_COL = True
I64_MIN, I64_MAX = -(2**63), 2**63 - 1
FLIP = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "<>": "<>"}


class Bail(Exception):
    pass


def _debug(what, why):
    if _sw.debug("fused"):
        print(f"[fused] {what}: fallback ({why})", flush=True)


def _floordiv(a: int, b: int) -> int:
    return a // b


def _ceildiv(a: int, b: int) -> int:
    return -((-a) // b)


class Spec:
    """Columns + filter terms (+ fallback mask) of one fused launch."""

    def __init__(self, b: Batch, ev):
        self.b = b
        self.ev = ev
        self.cols: List[torch.Tensor] = []
        self._idx: Dict[int, int] = {}
        self.terms: List[tuple] = []
        self.mask: Optional[torch.Tensor] = None
        self.always_false = False
        self._group = 0            # OR-group of the terms being added (0: top-level conjunct)
        self._group_false = False  # the current disjunct can never hold
        self._has_or = False

    def col(self, c: Column) -> int:
        if c.valid is not None or c.is_wide or (c.dtype.is_string and not c.is_dict):
            raise Bail("nullable / wide / plain-string column")
        x = narrow(c.data)
        if x.dtype in (torch.bool, torch.uint8):
            x = x.to(torch.int16)   # the kernels sign-extend 1/2/4/8-byte words
        if x.dtype not in (torch.int8, torch.int16, torch.int32, torch.int64) or x.dim() != 1:
            raise Bail(f"column dtype {x.dtype}")
        if not x.is_contiguous() or (x.element_size() < 4 and x.data_ptr() % 4):
            x = x.clone(memory_format=torch.contiguous_format)   # sub-dword columns start 4-byte aligned (ff_load)
        key = id(c.data)
        if key not in self._idx:
            if len(self.cols) >= MAX_COLS:
                raise Bail("too many columns")
            self._idx[key] = len(self.cols)
            self.cols.append(x)
        return self._idx[key]

    def colref(self, e: ColRef) -> Tuple[int, Column]:
        c = self.b.columns.get(e.cid)
        if c is None:
            raise Bail("column not in batch")
        return self.col(c), c

    # ------------------------------------------------------------- filter
    def add_predicate(self, pred: Expr) -> None:
        for c in conjuncts(pred):
            try:
                if isinstance(c, BinOp) and c.op == "or":
                    self._disjunction(c)
                else:
                    self._term(c)
            except Bail as why:
                _debug("conjunct", why)
                m = self.ev.mask(c, self.b)
                self.mask = m if self.mask is None else (self.mask & m)

    def _false(self) -> None:
        if self._group:
            self._group_false = True
        else:
            self.always_false = True

    def _disjunction(self, c: Expr) -> None:
        """OR of conjunctions (TPC-H Q19's three brand/container/quantity
        branches): every disjunct's terms carry its OR-group id; the kernel
        passes a row when all terms of some group hold. One OR per launch."""
        ds = _disjuncts(c)
        if self._has_or or len(ds) > MAX_OR_GROUPS:
            raise Bail("second OR / too many disjuncts")
        saved = list(self.terms)
        g, always_true = 0, False
        try:
            for d in ds:
                self._group, self._group_false = g + 1, False
                start = len(self.terms)
                for x in conjuncts(d):
                    if isinstance(x, BinOp) and x.op == "or":
                        raise Bail("nested OR")
                    self._term(x)
                if self._group_false:
                    del self.terms[start:]   # this disjunct never holds
                    continue
                if len(self.terms) == start:
                    always_true = True       # this disjunct always holds
                g += 1
        except Bail:
            self.terms = saved
            raise
        finally:
            self._group, self._group_false = 0, False
        if always_true:
            self.terms = saved
        elif g == 0:
            self.terms = saved
            self.always_false = True
        else:
            self._has_or = True

    def _range(self, ci: int, op: str, v: int):
        lo, hi, kind = I64_MIN, I64_MAX, 0
        if op == "=":
            lo = hi = v
        elif op == "<>":
            lo = hi = v
            kind = 1
        elif op == "<":
            if v == I64_MIN:
                self._false()
                return
            hi = v - 1
        elif op == "<=":
            hi = v
        elif op == ">":
            if v == I64_MAX:
                self._false()
                return
            lo = v + 1
        elif op == ">=":
            lo = v
        kind |= self._group << 8
        if kind == self._group << 8:
            # merge with a range on the same column and group (BETWEEN = two terms)
            for i, (c0, k0, lo0, hi0, s0) in enumerate(self.terms):
                if c0 == ci and k0 == kind:
                    lo, hi = max(lo, lo0), min(hi, hi0)
                    if lo > hi:
                        self._false()
                    self.terms[i] = (ci, kind, lo, hi, 0)
                    return
        if len(self.terms) >= MAX_TERMS:
            raise Bail("too many terms")
        self.terms.append((ci, kind, lo, hi, 0))

    def _term(self, c: Expr) -> None:
        if isinstance(c, InList):
            self._inlist(c)
            return
        if not (isinstance(c, BinOp) and c.op in FLIP):
            raise Bail(f"conjunct {type(c).__name__}")
        l, r, op = c.left, c.right, c.op
        if isinstance(l, Lit) and not isinstance(r, Lit):
            l, r, op = r, l, FLIP[op]
        cast_t = None
        # CAST(col AS wider decimal/int) only rescales exactly: compare the raw column
        while isinstance(l, Cast) and (l.dtype.is_decimal or l.dtype.is_integer) and \
                (l.x.dtype.is_decimal or l.x.dtype.is_integer) and \
                (l.dtype.scale if l.dtype.is_decimal else 0) >= (l.x.dtype.scale if l.x.dtype.is_decimal else 0):
            cast_t = cast_t or l.dtype
            l = l.x
        if isinstance(l, ColRef) and isinstance(r, ColRef) and cast_t is None and COL_COL:
            self._col_col(l, r, op)
            return
        if not (isinstance(l, ColRef) and isinstance(r, Lit)) or r.value is None:
            raise Bail("not column-vs-literal")
        ci, col = self.colref(l)
        if col.is_dict:
            if op not in ("=", "<>"):
                raise Bail("string range on a dictionary")
            code = _dict_code(col, str(r.value))
            if code is None:
                if op == "=":
                    self._false()
                return  # '<>' a value not in the dictionary: always true
            self._range(ci, op, code)
            return
        lt, rt = (cast_t or col.dtype), r.dtype
        if lt.is_float or rt.is_float or lt.is_string or rt.is_string:
            raise Bail("float / string comparison")
        if lt.kind in ("date32", "timestamp", "bool") or rt.kind in ("date32", "timestamp", "bool"):
            self._range(ci, op, int(r.value))
            return
        t = lt if lt == rt else T.common_numeric(lt, rt)
        cs = col.dtype.scale if col.dtype.is_decimal else 0
        ls = rt.scale if rt.is_decimal else 0
        ts = t.scale if t.is_decimal else 0
        L = int(r.value) * 10 ** (ts - ls)       # literal in the common scale
        f = 10 ** (ts - cs)                      # column multiplier into the common scale
        if f == 1:
            self._range(ci, op, L)
            return
        # col * f  OP  L   <=>   col OP' bound (exact integer bounds)
        if op == "<":
            self._range(ci, "<", _ceildiv(L, f))
        elif op == "<=":
            self._range(ci, "<=", _floordiv(L, f))
        elif op == ">":
            self._range(ci, ">", _floordiv(L, f))
        elif op == ">=":
            self._range(ci, ">=", _ceildiv(L, f))
        elif op == "=":
            if L % f:
                self._false()
            else:
                self._range(ci, "=", L // f)
        else:  # '<>'
            if L % f == 0:
                self._range(ci, "<>", L // f)

    def _col_col(self, l: ColRef, r: ColRef, op: str) -> None:
        """l OP r on two 4-byte integer-like columns of one type (dates, int32):
        a range term on l - r (kind 3), which cannot overflow in int64."""
        if op == "<>" or l.dtype != r.dtype or l.dtype.kind not in ("date32", "int32", "int16", "int8"):
            raise Bail("column-vs-column comparison")
        if len(self.terms) >= MAX_TERMS:
            raise Bail("too many terms")
        cl, coll = self.colref(l)
        cr, colr = self.colref(r)
        if coll.is_dict or colr.is_dict:
            raise Bail("dictionary column comparison")
        lo, hi = {"<": (I64_MIN, -1), "<=": (I64_MIN, 0), ">": (1, I64_MAX), ">=": (0, I64_MAX),
                  "=": (0, 0)}[op]
        self.terms.append((cl, 3 | self._group << 8, lo, hi, cr))

    def _inlist(self, c: InList) -> None:
        if not isinstance(c.x, ColRef) or any(v.value is None for v in c.values):
            raise Bail("IN over an expression / NULL")
        ci, col = self.colref(c.x)
        if not col.is_dict or len(col.dictionary) > 64:
            raise Bail("IN on a non-dictionary column")
        bits = 0
        for v in c.values:
            code = _dict_code(col, str(v.value))
            if code is not None:
                bits |= 1 << code
        if len(self.terms) >= MAX_TERMS:
            raise Bail("too many terms")
        if c.negated:
            bits = ~bits & ((1 << 64) - 1)
        if bits == 0:
            self._false()
            return
        self.terms.append((ci, 2 | self._group << 8, 0, 0, bits))

    def args(self):
        return ([(t.data_ptr(), t.element_size()) for t in self.cols], self.terms,
                self.mask.data_ptr() if self.mask is not None else 0)


NARROW = True
NARROW_MIN_ROWS = 1 << 20
_NARROW_TYPES = (torch.int8, torch.int16, torch.int32)


def narrow(x: torch.Tensor) -> torch.Tensor:
    """Narrowest signed integer copy of a RESIDENT int32/int64 column that
    holds all its values (``_igloo_resident`` is set by MemoryTable), made on
    first use and kept on the tensor: the fused scans then stream 1-4 bytes a
    row instead of 8 (TPC-H Q1 reads l_quantity as int16, l_discount / l_tax
    as int8, l_extendedprice as int32). Other tensors are returned as is."""
    if not NARROW or x.dtype not in (torch.int32, torch.int64) or x.numel() < NARROW_MIN_ROWS \
            or not getattr(x, "_igloo_resident", False):
        return x
    hit = getattr(x, "_igloo_narrow", None)
    if hit is None:
        check_not_capturing("narrow copy of a resident column")
        mn, mx = (int(v) for v in torch.aminmax(x))
        hit = x
        for t in _NARROW_TYPES:
            if t.itemsize >= x.element_size():
                break
            if torch.iinfo(t).min <= mn and mx <= torch.iinfo(t).max:
                hit = x.to(t)
                break
        try:
            x._igloo_narrow = hit
        except (AttributeError, RuntimeError):
            return x
    return hit


def _disjuncts(e: Expr) -> List[Expr]:
    if isinstance(e, BinOp) and e.op == "or":
        return _disjuncts(e.left) + _disjuncts(e.right)
    return [e]


def _dict_code(col: Column, s: str) -> Optional[int]:
    dc = col.dictionary.derived()
    cache = dc.get("code_of")
    if cache is None:
        cache = dc["code_of"] = {v: i for i, v in enumerate(col.dict_values())}
    return cache.get(s)


# ------------------------------------------------------------------ masks
def predicate_mask(pred: Expr, b: Batch, ev) -> Optional[torch.Tensor]:
    """Scan predicate -> bool mask with one fused kernel, or None (no term applies)."""
    from ..ops._lib import launch, stream
    if b.num_rows == 0:
        return None
    spec = Spec(b, ev)
    spec.add_predicate(pred)
    n = b.num_rows
    dev = ev.device(b)
    if spec.always_false:
        return torch.zeros(n, dtype=torch.bool, device=dev)
    if not spec.terms:
        return spec.mask  # every conjunct needed the generic evaluator
    out = torch.empty(n, dtype=torch.bool, device=dev)
    from . import fused_jit as FJ
    from ..ops.select import attach_tile_counts, fused_counts_ok
    tc = torch.empty(-(-n // FJ.SELECT_TILE) + 1, dtype=torch.int64, device=dev) \
        if FJ.TILE_COUNTS and fused_counts_ok(n) else None
    if FJ.jit_mask(spec, n, out, stream(out), tc):
        if tc is not None:
            attach_tile_counts(out, tc)
        return out
    cols, terms, mask = spec.args()
    launch("ff_mask").ff_mask(cols, terms, mask, n, out.data_ptr(), stream(out))
    return out


# -------------------------------------------------------------- aggregates
def _factors(e: Expr, spec: Spec) -> Tuple[List[tuple], int, bool]:
    """e == prod(a + b * col) -> (factors, scale, checked) in the Evaluator's
    representation of e.dtype; raises Bail otherwise."""
    t = e.dtype
    if isinstance(e, ColRef):
        ci, col = spec.colref(e)
        if col.is_dict or col.dtype.is_float:
            raise Bail("dictionary / float argument")
        return [(ci, 0, 1)], (col.dtype.scale if col.dtype.is_decimal else 0), False
    if isinstance(e, Lit):
        if e.value is None or t.is_float or t.is_string:
            raise Bail("literal argument")
        return [(-1, int(e.value), 0)], (t.scale if t.is_decimal else 0), False
    if isinstance(e, Cast) and t.is_decimal and (e.x.dtype.is_decimal or e.x.dtype.is_integer):
        fs, s, chk = _factors(e.x, spec)
        d = t.scale - s
        if d < 0 or len(fs) != 1:
            raise Bail("down-scaling cast")
        ci, a, b_ = fs[0]
        return [(ci, a * 10**d, b_ * 10**d)], t.scale, chk
    if isinstance(e, BinOp) and e.op == "*" and (t.is_decimal or t.is_integer):
        fl, sl, cl = _factors(e.left, spec)
        fr, sr, cr = _factors(e.right, spec)
        fs = fl + fr
        consts = [f for f in fs if f[0] < 0]
        var = [f for f in fs if f[0] >= 0]
        k = 1
        for f in consts:
            k *= f[1]
        fs = var + ([(-1, k, 0)] if k != 1 or not var else [])
        if len(fs) > MAX_FACTORS:
            raise Bail("too many factors")
        return fs, sl + sr, cl or cr or (t.is_decimal and t.precision > 18)
    if isinstance(e, BinOp) and e.op in ("+", "-") and (t.is_decimal or t.is_integer):
        l, r = e.left, e.right
        sign = 1 if e.op == "+" else -1
        if isinstance(l, Lit) and not isinstance(r, Lit):
            lit, x, lit_first = l, r, True
        elif isinstance(r, Lit):
            lit, x, lit_first = r, l, False
        else:
            raise Bail("sum of two columns")
        if lit.value is None:
            raise Bail("NULL literal")
        fx, sx, chk = _factors(x, spec)
        if len(fx) != 1 or fx[0][0] < 0:
            raise Bail("affine over a product")
        ts = t.scale if t.is_decimal else 0
        ls = lit.dtype.scale if lit.dtype.is_decimal else 0
        if ts < sx or ts < ls:
            raise Bail("down-scaling add")
        L = int(lit.value) * 10 ** (ts - ls)
        ci, a, b_ = fx[0]
        m = 10 ** (ts - sx)
        if lit_first:   # L +/- (a + b col)
            return [(ci, L + sign * a * m, sign * b_ * m)], ts, chk
        return [(ci, a * m + sign * L, b_ * m)], ts, chk  # (a + b col) +/- L
    raise Bail(f"argument {type(e).__name__}")


def _value_bits(fs, spec) -> int:
    """Bound on the two's-complement width of prod(a + b * col) from the
    (narrow) widths of the factor columns; the one-hot MFMA aggregation sizes
    its 7-bit limb decomposition with it (0 = unknown / 64 bits)."""
    widths = [w for _, w in spec.args()[0]]
    bound = 1
    for c, a, b in fs:
        c = int(c)
        if c < 0:
            f = abs(int(a))
        else:
            w = widths[c] if c < len(widths) else 8
            f = abs(int(a)) + abs(int(b)) * (1 << (8 * int(w) - 1))
        bound *= max(f, 1)
        if bound >= 1 << 63:
            return 0
    return bound.bit_length() + 1


def fused_scan_aggregate(groups, aggs, b: Batch, pred: Optional[Expr], ctx) -> Optional[Batch]:
    """GROUP BY (domain <= 16) over a scanned batch with the scan filter and the
    argument arithmetic fused into one kernel, or None if the shape does not fit."""
    from ..ops._lib import launch, stream
    from .aggregate import _avg
    dev = ctx.device
    if dev.type != "cuda" or b.num_rows == 0:
        return None
    n = b.num_rows
    try:
        spec = Spec(b, ctx.evaluator)
        keys, kinfo, G = [], [], 1
        for ci, e in groups:
            if not isinstance(e, ColRef):
                raise Bail("computed group key")
            k, col = spec.colref(e)
            if col.is_dict:
                lo, size = 0, len(col.dictionary)
            elif col.dtype.is_integer or col.dtype.kind in ("date32", "bool"):
                from ..ops.hashing import key_range
                rng = key_range(col.data) if col.data.dtype in (torch.int32, torch.int64) else None
                if rng is None:   # other widths / empty: one reduction
                    mn, mx = torch.aminmax(col.data)
                    rng = to_host_ints(torch.stack([mn.to(torch.int64), mx.to(torch.int64)]))
                lo, hi = rng
                size = hi - lo + 1
            else:
                raise Bail("group key type")
            kinfo.append((ci, col, k, lo, max(size, 1)))
            G *= max(size, 1)
            if G > MAX_GROUPS or len(kinfo) > 2:
                raise Bail("group domain")
        mul = 1
        for ci, col, k, lo, size in reversed(kinfo):
            keys.append((k, lo, mul))
            mul *= size
        plan = []
        descs = []
        for ci, a in aggs:
            if a.distinct or a.filter is not None or a.func not in ("sum", "count", "avg", "min", "max"):
                raise Bail(f"aggregate {a.func}")
            if a.func == "count":
                if a.arg is not None:
                    c = ctx.evaluator.eval(a.arg, b) if not isinstance(a.arg, ColRef) else b.columns.get(a.arg.cid)
                    if c is None or getattr(c, "valid", None) is not None:
                        raise Bail("count over a nullable argument")
                plan.append((ci, a, None))
                continue
            if a.arg.dtype.is_float or a.arg.dtype.is_string:
                raise Bail("float / string argument")
            fs, scale, chk = _factors(a.arg, spec)
            want = a.arg.dtype.scale if a.arg.dtype.is_decimal else 0
            if scale != want:
                raise Bail(f"scale {scale} != {want}")
            op = {"sum": 0, "avg": 0, "min": 2, "max": 3}[a.func]
            d = (op, int(chk), tuple(fs))
            if d not in descs:   # avg(x) next to sum(x): one accumulator
                descs.append(d)
            plan.append((ci, a, d))
        # lexicographic factor order puts a product right after its prefix, so
        # the kernel extends the previous value instead of recomputing it
        descs.sort(key=lambda d: (d[2], d[0], d[1]))
        pos = {d: i for i, d in enumerate(descs)}
        plan = [(ci, a, None if d is None else pos[d]) for ci, a, d in plan]
        if len(descs) > MAX_AGGS:
            raise Bail("too many aggregates")
        if pred is not None:
            spec.add_predicate(pred)
    except Bail as why:
        _debug("aggregate", why)
        return None
    counts = torch.zeros(G, dtype=torch.int64, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    bufs, kaggs = [], []
    prev = None
    for op, chk, fs in descs:
        if op == 0:
            d, d2 = torch.zeros(G, dtype=torch.int64, device=dev), torch.zeros(G, dtype=torch.int64, device=dev)
        else:
            d = torch.full((G,), I64_MAX if op == 2 else I64_MIN, dtype=torch.int64, device=dev)
            d2 = None
        bufs.append((d, d2))
        # reuse the previous product when it is a prefix of this one (an
        # unchecked predecessor may have wrapped, so a checked one needs a checked prefix)
        shared = 0
        if prev is not None and prev[2] and len(prev[2]) < len(fs) and fs[:len(prev[2])] == prev[2] \
                and (prev[1] or not chk):
            shared = len(prev[2])
        prev = (op, chk, fs)
        kaggs.append((op, chk, [(int(c), int(a_), int(b_)) for c, a_, b_ in fs], d.data_ptr(),
                      d2.data_ptr() if d2 is not None else 0, shared, _value_bits(fs, spec)))
    if not spec.always_false:
        from .fused_jit import jit_aggregate
        cols, terms, mask = spec.args()
        with ctx.span("agg.fused_scan"):
            if not jit_aggregate(spec, keys, G, kaggs, counts, ovf, n, stream(counts)):
                launch("ff_aggregate").ff_aggregate(cols, terms, mask, keys, G, kaggs, counts.data_ptr(),
                                                    ovf.data_ptr(), n, stream(counts))
    # ONE readback for the overflow flag, whether each 128-bit sum fits in 64
    # bits and the number of non-empty groups (Q1: 7 readbacks -> 1)
    from ..ops.agg import _wide_flags
    checked = any(chk for _, chk, _ in descs)
    wide = [(d, d2) for d, d2 in bufs if d2 is not None]
    parts = []
    if checked:
        parts.append(ovf.reshape(-1)[:1].to(torch.int64))
    if wide:
        parts.append(_wide_flags(wide).to(torch.int64))
    if groups:
        parts.append((counts > 0).sum().reshape(1))
    vals = to_host_ints(torch.cat(parts)) if parts else []
    pos = 0
    if checked:
        if vals[0]:
            raise ExecutionError("decimal multiplication overflows 64-bit fixed point; CAST to DOUBLE")
        pos = 1
    flags = iter(vals[pos:pos + len(wide)])
    pos += len(wide)
    res = [d if d2 is None else (d if not next(flags) else torch.stack([d, d2], dim=1)) for d, d2 in bufs]
    if groups:
        from ..ops.select import mask_to_indices
        ng = vals[pos]
        keep = mask_to_indices(counts > 0, total=ng)
    else:
        keep, ng = None, 1

    def sel(x):
        return x if keep is None else x.index_select(0, keep)
    out: Dict[int, Column] = {}
    if groups:
        stride = 1
        for ci, col, k, lo, size in reversed(kinfo):
            code = (keep // stride) % size + lo
            stride *= size
            if col.is_dict:
                out[ci.cid] = Column(col.dtype, code.to(torch.int32), None, dictionary=col.dictionary)
            else:
                out[ci.cid] = Column(col.dtype, code.to(col.data.dtype), None)
    cnt = sel(counts)
    for ci, a, i in plan:
        t = a.dtype
        if a.func == "count":
            out[ci.cid] = Column(T.INT64, cnt)
            continue
        v = sel(res[i])
        nonempty = cnt > 0
        valid = None if groups else nonempty
        if a.func == "avg":
            out[ci.cid] = Column(t, _avg(v, cnt, a.arg.dtype, t), nonempty)
        elif a.func == "sum":
            out[ci.cid] = Column(t, v, valid)
        else:
            out[ci.cid] = Column(t, v.to(t.torch_dtype), valid)
    return Batch(out, ng)
