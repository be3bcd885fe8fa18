"""Generated expression kernels: a whole scalar expression tree in one HIP
kernel (compiled with hiprtc, ops/jit.py).

The node-by-node evaluator (``expr_eval.Evaluator``) runs one ATen
elementwise kernel per operator and materialises every intermediate column
(plus validity masks) in HBM. For a GPU batch this module instead emits one
kernel that reads the input columns once, evaluates the tree in registers -
arithmetic on fixed-point decimals / ints / floats / dates, comparisons,
three-valued AND / OR / NOT, CASE, CAST, IN lists, COALESCE, abs / round /
date parts / add_months / float math - and writes the result and its validity.

Semantics mirror the evaluator exactly (same conversions: decimal rescaling
rounds half away from zero, float -> decimal uses round-half-even, integer
division truncates and divides-by-zero to NULL, decimal products above 18
digits are overflow-checked - per row here). A subtree the generator does not
cover (strings, LIKE, subqueries over columns, ...) is evaluated by the
evaluator and enters the kernel as an input column, so numeric glue around
string predicates is still fused.

Reference: DataFusion ``PhysicalExpr::evaluate`` called by the reference's
ProjectionExec / FilterExec (reference crates/engine/src/operators/
projection.rs:60-64, filter.rs:47-57).
"""
from __future__ import annotations

from ..utils import switches as _sw
import os
from typing import Dict, List, Optional, Tuple

import torch

from .. import types as T
from ..columnar import Batch, Column
from ..ops import jit
from ..sql.expr import BinOp, Case, Cast, ColRef, Expr, Func, InList, IsNull, Lit, Neg, Not, SubqueryExpr
from ..types import DataType
from ..utils.errors import ExecutionError

ENABLED = os.environ.get("IGLOO_JIT", "async").lower() != "off"
_DEBUG = _sw.debug("jit")
BLOCK = 256
PENDING = object()   # compile submitted, not ready: evaluate node by node this time

_CTYPE = {"bool": "bool", "int8": "i32", "int16": "i32", "int32": "i32", "int64": "i64", "float32": "float",
          "float64": "double", "date32": "i32", "timestamp": "i64", "decimal": "i64"}
_STORE = {"bool": "u8", "int8": "i8", "int16": "i16", "int32": "i32", "int64": "i64", "float32": "float",
          "float64": "double", "date32": "i32", "timestamp": "i64", "decimal": "i64"}
_UNS = {"i32": "u32", "i64": "u64"}

PRELUDE = r"""
typedef signed char i8; typedef short i16; typedef int i32; typedef long long i64;
typedef unsigned char u8; typedef unsigned int u32; typedef unsigned long long u64;
__device__ __forceinline__ double i2d(i64 x) { union { i64 i; double d; } u; u.i = x; return u.d; }
__device__ __forceinline__ void civil(i32 z0, i32* y, i32* m, i32* d) {
  i64 z = (i64)z0 + 719468;
  i64 era = (z >= 0 ? z : z - 146096) / 146097;
  i64 doe = z - era * 146097;
  i64 yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  i64 doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  i64 mp = (5 * doy + 2) / 153;
  i64 mm = mp < 10 ? mp + 3 : mp - 9;
  *y = (i32)(yoe + era * 400 + (mm <= 2));
  *m = (i32)mm;
  *d = (i32)(doy - (153 * mp + 2) / 5 + 1);
}
__device__ __forceinline__ i64 days_from_civil(i64 y, i32 m, i32 d) {
  y -= m <= 2;
  i64 era = (y >= 0 ? y : y - 399) / 400;
  i64 yoe = y - era * 400;
  i64 doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  i64 doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
__device__ __forceinline__ i32 date_part(i32 z, int f) {
  i32 y, m, d;
  civil(z, &y, &m, &d);
  switch (f) {
    case 0: return y;
    case 1: return m;
    case 2: return d;
    case 3: return (m - 1) / 3 + 1;
    case 4: return (i32)(((i64)z % 7 + 7 + 4) % 7);
    default: return (i32)((i64)z - days_from_civil(y, 1, 1) + 1);
  }
}
__device__ __forceinline__ i32 add_months(i32 z, i64 months, i64 days) {
  i32 y, m, d;
  civil(z, &y, &m, &d);
  i64 mi = (i64)y * 12 + (m - 1) + months;          // month index of the target month
  i64 ny = mi >= 0 ? mi / 12 : -((-mi + 11) / 12);
  i32 nm = (i32)(mi - ny * 12) + 1;
  i64 start = days_from_civil(ny, nm, 1);
  i64 ni = mi + 1;
  i64 ny2 = ni >= 0 ? ni / 12 : -((-ni + 11) / 12);
  i64 next = days_from_civil(ny2, (i32)(ni - ny2 * 12) + 1, 1);
  i64 r = start + (d - 1);
  if (r > next - 1) r = next - 1;
  return (i32)(r + days);
}
"""


class Bail(Exception):
    pass


def _ct(t: DataType) -> str:
    c = _CTYPE.get(t.kind)
    if c is None:
        raise Bail(f"type {t.kind}")
    return c


def _flit(x: float) -> str:
    import math
    if not math.isfinite(x):
        raise Bail("non-finite literal")
    return f"{float(x).hex()}"


def _lit(x, t: DataType) -> str:
    c = _ct(t)
    if c == "bool":
        return "true" if x else "false"
    if c in ("double", "float"):
        return f"(({c}){_flit(float(x))})"
    x = int(x)
    if c == "i32":
        if not -(2**31) <= x < 2**31:
            x = (x + 2**31) % 2**32 - 2**31
        return f"((i32){x})" if x != -(2**31) else "((i32)(-2147483647 - 1))"
    if not -(2**63) <= x < 2**63:
        raise Bail("literal beyond int64")
    return f"((i64){x}LL)" if x != -(2**63) else "((i64)(-9223372036854775807LL - 1))"


class _Gen:
    """Emits straight-line C for one row; inputs are columns read at row i."""

    def __init__(self, b: Batch, ev):
        self.b, self.ev = b, ev
        self.inputs: List[Column] = []
        self.in_key: List[tuple] = []
        self._idx: Dict[int, int] = {}
        self.lines: List[str] = []
        self.n = 0
        self.guard = False
        # literal / scalar-subquery values travel as 64-bit kernel arguments
        # (p0, p1, ...): statements that differ only in their constants (TPC-H
        # substitution parameters, a subquery's result) share one kernel
        self.params: List[int] = []

    def tmp(self) -> str:
        self.n += 1
        return f"t{self.n}"

    def input(self, c: Column) -> int:
        if c.is_wide or c.dtype.is_string or c.dtype.kind not in _STORE or c.data.dim() != 1:
            raise Bail("input column type")
        if c.data.dtype != c.dtype.torch_dtype:
            raise Bail("input storage dtype")
        k = self._idx.get(id(c))
        if k is None:
            k = len(self.inputs)
            self._idx[id(c)] = k
            self.inputs.append(c)
            self.in_key.append((c.dtype.kind, c.dtype.precision, c.dtype.scale, c.valid is not None))
        return k

    # value = (expr, valid-expr or None, DataType)
    def emit(self, e: Expr):
        m = getattr(self, "_" + type(e).__name__, None)
        if m is None:
            return self._sub(e)
        try:
            return m(e)
        except Bail:
            if isinstance(e, (ColRef, Lit)):
                raise
            return self._sub(e)

    def _sub(self, e: Expr):
        """Evaluate a subtree the generator does not cover with the node-by-node
        evaluator; its result enters the kernel as an input column."""
        self.ev._jit_off += 1
        try:
            v = self.ev.eval(e, self.b)
        finally:
            self.ev._jit_off -= 1
        if not isinstance(v, Column):
            return self._lit_value(v.value, v.dtype if v.dtype.kind != "null" else e.dtype)
        return self._col(v)

    def _col(self, c: Column):
        k = self.input(c)
        t = c.dtype
        name = self.tmp()
        if t.kind == "bool":
            self.lines.append(f"const bool {name} = c{k}[i] != 0;")
        else:
            self.lines.append(f"const {_ct(t)} {name} = ({_ct(t)})c{k}[i];")
        return name, (f"(v{k}[i] != 0)" if c.valid is not None else None), t

    def param(self, x, t: DataType) -> str:
        """C expression of constant ``x`` of type ``t`` read from a kernel
        argument (booleans stay inline: they only select code)."""
        import struct
        c = _ct(t)
        if c == "bool":
            return _lit(x, t)
        j = len(self.params)
        if c in ("double", "float"):
            _flit(float(x))                   # non-finite constants are not generated
            self.params.append(struct.unpack("<q", struct.pack("<d", float(x)))[0])
            return f"(({c})i2d(p{j}))"
        x = int(x)
        if c == "i32":
            x = (x + 2**31) % 2**32 - 2**31
        elif not -(2**63) <= x < 2**63:
            raise Bail("literal beyond int64")
        self.params.append(x)
        return f"(({c})p{j})"

    def _lit_value(self, x, t: DataType):
        if x is None:
            return ("0" if _ct(t) != "bool" else "false"), "false", t
        return self.param(x, t), None, t

    def _ColRef(self, e: ColRef):
        c = self.b.columns.get(e.cid)
        if c is None:
            raise Bail("column not in batch")
        return self._col(c)

    def _Passthrough(self, e):
        return self._ColRef(e)

    def _Lit(self, e: Lit):
        t = e.dtype
        if t.kind == "null":
            return "0", "false", T.INT64
        if t.is_string:
            raise Bail("string literal")
        return self._lit_value(e.value, t)

    def _SubqueryExpr(self, e: SubqueryExpr):
        if e.kind != "scalar" or self.ev.ctx is None:
            raise Bail("subquery")
        if e.dtype.is_string:
            raise Bail("string subquery")
        return self._lit_value(self.ev.ctx.scalar_subquery(e), e.dtype)

    # ------------------------------------------------------------ helpers
    def conv(self, v, t: DataType) -> str:
        """expr of value v (expr, valid, src type) in the representation of t
        (expr_eval._convert_tensor)."""
        x, _, src = v
        if src.kind == "null":
            return "0"
        if src == t or (_ct(src) == _ct(t) and not t.is_decimal and not src.is_decimal):
            return x
        if t.is_decimal:
            if src.is_decimal:
                d = t.scale - src.scale
                if d == 0:
                    return x
                if d > 0:
                    return f"(i64)((u64)(i64)({x}) * {10**d}ull)"
                f = 10 ** (-d)
                return f"(((i64)({x}) + ((i64)({x}) > 0 ? {f // 2}LL : ((i64)({x}) < 0 ? -{f // 2}LL : 0LL))) / {f}LL)"
            if src.is_float:
                return f"(i64)__builtin_rint((double)({x}) * {_flit(float(10**t.scale))})"
            return f"(i64)((u64)(i64)({x}) * {10**t.scale}ull)"
        if t.is_float:
            c = _ct(t)
            if src.is_decimal:
                return f"({c})((double)({x}) / {_flit(float(10**src.scale))})"
            return f"({c})({x})"
        if t.is_integer or t.kind in ("date32", "timestamp"):
            c = _ct(t)
            if src.is_decimal:
                return f"({c})((i64)({x}) / {10**src.scale}LL)"
            return f"({c})({x})"
        if t.kind == "bool":
            return f"(({x}) != 0)"
        raise Bail("conversion")

    def convs(self, v, t: DataType) -> str:
        """v converted to t, for a literal via the evaluator's scalar rules."""
        return self.conv(v, t)

    @staticmethod
    def vand(*vs) -> Optional[str]:
        vs = [v for v in vs if v is not None]
        if not vs:
            return None
        return "(" + " && ".join(vs) + ")"

    def bind(self, ctype: str, expr: str) -> str:
        name = self.tmp()
        self.lines.append(f"const {ctype} {name} = {expr};")
        return name

    def wrap(self, ctype: str, a: str, op: str, c: str) -> str:
        if ctype in _UNS:
            u = _UNS[ctype]
            return f"({ctype})(({u})({a}) {op} ({u})({c}))"
        return f"(({a}) {op} ({c}))"

    # -------------------------------------------------------------- nodes
    def _BinOp(self, e: BinOp):
        op = e.op
        if op in ("and", "or"):
            lv, la, _ = self.emit(e.left)
            rv, ra, _ = self.emit(e.right)
            lv, rv = f"({lv})", f"({rv})"
            if la is None and ra is None:
                return self.bind("bool", f"{lv} {'&&' if op == 'and' else '||'} {rv}"), None, T.BOOL
            la, ra = la or "true", ra or "true"
            if op == "and":
                val = f"{lv} && {rv} && {la} && {ra}"
                valid = f"({la} && {ra}) || ({la} && !{lv}) || ({ra} && !{rv})"
            else:
                val = f"({lv} && {la}) || ({rv} && {ra})"
                valid = f"({la} && {ra}) || ({la} && {lv}) || ({ra} && {rv})"
            return self.bind("bool", val), self.bind("bool", valid), T.BOOL
        if op in ("is_distinct_from", "is_not_distinct_from"):
            raise Bail("distinct-from")
        l = self.emit(e.left)
        r = self.emit(e.right)
        lt, rt = l[2], r[2]
        if op in ("=", "<>", "<", "<=", ">", ">="):
            if lt.is_string or rt.is_string:
                raise Bail("string compare")
            t = lt if lt == rt else T.common_numeric(lt, rt)
            rep = T.INT64 if t.kind in ("date32", "timestamp", "bool") else t
            if t.kind == "bool":
                a, c = f"(i32)({l[0]})", f"(i32)({r[0]})"
            else:
                a, c = self.convs(l, rep), self.convs(r, rep)
            cop = {"=": "==", "<>": "!="}.get(op, op)
            return self.bind("bool", f"({a}) {cop} ({c})"), self.vand(l[1], r[1]), T.BOOL
        t = e.dtype
        valid = self.vand(l[1], r[1])
        if t.kind == "date32":
            a = self.conv(l, T.INT32 if lt.kind == "date32" else T.INT64)
            c = self.conv(r, T.INT32 if rt.kind == "date32" else T.INT64)
            return self.bind("i32", f"(i32)" + self.wrap("i64", f"(i64)({a})", op, f"(i64)({c})")), valid, t
        if t.is_decimal and op == "*":
            a = self.conv(l, lt if lt.is_decimal else T.DECIMAL(19, 0))
            c = self.conv(r, rt if rt.is_decimal else T.DECIMAL(19, 0))
            if t.precision > 18:
                self.guard = True
                name = self.tmp()
                self.lines.append(f"i64 {name}; if (__builtin_mul_overflow((i64)({a}), (i64)({c}), &{name})"
                                  f" && {valid or 'true'}) err = 1;")
                return name, valid, t
            return self.bind("i64", self.wrap("i64", f"(i64)({a})", "*", f"(i64)({c})")), valid, t
        if t.kind == "int64" and op == "-" and lt.kind == "date32":
            a, c = self.conv(l, T.INT64), self.conv(r, T.INT64)
            return self.bind("i64", self.wrap("i64", a, "-", c)), valid, t
        ct = _ct(t)
        a, c = self.convs(l, t), self.convs(r, t)
        if op in ("+", "-", "*"):
            return self.bind(ct, self.wrap(ct, a, op, c)), valid, t
        if op == "/":
            cn = self.bind(ct, c)
            zero = f"({cn} == ({ct})0)"
            valid = self.vand(valid, f"!{zero}")
            if ct in ("double", "float"):
                return self.bind(ct, f"({a}) / {cn}"), self.bind("bool", valid), t
            if ct in _UNS:
                # trunc division; the value at a zero divisor is never read (NULL)
                mn = "(-9223372036854775807LL - 1)" if ct == "i64" else "(-2147483647 - 1)"
                return (self.bind(ct, f"{zero} ? ({ct})({a}) : (({cn} == ({ct})-1 && ({a}) == {mn}) ? ({ct})({a}) : "
                                      f"({ct})(({a}) / {cn}))"), self.bind("bool", valid), t)
            raise Bail("division type")
        if op == "%":
            if ct in ("double", "float"):
                return self.bind(ct, f"__builtin_fmod{'f' if ct == 'float' else ''}({a}, {c})"), valid, t
            # integers: only a non-zero literal divisor (torch.fmod's result at
            # a zero divisor is not a value worth reproducing)
            if r[1] is None and isinstance(e.right, Lit) and e.right.value not in (None, 0) and ct in _UNS:
                return self.bind(ct, f"({c}) == ({ct})-1 ? ({ct})0 : ({ct})(({a}) % ({c}))"), valid, t
        raise Bail(f"operator {op}")

    def _Not(self, e: Not):
        v, va, t = self.emit(e.x)
        if t.kind != "bool":
            v = f"(({v}) != 0)"
        return self.bind("bool", f"!({v})"), va, T.BOOL

    def _Neg(self, e: Neg):
        v, va, t = self.emit(e.x)
        ct = _ct(t)
        if ct == "bool":
            raise Bail("neg bool")
        return self.bind(ct, self.wrap(ct, f"({ct})0", "-", v) if ct in _UNS else f"-({v})"), va, t

    def _IsNull(self, e: IsNull):
        _, va, _ = self.emit(e.x)
        if va is None:
            return ("true" if e.negated else "false"), None, T.BOOL
        return self.bind("bool", va if e.negated else f"!({va})"), None, T.BOOL

    def _Cast(self, e: Cast):
        t = e.dtype
        v = self.emit(e.x)
        src = v[2]
        if t.is_string or src.is_string or src.kind == "null":
            raise Bail("string / null cast")
        if src == t:
            return v
        if t.kind == "bool":
            return self.bind("bool", f"({v[0]}) != 0"), v[1], t
        x = self.conv(v, t if t.kind != "date32" else T.INT32)
        return self.bind(_ct(t), f"({_ct(t)})({x})"), v[1], t

    def _Case(self, e: Case):
        t = e.dtype
        if t.is_string or t.kind == "null":
            raise Bail("string case")
        ct = _ct(t)
        arms = []
        for cond, val in e.whens:
            cv, cva, ctt = self.emit(cond)
            m = cv if ctt.kind == "bool" else f"(({cv}) != 0)"
            if cva is not None:
                m = f"({m} && {cva})"
            arms.append((self.bind("bool", m), self.emit(val)))
        els = self.emit(e.else_) if e.else_ is not None else ("0", "false", t)
        out = self.bind(ct, f"({ct})({self.conv(els, t)})") if els[2].kind != "null" else self.bind(ct, "0")
        nullable = els[1] is not None or any(v[1] is not None for _, v in arms)
        ov = self.bind("bool", els[1] or "true") if nullable else None
        name, vname = self.tmp(), self.tmp()
        self.lines.append(f"{ct} {name} = {out};")
        if nullable:
            self.lines.append(f"bool {vname} = {ov};")
        for m, v in reversed(arms):
            x = f"({ct})({self.conv(v, t)})" if v[2].kind != "null" else "0"
            self.lines.append(f"if ({m}) {{ {name} = {x};" + (f" {vname} = {v[1] or 'true'};" if nullable else "")
                              + " }")
        return name, (vname if nullable else None), t

    def _InList(self, e: InList):
        v, va, t = self.emit(e.x)
        if t.is_string or t.kind == "null":
            raise Bail("string IN")
        from .expr_eval import _convert_scalar
        lits = [_convert_scalar(x.value, x.dtype, t) for x in e.values if x.value is not None]
        ct = _ct(t)
        x = self.bind(ct, v)
        hit = " || ".join(f"{x} == {self.param(c, t)}" for c in lits) or "false"
        return self.bind("bool", f"!({hit})" if e.negated else f"({hit})"), va, T.BOOL

    def _Func(self, e: Func):
        name = e.name
        if name == "coalesce":
            t = e.dtype
            if t.is_string or t.kind == "null":
                raise Bail("string coalesce")
            args = [self.emit(a) for a in e.args]
            ct = _ct(t)
            last = args[-1]
            out, vout = self.tmp(), self.tmp()
            self.lines.append(f"{ct} {out} = ({ct})({self.conv(last, t) if last[2].kind != 'null' else '0'});")
            self.lines.append(f"bool {vout} = {last[1] or 'true'};")
            for a in reversed(args[:-1]):
                x = f"({ct})({self.conv(a, t)})" if a[2].kind != "null" else "0"
                if a[1] is None:
                    self.lines.append(f"{out} = {x}; {vout} = true;")
                else:
                    self.lines.append(f"if ({a[1]}) {{ {out} = {x}; {vout} = true; }}")
            return out, vout, t
        args = [self.emit(a) for a in e.args]
        if name == "abs":
            v, va, t = args[0]
            ct = _ct(t)
            return self.bind(ct, f"({v}) < 0 ? " + (self.wrap(ct, f"({ct})0", "-", v) if ct in _UNS else f"-({v})")
                             + f" : ({v})"), va, t
        if name == "date_part":
            v, va, t = args[0]
            if t.kind != "date32":
                raise Bail("date_part of non-date")
            from ..ops.misc import DATE_FIELDS
            if e.options[0] not in DATE_FIELDS:
                raise Bail(f"date_part {e.options[0]}")
            return self.bind("i32", f"date_part((i32)({v}), {DATE_FIELDS[e.options[0]]})"), va, T.INT32
        if name == "add_months":
            v, va, t = args[0]
            if t.kind != "date32":
                raise Bail("add_months of non-date")
            months, days = e.options
            return self.bind("i32", f"add_months((i32)({v}), {int(months)}LL, {int(days)}LL)"), va, T.DATE32
        if name == "round":
            v, va, t = args[0]
            d = e.options[0]
            if t.is_decimal:
                s = t.scale
                drop = s - min(s, max(d, 0))
                if drop <= 0:
                    return v, va, e.dtype
                f = 10**drop
                x = self.bind("i64", v)
                return (self.bind("i64", f"((({x}) < 0 ? -(i64)({x}) : (i64)({x})) + {f // 2}LL) / {f}LL * "
                                         f"(({x}) > 0 ? 1LL : (({x}) < 0 ? -1LL : 0LL))"), va, e.dtype)
            if t.is_integer:
                return v, va, t
            if not t.is_float:
                raise Bail("round type")
            f = _flit(10.0**d)
            # half away from zero, like the CPU path (Rust f64::round)
            return self.bind("double", f"__builtin_round((double)({v}) * {f}) / {f}"), va, T.FLOAT64
        if name in ("sqrt", "ln", "log10", "exp", "floor", "ceil"):
            v, va, t = args[0]
            x = self.conv((v, va, t), T.FLOAT64)
            fn = {"sqrt": "__builtin_sqrt", "ln": "__ocml_log_f64", "log10": "__ocml_log10_f64",
                  "exp": "__ocml_exp_f64", "floor": "__builtin_floor", "ceil": "__builtin_ceil"}[name]
            return self.bind("double", f"{fn}({x})"), va, T.FLOAT64
        if name == "power":
            a = self.conv(args[0], T.FLOAT64)
            c = self.conv(args[1], T.FLOAT64)
            return self.bind("double", f"__ocml_pow_f64({a}, {c})"), self.vand(args[0][1], args[1][1]), T.FLOAT64
        raise Bail(f"function {name}")


def _source(g: _Gen, out_t: DataType, val: str, valid: Optional[str]) -> str:
    ps = []
    for k, c in enumerate(g.inputs):
        ps.append(f"const {_STORE[c.dtype.kind]}* __restrict__ c{k}")
        if c.valid is not None:
            ps.append(f"const u8* __restrict__ v{k}")
    ps.append(f"{_STORE[out_t.kind]}* __restrict__ out")
    if valid is not None:
        ps.append("u8* __restrict__ outv")
    ps += ["int* __restrict__ errp", "i64 n"] + [f"i64 p{j}" for j in range(len(g.params))]
    body = "\n".join(g.lines)
    # device math library entry points, declared only where used (hiprtc links
    # ocml; a bare __builtin_exp / log / pow has no gfx950 lowering), so the
    # recorded sources of other kernels (igloo_amd/jit_sources) stay valid
    ocml = "".join(f'extern "C" __device__ double {fn}({args});\n' for fn, args in _OCML if fn in body)
    L = [PRELUDE + ocml, f"extern \"C\" __global__ __launch_bounds__({BLOCK}) void igloo_jit_expr(" + ", ".join(ps) + ") {",
         "  int err = 0;",
         f"  for (i64 i = (i64)blockIdx.x * {BLOCK} + threadIdx.x; i < n; i += (i64)gridDim.x * {BLOCK}) {{"]
    L += ["    " + s for s in g.lines]
    store = f"({_STORE[out_t.kind]})({val})" if out_t.kind != "bool" else f"(u8)(({val}) ? 1 : 0)"
    L.append(f"    out[i] = {store};")
    if valid is not None:
        L.append(f"    outv[i] = ({valid}) ? 1 : 0;")
    L.append("  }")
    L.append("  if (err) atomicOr(errp, 1);")
    L.append("}")
    return "\n".join(L)


_OCML = (("__ocml_exp_f64", "double"), ("__ocml_log_f64", "double"), ("__ocml_log10_f64", "double"),
         ("__ocml_pow_f64", "double, double"))
def _bound(e: Expr, b: Batch) -> Optional[Tuple[float, float]]:
    r = _bound_node(e, b)
    if r is not None:
        # a node whose values could leave its stored type would wrap in the kernel
        t = e.dtype
        sc = 10 ** t.scale if t.is_decimal else 1
        lim = 2.0 ** (8 * t.torch_dtype.itemsize - 1) * 0.5
        if not (-lim <= r[0] * sc and r[1] * sc <= lim):
            return None
    return r


def _bound_node(e: Expr, b: Batch) -> Optional[Tuple[float, float]]:
    """Interval of the real values of an integer / decimal expression, from
    readback-free bounds of its columns (ops/hashing.py key_bound: the range
    of the resident column a column was gathered from) through + - *,
    negation, casts and CASE arms; None when any part is unbounded. The
    result bounds the kernel's output (``_igloo_bound``), so an integer SUM
    over it needs no "fits in int64" readback (ops/agg.py _sum_fits):
    sum(l_extendedprice * (1 - l_discount)) over 600M rows provably fits."""
    t = e.dtype
    if not (t.is_integer or t.is_decimal):
        return None
    sc = float(10 ** t.scale) if t.is_decimal else 1.0
    if isinstance(e, Lit):
        return None if e.value is None else (int(e.value) / sc, int(e.value) / sc)
    if isinstance(e, ColRef):
        c = b.columns.get(e.cid)
        if c is None or c.data.dim() != 1 or c.data.dtype not in (torch.int32, torch.int64):
            return None
        from ..ops.hashing import key_bound
        kb = key_bound(c.data)
        return None if kb is None else (kb[0] / sc, kb[1] / sc)
    if isinstance(e, BinOp) and e.op in ("+", "-", "*"):
        if not (e.left.dtype.is_integer or e.left.dtype.is_decimal) or \
                not (e.right.dtype.is_integer or e.right.dtype.is_decimal):
            return None
        l, r = _bound(e.left, b), _bound(e.right, b)
        if l is None or r is None:
            return None
        if e.op == "+":
            return l[0] + r[0], l[1] + r[1]
        if e.op == "-":
            return l[0] - r[1], l[1] - r[0]
        p = [l[0] * r[0], l[0] * r[1], l[1] * r[0], l[1] * r[1]]
        return min(p), max(p)
    if isinstance(e, Neg):
        x = _bound(e.x, b)
        return None if x is None else (-x[1], -x[0])
    if isinstance(e, Cast):
        return _bound(e.x, b)
    if isinstance(e, Func) and e.name == "date_part" and e.options:
        field = e.options[0]
        fixed = {"month": (1, 12), "day": (1, 31), "quarter": (1, 4), "dow": (0, 6), "doy": (1, 366)}
        if field in fixed:
            return fixed[field]
        x = e.args[0] if e.args else None
        if field != "year" or not isinstance(x, ColRef) or x.dtype.kind != "date32":
            return None
        c = b.columns.get(x.cid)
        if c is None or c.data.dim() != 1 or c.data.dtype not in (torch.int32, torch.int64):
            return None
        from ..ops.hashing import key_bound
        kb = key_bound(c.data)
        if kb is None:
            return None
        import datetime
        try:
            d0 = datetime.date(1970, 1, 1)
            return (d0 + datetime.timedelta(days=kb[0])).year, (d0 + datetime.timedelta(days=kb[1])).year
        except OverflowError:
            return None
    if isinstance(e, Case):
        arms = [v for _, v in e.whens] + ([e.else_] if e.else_ is not None else [])
        bs = [_bound(v, b) for v in arms]
        if not bs or any(x is None for x in bs):
            return None
        return min(x[0] for x in bs), max(x[1] for x in bs)
    return None


def _raw_bound(e: Expr, b: Batch, t: DataType) -> Optional[Tuple[int, int]]:
    """``_bound`` in the output's stored representation (scaled for decimals),
    widened for rounding; None past int64."""
    import math
    try:
        bd = _bound(e, b)
    except (KeyError, AttributeError, TypeError):
        return None
    if bd is None:
        return None
    sc = 10 ** t.scale if t.is_decimal else 1
    lo, hi = bd[0] * sc, bd[1] * sc
    pad = 2 + 1e-9 * max(abs(lo), abs(hi))
    lo, hi = math.floor(lo - pad), math.ceil(hi + pad)
    lim = 2**31 if t.torch_dtype == torch.int32 else 2**63
    return (lo, hi) if -lim <= lo and hi < lim else None


_SIMPLE = (ColRef, Lit)
_ROOTS = (BinOp, Case, Cast, Func, Not, Neg, IsNull, InList)


_SOURCE_SINK: Optional[list] = None


def evaluate(e: Expr, b: Batch, ev) -> object:
    """Column for ``e`` from one generated kernel; None when the expression is
    not worth / not able to be generated; PENDING while it compiles."""
    if not (ENABLED and jit.enabled()) or isinstance(e, _SIMPLE) or b.num_rows == 0:
        return None
    if e.dtype.is_string or e.dtype.kind not in _STORE:
        return None
    if not isinstance(e, _ROOTS):
        return None
    g = _Gen(b, ev)
    try:
        # the root itself must be generated (a fallback root would only copy)
        val, valid, t = getattr(g, "_" + type(e).__name__)(e)
    except Bail as why:
        if _DEBUG:
            print(f"[expr_jit] {e.sql()}: not generated ({why})", flush=True)
        return None
    if not g.inputs or t.kind not in _STORE or t.is_string:
        return None          # constant folding is the evaluator's job
    out_t = t                # the evaluator's result type for this node
    src = _source(g, out_t, val, valid)
    if _SOURCE_SINK is not None:      # tests: collect generated sources
        _SOURCE_SINK.append(src)
        return None
    k = jit.get(src, "igloo_jit_expr")
    if k is None:
        return PENDING
    n = b.num_rows
    dev = g.inputs[0].data.device
    out = torch.empty(n, dtype=out_t.torch_dtype, device=dev)
    outv = torch.empty(n, dtype=torch.bool, device=dev) if valid is not None else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    args = []
    for c in g.inputs:
        args.append(c.data.data_ptr())
        if c.valid is not None:
            args.append(c.valid.data_ptr())
    args.append(out.data_ptr())
    if outv is not None:
        args.append(outv.data_ptr())
    args += [err.data_ptr(), n] + g.params
    from ..ops._lib import stream, to_host_ints
    grid = max(1, min(-(-n // BLOCK), 256 * 16))
    k.launch(grid, BLOCK, 0, stream(out), args)
    if g.guard:
        msg = "decimal multiplication overflows 64-bit fixed point; CAST to DOUBLE"
        qctx = getattr(ev, "ctx", None)
        if qctx is not None and hasattr(qctx, "deferred_checks"):
            qctx.deferred_checks.append((err, msg))     # checked once at the end of the query
        elif to_host_ints(err)[0]:
            raise ExecutionError(msg)
    if outv is None and out.dtype in (torch.int32, torch.int64) and (out_t.is_integer or out_t.is_decimal):
        rb = _raw_bound(e, b, out_t)
        if rb is not None:
            out._igloo_bound = rb
    return Column(out_t, out, outv)
