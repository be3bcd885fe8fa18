"""Vectorized evaluation of bound expressions over a device ``Batch``.

Numeric work is elementwise torch on the batch's device (fully on-GPU for
GPU batches); string predicates/transforms, date parts, gathers and
hash-based operators dispatch to the gfx950 kernels in ``igloo_amd.ops``.
NULLs follow SQL three-valued logic via validity masks.

Parity: DataFusion ``PhysicalExpr::evaluate`` as called by the reference's
FilterExec / ProjectionExec (reference crates/engine/src/operators/filter.rs:47,
projection.rs:60-64).
"""
from __future__ import annotations

import math
import os
from typing import Any, Optional, Tuple, Union

import numpy as np
import re

import pyarrow as pa
import pyarrow.compute as pc
import torch

from .. import types as T
from ..columnar import Batch, Column, batch_device
from ..ops import misc as M
from ..ops._lib import to_host_ints
from ..ops import strings as S
from ..sql.expr import (AggCall, BinOp, Case, Cast, ColRef, Expr, Func, InList, IsNull, Like, Lit, Neg, Not,
                        SubqueryExpr, col_refs)
from ..types import DataType
from ..utils.errors import ExecutionError, NotSupported

#: generated expression kernels (exec/expr_jit.py) for composite expressions
#: over GPU batches of at least this many rows
JIT_MIN_ROWS = 1
_JIT_ROOTS = {BinOp, Case, Cast, Func, Not, Neg, IsNull, InList}
_JIT_ON_CPU = False   # tests: run the generator (source collection only) on CPU batches


_NESTED = ("make_array", "struct", "array_length", "array_element", "get_field", "array_has", "array_to_string",
           "regexp_match", "unnest")


class Scalar:
    __slots__ = ("value", "dtype")

    def __init__(self, value: Any, dtype: DataType):
        self.value = value
        self.dtype = dtype

    def __repr__(self):
        return f"Scalar({self.value!r}, {self.dtype})"


Value = Union[Column, Scalar]


def _and_valid(a: Optional[torch.Tensor], b: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if a is None:
        return b
    if b is None:
        return a
    return a & b


class Evaluator:
    def __init__(self, ctx=None):
        self.ctx = ctx

    # ------------------------------------------------------------------ entry
    _jit_off = 0   # > 0 while a generated kernel's uncovered subtree is evaluated here

    def eval(self, e: Expr, b: Batch) -> Value:
        if not self._jit_off and type(e) in _JIT_ROOTS and b.num_rows >= JIT_MIN_ROWS and b.columns \
                and (_JIT_ON_CPU or getattr(batch_device(b), "type", None) == "cuda"):
            from . import expr_jit
            r = expr_jit.evaluate(e, b, self)
            if isinstance(r, Column):
                return r
            if r is expr_jit.PENDING:
                # compiling in the background: this run goes node by node without
                # generating code for the subtrees as well
                self._jit_off += 1
                try:
                    return self._eval_nodes(e, b)
                finally:
                    self._jit_off -= 1
        return self._eval_nodes(e, b)

    def _eval_nodes(self, e: Expr, b: Batch) -> Value:
        m = getattr(self, "_" + type(e).__name__, None)
        if m is None:
            if isinstance(e, ColRef):
                return self._ColRef(e, b)
            raise NotSupported(f"cannot evaluate {type(e).__name__}")
        return m(e, b)

    @staticmethod
    def prefetch(exprs, b: Batch) -> None:
        """A join result's (LateBatch) columns read by ``exprs``: gathered
        together, part by part, before they are read one by one."""
        pf = getattr(b, "prefetch", None)
        if pf is not None:
            cids = set()
            for e in exprs:
                if e is not None:
                    cids |= col_refs(e)
            if len(cids) > 1:
                pf(cids)

    def column(self, e: Expr, b: Batch) -> Column:
        """Evaluate and broadcast to a full column."""
        self.prefetch((e,), b)
        v = self.eval(e, b)
        if isinstance(v, Scalar):
            return Column.full(v.value, e.dtype if v.dtype.kind == "null" else v.dtype, b.num_rows, self.device(b))
        return v

    def mask(self, e: Expr, b: Batch) -> torch.Tensor:
        """Predicate -> bool tensor (NULL counts as False)."""
        self.prefetch((e,), b)
        v = self.eval(e, b)
        dev = self.device(b)
        if isinstance(v, Scalar):
            return torch.full((b.num_rows,), bool(v.value) if v.value is not None else False, dtype=torch.bool, device=dev)
        m = v.data if v.data.dtype == torch.bool else v.data != 0
        if v.valid is not None:
            m = m & v.valid
        return m

    def device(self, b: Batch) -> torch.device:
        d = batch_device(b)
        if d is not None:
            return d
        return torch.device(self.ctx.device if self.ctx is not None else "cpu")

    # ------------------------------------------------------------ leaf nodes
    def _ColRef(self, e: ColRef, b: Batch) -> Value:
        try:
            return b.columns[e.cid]
        except KeyError:
            raise ExecutionError(f"column {e.sql()} not available in batch {list(b.columns)}") from None

    def _Passthrough(self, e, b):
        return self._ColRef(e, b)

    def _Lit(self, e: Lit, b: Batch) -> Value:
        return Scalar(e.value, e.dtype)

    def _SubqueryExpr(self, e: SubqueryExpr, b: Batch) -> Value:
        if e.kind != "scalar":
            raise ExecutionError("unexpected EXISTS/IN subquery at execution (not decorrelated)")
        if self.ctx is None:
            raise ExecutionError("scalar subquery needs an execution context")
        val = self.ctx.scalar_subquery(e)
        return Scalar(val, e.dtype)

    # ------------------------------------------------------- numeric helpers
    def _num(self, v: Value, t: DataType):
        """Value -> (tensor | python number, validity) in representation of type t."""
        if isinstance(v, Scalar):
            x = v.value
            if x is None:
                return None, None
            return _convert_scalar(x, v.dtype, t), None
        return _convert_tensor(v, t), v.valid

    # ---------------------------------------------------------------- binops
    def _BinOp(self, e: BinOp, b: Batch) -> Value:
        op = e.op
        if op in ("and", "or"):
            return self._logic(e, b)
        l = self.eval(e.left, b)
        r = self.eval(e.right, b)
        if op in ("=", "<>", "<", "<=", ">", ">=", "is_distinct_from", "is_not_distinct_from"):
            return self._compare(op, l, r, e.left.dtype, e.right.dtype, b)
        if isinstance(l, Scalar) and isinstance(r, Scalar):
            from ..sql.binder import _fold
            f = _fold(BinOp(op, Lit(l.value, l.dtype), Lit(r.value, r.dtype), e.dtype))
            if isinstance(f, Lit):
                return Scalar(f.value, f.dtype)
        t = e.dtype
        if t.kind == "date32":
            a, va = self._num(l, T.INT32 if l.dtype.kind == "date32" else T.INT64)
            c, vc = self._num(r, T.INT32 if r.dtype.kind == "date32" else T.INT64)
            out = a + c if op == "+" else a - c
            return self._mk(out, t, _and_valid(va, vc), b)
        lt = t
        if t.is_decimal and op == "*":
            a, va = self._num(l, l.dtype if l.dtype.is_decimal else T.DECIMAL(19, 0))
            c, vc = self._num(r, r.dtype if r.dtype.is_decimal else T.DECIMAL(19, 0))
            if t.precision > 18:
                a, c = _overflow_guard(a, c)
            out = a * c
            return self._mk(out, t, _and_valid(va, vc), b)
        if t.kind == "int64" and op in ("-",) and l.dtype.kind == "date32":
            a, va = self._num(l, T.INT64)
            c, vc = self._num(r, T.INT64)
            return self._mk(a - c, t, _and_valid(va, vc), b)
        a, va = self._num(l, lt)
        c, vc = self._num(r, lt)
        valid = _and_valid(va, vc)
        if a is None or c is None:
            return Scalar(None, t)
        if op == "+":
            out = a + c
        elif op == "-":
            out = a - c
        elif op == "*":
            out = a * c
        elif op == "/":
            if t.is_float:
                out = a / c
                zero = (c == 0) if isinstance(c, torch.Tensor) else None
                if zero is not None and _any(zero):
                    valid = _and_valid(valid, ~zero)
                elif not isinstance(c, torch.Tensor) and c == 0:
                    return Scalar(None, t)
            else:
                if isinstance(c, torch.Tensor):
                    zero = c == 0
                    safe = torch.where(zero, torch.ones_like(c), c)
                    out = torch.div(a, safe, rounding_mode="trunc")
                    if _any(zero):
                        valid = _and_valid(valid, ~zero)
                else:
                    if c == 0:
                        return Scalar(None, t)
                    out = torch.div(a, c, rounding_mode="trunc")
        elif op == "%":
            out = torch.fmod(a, c) if isinstance(a, torch.Tensor) else torch.fmod(torch.as_tensor(a), c)
        else:
            raise NotSupported(f"operator {op}")
        return self._mk(out, t, valid, b)

    def _mk(self, out, t: DataType, valid, b: Batch) -> Value:
        if not isinstance(out, torch.Tensor):
            return Scalar(out, t)
        if out.dim() == 0:
            out = out.expand(b.num_rows)
        return Column(t, out.to(t.torch_dtype) if t.kind != "decimal" else out.to(torch.int64), valid)

    def _logic(self, e: BinOp, b: Batch) -> Value:
        l = self.eval(e.left, b)
        r = self.eval(e.right, b)
        is_and = e.op == "and"
        # scalar short-circuits
        for x, y in ((l, r), (r, l)):
            if isinstance(x, Scalar):
                if x.value is None:
                    if isinstance(y, Scalar):
                        return Scalar(None if (y.value is None or y.value == is_and) else y.value, T.BOOL)
                    # NULL AND y -> (y false -> false else null); NULL OR y -> (y true -> true else null)
                    yv, yvalid = _bool_parts(y)
                    known = (~yv if is_and else yv)
                    if yvalid is not None:
                        known = known & yvalid
                    return Column(T.BOOL, yv if not is_and else torch.zeros_like(yv), known)
                if bool(x.value) == (not is_and):
                    return Scalar(not is_and, T.BOOL)
                return y
        lv, lval = _bool_parts(l)
        rv, rval = _bool_parts(r)
        if is_and:
            out = lv & rv
            if lval is None and rval is None:
                return Column(T.BOOL, out)
            la = lval if lval is not None else torch.ones_like(lv)
            ra = rval if rval is not None else torch.ones_like(rv)
            valid = (la & ra) | (la & ~lv) | (ra & ~rv)
            return Column(T.BOOL, out & la & ra, valid)
        out = lv | rv
        if lval is None and rval is None:
            return Column(T.BOOL, out)
        la = lval if lval is not None else torch.ones_like(lv)
        ra = rval if rval is not None else torch.ones_like(rv)
        valid = (la & ra) | (la & lv) | (ra & rv)
        return Column(T.BOOL, (lv & la) | (rv & ra), valid)

    def _compare(self, op, l: Value, r: Value, lt: DataType, rt: DataType, b: Batch) -> Value:
        if isinstance(l, Scalar) and isinstance(r, Scalar):
            if l.value is None or r.value is None:
                return Scalar(None, T.BOOL)
            import operator as o
            f = {"=": o.eq, "<>": o.ne, "<": o.lt, "<=": o.le, ">": o.gt, ">=": o.ge}[op]
            return Scalar(bool(f(l.value, r.value)), T.BOOL)
        if lt.is_string or rt.is_string:
            return self._compare_strings(op, l, r, b)
        if isinstance(l, Scalar) and l.value is None or isinstance(r, Scalar) and r.value is None:
            return Scalar(None, T.BOOL)
        t = lt if lt == rt else T.common_numeric(lt, rt)
        rep = T.INT64 if t.kind in ("date32", "timestamp", "bool") else t
        if t.kind == "bool":
            def bpart(v):
                if isinstance(v, Scalar):
                    return int(bool(v.value)), None
                return _bool_parts(v)[0].to(torch.int8), v.valid
            a, va = bpart(l)
            c, vc = bpart(r)
        else:
            a, va = self._num(l, rep)
            c, vc = self._num(r, rep)
        fn = {"=": torch.eq, "<>": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}[op]
        if not isinstance(a, torch.Tensor):
            # flip so the tensor is on the left
            flip = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "<>": "<>"}[op]
            fn = {"=": torch.eq, "<>": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}[flip]
            a, c = c, a
        out = fn(a, c)
        return Column(T.BOOL, out, _and_valid(va, vc))

    def _compare_strings(self, op, l: Value, r: Value, b: Batch) -> Value:
        if isinstance(r, Scalar) or isinstance(l, Scalar):
            if isinstance(l, Scalar):
                flip = {"<": ">", "<=": ">=", ">": "<", ">=": "<=", "=": "=", "<>": "<>"}[op]
                l, r, op = r, l, flip
            if r.value is None:
                return Scalar(None, T.BOOL)
            return Column(T.BOOL, S.compare_const(l, op, str(r.value)), l.valid)
        # two string columns: compare through one shared dictionary
        if l.is_dict and r.is_dict and l.dictionary is r.dictionary and op in ("=", "<>"):
            out = l.data == r.data if op == "=" else l.data != r.data
            return Column(T.BOOL, out, _and_valid(l.valid, r.valid))
        n = len(l)
        both = _concat_strings(S.decode(l), S.decode(r))
        ranks = S.sort_ranks(both)
        a, c = ranks[:n], ranks[n:]
        fn = {"=": torch.eq, "<>": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}[op]
        return Column(T.BOOL, fn(a, c), _and_valid(l.valid, r.valid))

    # ---------------------------------------------------------------- unary
    def _Not(self, e: Not, b: Batch) -> Value:
        v = self.eval(e.x, b)
        if isinstance(v, Scalar):
            return Scalar(None if v.value is None else not v.value, T.BOOL)
        d, valid = _bool_parts(v)
        return Column(T.BOOL, ~d, valid)

    def _Neg(self, e: Neg, b: Batch) -> Value:
        v = self.eval(e.x, b)
        if isinstance(v, Scalar):
            return Scalar(None if v.value is None else -v.value, v.dtype)
        return Column(v.dtype, -v.data, v.valid)

    def _IsNull(self, e: IsNull, b: Batch) -> Value:
        v = self.eval(e.x, b)
        if isinstance(v, Scalar):
            return Scalar((v.value is None) != e.negated, T.BOOL)
        dev = v.device
        if v.valid is None:
            return Scalar(e.negated, T.BOOL)
        return Column(T.BOOL, v.valid.clone() if e.negated else ~v.valid)

    # ------------------------------------------------------------- functions
    def _Cast(self, e: Cast, b: Batch) -> Value:
        v = self.eval(e.x, b)
        t = e.dtype
        if isinstance(v, Scalar):
            from ..sql.binder import _fold_cast
            return Scalar(_fold_cast(Lit(v.value, v.dtype), t).value, t)
        src = v.dtype
        if src == t:
            return v
        if t.is_string:
            if src.is_string:
                return v
            if src.is_decimal or src.kind in ("date32",) or src.is_numeric or src.kind == "bool":
                return S.to_string(v)       # GPU text formatting (strexpr.hip)
        if t.kind == "timestamp" and src.kind == "date32":
            return Column(t, v.data.to(torch.int64) * _US_DAY, v.valid)
        if t.kind == "date32" and src.kind == "timestamp":
            return Column(t, torch.div(v.data, _US_DAY, rounding_mode="floor").to(torch.int32), v.valid)
        if src.is_string and t.kind == "timestamp":
            return _parse_ts_host(v)
        if src.is_string:
            return S.parse(v, t)            # GPU parse (strexpr.hip); malformed -> error
        if t.kind == "bool":
            return Column(t, v.data != 0, v.valid)
        if src.kind == "null":
            return Column.full(None, t, len(v), v.device)
        return Column(t, _convert_tensor(v, t if t.kind not in ("date32",) else T.INT32).to(t.torch_dtype), v.valid)

    def _Case(self, e: Case, b: Batch) -> Value:
        n = b.num_rows
        dev = self.device(b)
        t = e.dtype
        vals = []
        for cond, val in e.whens:
            vals.append((self.mask(cond, b), self.eval(val, b)))
        els = self.eval(e.else_, b) if e.else_ is not None else Scalar(None, t)
        if t.is_string:
            return self._case_strings(vals, els, n, dev)
        rep = t
        out_v, out_valid = _full_of(els, rep, n, dev)
        for m, v in reversed(vals):
            x, xv = _full_of(v, rep, n, dev)
            out_v = torch.where(m, x, out_v)
            if out_valid is not None or xv is not None:
                ov = out_valid if out_valid is not None else torch.ones(n, dtype=torch.bool, device=dev)
                xvv = xv if xv is not None else torch.ones(n, dtype=torch.bool, device=dev)
                out_valid = torch.where(m, xvv, ov)
        return Column(t, out_v.to(t.torch_dtype) if t.kind != "null" else out_v, out_valid)

    def _case_strings(self, vals, els, n, dev) -> Column:
        branches = [v for _, v in vals] + [els]
        if all(isinstance(v, Scalar) for v in branches):
            lits = []
            for v in branches:
                if v.value is not None and v.value not in lits:
                    lits.append(v.value)
            code = {s: i for i, s in enumerate(lits)}
            ev = els.value
            codes = torch.full((n,), code.get(ev, 0), dtype=torch.int32, device=dev)
            valid = None if ev is not None else torch.zeros(n, dtype=torch.bool, device=dev)
            for m, v in reversed(vals):
                codes = torch.where(m, torch.full_like(codes, code.get(v.value, 0)), codes)
                if valid is not None or v.value is None:
                    valid = torch.where(m, torch.full((n,), v.value is not None, dtype=torch.bool, device=dev),
                                        valid if valid is not None else torch.ones(n, dtype=torch.bool, device=dev))
            dic = Column.from_arrow(pa.array(lits or [""], pa.large_string()), device=dev, dict_encode=False)
            return Column(T.UTF8, codes, valid, dictionary=dic)
        # general case: the first matching WHEN picks its branch (else the
        # ELSE branch); one device string gather assembles the rows
        choice = torch.full((n,), len(vals), dtype=torch.int64, device=dev)
        for k in range(len(vals) - 1, -1, -1):
            choice = torch.where(vals[k][0], torch.full_like(choice, k), choice)
        return S.select_rows([self._str_col(v, dev) for v in branches], choice, n)

    @staticmethod
    def _str_col(v, dev) -> Column:
        """A string operand as a column (a scalar becomes a one-row constant;
        NULL a one-row NULL)."""
        if isinstance(v, Scalar):
            if v.value is None:
                c = S.const_column("", dev)
                return Column(T.UTF8, c.data, torch.zeros(1, dtype=torch.bool, device=dev), offsets=c.offsets)
            return S.const_column(str(v.value), dev)
        return v

    def _InList(self, e: InList, b: Batch) -> Value:
        x = e.x
        if isinstance(x, Func) and x.name == "substr" and x.options[0] == 1 and x.options[1] \
                and x.options[1] >= 1 and all(isinstance(y, Lit) for y in e.values):
            # substr(s, 1, L) IN (...): the prefixes compared in place (ops/strings.py in_set)
            c = self.eval(x.args[0], b)
            if isinstance(c, Column) and c.is_plain_string and c.data.is_cuda:
                m = S.in_set(c, [str(y.value) for y in e.values if y.value is not None], prefix_chars=x.options[1])
                return Column(T.BOOL, ~m if e.negated else m, c.valid)
        v = self.eval(e.x, b)
        if isinstance(v, Scalar):
            hit = any(x.value == v.value for x in e.values)
            return Scalar(hit != e.negated if v.value is not None else None, T.BOOL)
        vals = [x.value for x in e.values if x.value is not None]
        if v.dtype.is_string:
            m = S.in_list(v, [str(x) for x in vals])
        else:
            t = v.dtype
            lits = torch.tensor([_convert_scalar(x, xx.dtype, t) for x, xx in zip(vals, [y for y in e.values if y.value is not None])],
                                dtype=v.data.dtype, device=v.device)
            m = torch.isin(v.data, lits)
        if e.negated:
            m = ~m
        return Column(T.BOOL, m, v.valid)

    def _Like(self, e: Like, b: Batch) -> Value:
        v = self.eval(e.x, b)
        if isinstance(v, Scalar):
            if v.value is None:
                return Scalar(None, T.BOOL)
            rx = S.like_regex(e.pattern, e.case_insensitive, e.escape)
            return Scalar((rx.fullmatch(v.value) is not None) != e.negated, T.BOOL)
        return Column(T.BOOL, S.like(v, e.pattern, e.case_insensitive, e.negated, e.escape), v.valid)

    def _Func(self, e: Func, b: Batch) -> Value:
        name = e.name
        args = [self.eval(a, b) for a in e.args]
        if args and all(isinstance(a, Scalar) for a in args) and name not in ("coalesce",):
            return self._func_scalar(e, args)
        if name in _NESTED:
            return self._nested(e, args, b)
        if name in ("hex_digest", "to_char"):
            from ..ops import digest as DG
            c = args[0]
            if isinstance(c, Scalar):
                c = Column.full(c.value, e.args[0].dtype, b.num_rows, self.device(b))
            return DG.hex_digest(c, e.options[0]) if name == "hex_digest" else DG.to_char(c, e.options[0])
        if name == "upper":
            return S.upper(args[0])
        if name == "lower":
            return S.lower(args[0])
        if name == "substr":
            start, ln = e.options
            return S.substr(args[0], start, ln)
        if name == "char_length":
            c = args[0]
            return Column(T.INT32, S.char_length(c), c.valid)
        if name == "date_part":
            c = args[0]
            if e.options[0] == "week":
                return Column(T.INT32, iso_week(c.data.to(torch.int64)).to(torch.int32), c.valid)
            return Column(T.INT32, M.date_part(c.data, e.options[0]), c.valid)
        if name in _STRFN:
            from ..ops import strfuncs as SF
            c = args[0]
            return SF.apply(c, name, e.options)
        if name in ("strpos", "ascii", "octet_length"):
            from ..ops import strfuncs as SF
            c = args[0]
            return Column(T.INT32, SF.apply_int(c, name, e.options), c.valid)
        if name in ("regexp_like", "regexp_count", "regexp_replace"):
            from ..ops import strfuncs as SF
            c = args[0]
            if name == "regexp_replace":
                pat, rep, flags = e.options
                return SF.regexp(c, name, pat, rep, flags)
            pat, flags = e.options
            return Column(e.dtype, SF.regexp(c, name, pat, None, flags), c.valid)
        if name in _MATH1:
            c = args[0]
            x = _convert_tensor(c, T.FLOAT64) if name != "factorial" else c.data.to(torch.int64)
            return Column(e.dtype, _math1(name, x, e.options), c.valid)
        if name in ("logb", "atan2", "nanvl"):
            a, va = self._num(args[0], T.FLOAT64)
            c, vc = self._num(args[1], T.FLOAT64)
            a = a if isinstance(a, torch.Tensor) else torch.tensor(a, dtype=torch.float64, device=self.device(b))
            if name == "logb":
                out = torch.log(c) / torch.log(a)
            elif name == "atan2":
                out = torch.atan2(a, c)
            else:
                out = torch.where(torch.isnan(a), c if isinstance(c, torch.Tensor) else torch.full_like(a, c), a)
            return self._mk(out, T.FLOAT64, _and_valid(va, vc), b)
        if name == "random":
            return Column(T.FLOAT64, torch.rand(b.num_rows, dtype=torch.float64, device=self.device(b)))
        if name == "uuid":
            from ..ops import digest as DG
            return DG.uuid_column(b.num_rows, self.device(b))
        if name in ("greatest", "least"):
            return self._extreme(e, args, b)
        if name in ("gcd", "lcm"):
            a, va = self._num(args[0], T.INT64)
            c, vc = self._num(args[1], T.INT64)
            a = a if isinstance(a, torch.Tensor) else torch.full((b.num_rows,), a, dtype=torch.int64,
                                                                  device=self.device(b))
            g = torch.gcd(a, c if isinstance(c, torch.Tensor) else torch.full_like(a, c))
            out = g if name == "gcd" else torch.where(g == 0, torch.zeros_like(g), (a * c).abs() // g.clamp(min=1))
            return self._mk(out, T.INT64, _and_valid(va, vc), b)
        if name == "date_trunc":
            c = args[0]
            return Column(T.TIMESTAMP, trunc_ts(c.data.to(torch.int64), e.options[0]), c.valid)
        if name == "ts_add":
            c = args[0]
            return Column(T.TIMESTAMP, ts_add(c.data.to(torch.int64), *e.options), c.valid)
        if name == "ts_part":
            c = args[0]
            out = ts_part(c.data.to(torch.int64), e.options[0])
            return Column(e.dtype, out.to(e.dtype.torch_dtype), c.valid)
        if name == "to_unixtime":
            c = args[0]
            return Column(T.INT64, torch.div(c.data.to(torch.int64), 1_000_000, rounding_mode="floor"), c.valid)
        if name == "ts_from_float":
            c = args[0]
            return Column(T.TIMESTAMP, (c.data.to(torch.float64) * 1e6).round().to(torch.int64), c.valid)
        if name == "make_date":
            ys, ms, ds = [self._num(a, T.INT64) for a in args]
            vals = [x if isinstance(x, torch.Tensor) else torch.full((b.num_rows,), x, dtype=torch.int64,
                                                                    device=self.device(b)) for x, _ in (ys, ms, ds)]
            valid = _and_valid(_and_valid(ys[1], ms[1]), ds[1])
            return Column(T.DATE32, days_from_civil(*vals).to(torch.int32), valid)
        if name == "add_months":
            months, days = e.options
            c = args[0]
            return Column(T.DATE32, add_months(c.data, months, days), c.valid)
        if name == "abs":
            c = args[0]
            return Column(c.dtype, c.data.abs(), c.valid)
        if name == "round":
            c = args[0]
            d = e.options[0]
            if c.dtype.is_decimal:
                s = c.dtype.scale
                drop = s - min(s, max(d, 0))
                if drop <= 0:
                    return Column(e.dtype, c.data, c.valid)
                f = 10**drop
                q = torch.div(c.data.abs() + f // 2, f, rounding_mode="floor") * torch.sign(c.data)
                return Column(e.dtype, q, c.valid)
            if c.dtype.is_integer:
                return c
            f = 10.0**d
            x = c.data.double() * f
            # half away from zero (Rust f64::round, what DataFusion's round uses)
            return Column(T.FLOAT64, torch.sign(x) * torch.floor(x.abs() + 0.5) / f, c.valid)
        if name == "coalesce":
            return self._coalesce(e, args, b)
        if name == "concat":
            dev = self.device(b)
            l, r = [self._str_col(a, dev) if isinstance(a, Scalar) else a for a in args]
            return S.concat(l, r, b.num_rows)
        if name in ("sqrt", "ln", "log10", "exp", "floor", "ceil"):
            c = args[0]
            x = _convert_tensor(c, T.FLOAT64)
            fn = {"sqrt": torch.sqrt, "ln": torch.log, "log10": torch.log10, "exp": torch.exp, "floor": torch.floor,
                  "ceil": torch.ceil}[name]
            return Column(T.FLOAT64, fn(x), c.valid)
        if name == "power":
            a, va = self._num(args[0], T.FLOAT64)
            c, vc = self._num(args[1], T.FLOAT64)
            return self._mk(torch.pow(a, c) if isinstance(a, torch.Tensor) else torch.pow(torch.as_tensor(a), c), T.FLOAT64, _and_valid(va, vc), b)
        raise NotSupported(f"function {name}")

    def _nested(self, e: Func, args, b: Batch) -> Value:
        from ..ops import nested as NS
        name = e.name
        n = b.num_rows
        dev = self.device(b)

        def col(i):
            a = args[i]
            if isinstance(a, Scalar):
                return Column.full(a.value, e.args[i].dtype if a.dtype.kind == "null" else a.dtype, n, dev)
            return a
        if name == "make_array":
            return NS.make_list([col(i) for i in range(len(args))], n, e.dtype, dev)
        if name == "struct":
            return NS.make_struct(list(e.options), [col(i) for i in range(len(args))], n, e.dtype, dev)
        if name == "array_length":
            c = col(0)
            return Column(T.INT64, NS.lengths(c).clone(), c.valid)
        if name == "array_element":
            c = col(0)
            if len(args) > 1:
                p = col(1)
                return NS.element(c, p.data, p.valid)
            return NS.element(c, e.options[0])
        if name == "get_field":
            return NS.field(col(0), e.options[0])
        if name == "array_has":
            return NS.has(col(0), e.options[0])
        if name == "array_to_string":
            c = col(0)
            return NS.to_string(c, *e.options)
        if name == "regexp_match":
            import pyarrow.compute as pc
            c = col(0)
            pat, flags = e.options
            rx = re.compile(pat, re.I if "i" in flags else 0)
            vals = []
            for v in c.to_arrow().to_pylist():
                m = rx.search(v) if v is not None else None
                vals.append(None if m is None else (list(m.groups()) if rx.groups else [m.group(0)]))
            from ..ops._lib import HOST_STEPS
            HOST_STEPS["regexp_match"] += 1
            return Column.from_arrow(pa.array(vals, pa.list_(pa.large_string())), device=dev, dtype=e.dtype)
        if name == "unnest":
            raise ExecutionError("unnest() is only valid as a SELECT list item or in FROM")
        raise NotSupported(f"function {name}")

    def _func_scalar(self, e: Func, args) -> Scalar:
        vals = [a.value for a in args]
        name = e.name
        if name == "make_array":
            return Scalar(list(vals), e.dtype)
        if name == "struct":
            return Scalar(dict(zip(e.options, vals)), e.dtype)
        if any(v is None for v in vals):
            return Scalar(None, e.dtype)
        if name == "upper":
            return Scalar(vals[0].upper(), T.UTF8)
        if name == "lower":
            return Scalar(vals[0].lower(), T.UTF8)
        if name == "substr":
            return Scalar(S._py_substr(vals[0], *e.options), T.UTF8)
        if name == "char_length":
            return Scalar(len(vals[0]), T.INT32)
        if name == "date_part":
            from ..sql.binder import _date_part_py
            return Scalar(_date_part_py(vals[0], e.options[0]), T.INT32)
        if name == "abs":
            return Scalar(abs(vals[0]), e.dtype)
        if name == "concat":
            return Scalar(str(vals[0]) + str(vals[1]), T.UTF8)
        if name == "round":
            if e.dtype.is_decimal:
                s = args[0].dtype.scale
                drop = s - e.dtype.scale
                f = 10**drop
                q = (abs(vals[0]) + f // 2) // f
                return Scalar(q if vals[0] >= 0 else -q, e.dtype)
            return Scalar(round(float(vals[0]), e.options[0]), e.dtype)
        if name in ("sqrt", "ln", "log10", "exp", "floor", "ceil", "power"):
            f = {"sqrt": math.sqrt, "ln": math.log, "log10": math.log10, "exp": math.exp, "floor": math.floor,
                 "ceil": math.ceil, "power": math.pow}[name]
            return Scalar(float(f(*[float(v) for v in vals])), T.FLOAT64)
        # everything else: the column path over a one-row batch
        dev = torch.device(self.ctx.device if self.ctx is not None else "cpu")
        cols = {i: Column.full(v, a.dtype, 1, dev) for i, (v, a) in enumerate(zip(vals, args))}
        from ..sql.expr import ColRef as _CR
        e1 = Func(e.name, [_CR(i, f"a{i}", a.dtype) for i, a in enumerate(args)], e.dtype, e.options)
        r = self._Func(e1, Batch(cols, 1))
        if isinstance(r, Scalar):
            return r
        return Scalar(_host_value(r, e.dtype), e.dtype)

    def _extreme(self, e: Func, args, b: Batch) -> Value:
        """greatest / least: the largest / smallest non-NULL argument."""
        n = b.num_rows
        dev = self.device(b)
        t = e.dtype
        out, valid = None, None
        for a in args:
            x, xv = _full_of(a, t, n, dev)
            ok = xv if xv is not None else torch.ones(n, dtype=torch.bool, device=dev)
            if out is None:
                out, valid = x, ok
                continue
            better = (x > out) if e.name == "greatest" else (x < out)
            take_x = ok & (~valid | better)
            out = torch.where(take_x, x, out)
            valid = valid | ok
        return Column(t, out, None if bool(valid.all()) and not valid.is_cuda else valid)

    def _coalesce(self, e: Func, args, b: Batch) -> Value:
        n = b.num_rows
        dev = self.device(b)
        t = e.dtype
        if t.is_string:
            # first non-NULL argument per row, assembled by one device gather
            choice = torch.full((n,), len(args) - 1, dtype=torch.int64, device=dev)
            for k in range(len(args) - 2, -1, -1):
                a = args[k]
                if isinstance(a, Scalar):
                    if a.value is not None:
                        choice = torch.full_like(choice, k)
                    continue
                ok = a.valid if a.valid is not None else torch.ones(n, dtype=torch.bool, device=dev)
                choice = torch.where(ok, torch.full_like(choice, k), choice)
            return S.select_rows([self._str_col(a, dev) for a in args], choice, n)
        out, valid = _full_of(args[-1], t, n, dev)
        for a in reversed(args[:-1]):
            x, xv = _full_of(a, t, n, dev)
            if xv is None:
                out, valid = x, None
                continue
            out = torch.where(xv, x, out)
            valid = xv | valid if valid is not None else None
        return Column(t, out, valid)


_STRFN = ("trim", "replace", "lpad", "rpad", "reverse", "repeat", "left", "right", "initcap", "translate",
          "split_part")
_MATH1 = ("sign", "trunc", "log2", "cbrt", "degrees", "radians", "sin", "cos", "tan", "asin", "acos", "atan", "sinh",
          "cosh", "tanh", "isnan", "iszero", "factorial")
_US_DAY = 86_400_000_000


def _math1(name: str, x: torch.Tensor, options) -> torch.Tensor:
    if name == "sign":
        return torch.sign(x)
    if name == "trunc":
        d = options[0] if options else 0
        f = 10.0 ** d
        return torch.trunc(x * f) / f
    if name == "log2":
        return torch.log2(x)
    if name == "cbrt":
        return torch.sign(x) * x.abs().pow(1.0 / 3.0)
    if name == "degrees":
        return torch.rad2deg(x)
    if name == "radians":
        return torch.deg2rad(x)
    if name == "isnan":
        return torch.isnan(x)
    if name == "iszero":
        return x == 0
    if name == "factorial":
        lut = torch.tensor([math.factorial(i) for i in range(21)], dtype=torch.int64, device=x.device)
        return lut.index_select(0, x.clamp(0, 20))
    return getattr(torch, name)(x)


def civil_from_days(days: torch.Tensor):
    """(year, month, day) int64 tensors from days since 1970-01-01 (Hinnant)."""
    z = days.to(torch.int64) + 719468
    era = torch.div(z, 146097, rounding_mode="floor")
    doe = z - era * 146097
    yoe = torch.div(doe - torch.div(doe, 1460, rounding_mode="floor") + torch.div(doe, 36524, rounding_mode="floor")
                    - torch.div(doe, 146096, rounding_mode="floor"), 365, rounding_mode="floor")
    doy = doe - (365 * yoe + torch.div(yoe, 4, rounding_mode="floor") - torch.div(yoe, 100, rounding_mode="floor"))
    mp = torch.div(5 * doy + 2, 153, rounding_mode="floor")
    d = doy - torch.div(153 * mp + 2, 5, rounding_mode="floor") + 1
    m = torch.where(mp < 10, mp + 3, mp - 9)
    y = yoe + era * 400 + (m <= 2).to(torch.int64)
    return y, m, d


def days_from_civil(y: torch.Tensor, m: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    yy = y - (m <= 2).to(torch.int64)
    era = torch.div(yy, 400, rounding_mode="floor")
    yoe = yy - era * 400
    doy = torch.div(153 * torch.where(m > 2, m - 3, m + 9) + 2, 5, rounding_mode="floor") + d - 1
    doe = yoe * 365 + torch.div(yoe, 4, rounding_mode="floor") - torch.div(yoe, 100, rounding_mode="floor") + doy
    return era * 146097 + doe - 719468


def iso_week(days: torch.Tensor) -> torch.Tensor:
    wd = torch.remainder(days + 3, 7)            # Monday = 0 (1970-01-01 was a Thursday)
    thu = days - wd + 3
    y, _, _ = civil_from_days(thu)
    jan1 = days_from_civil(y, torch.ones_like(y), torch.ones_like(y))
    return torch.div(thu - jan1, 7, rounding_mode="floor") + 1


def trunc_ts(us: torch.Tensor, unit: str) -> torch.Tensor:
    """date_trunc over timestamps (microseconds since the epoch)."""
    step = {"microsecond": 1, "millisecond": 1000, "second": 1_000_000, "minute": 60_000_000,
            "hour": 3_600_000_000, "day": _US_DAY}.get(unit)
    if step is not None:
        return torch.div(us, step, rounding_mode="floor") * step
    days = torch.div(us, _US_DAY, rounding_mode="floor")
    if unit == "week":
        return (days - torch.remainder(days + 3, 7)) * _US_DAY
    y, m, _ = civil_from_days(days)
    if unit == "quarter":
        m = torch.div(m - 1, 3, rounding_mode="floor") * 3 + 1
    elif unit == "year":
        m = torch.ones_like(m)
    return days_from_civil(y, m, torch.ones_like(m)) * _US_DAY


def ts_add(us: torch.Tensor, months: int, days: int, micros: int) -> torch.Tensor:
    d = torch.div(us, _US_DAY, rounding_mode="floor")
    rem = us - d * _US_DAY
    if months:
        d = add_months(d, months).to(torch.int64)
    return (d + days) * _US_DAY + rem + micros


def ts_part(us: torch.Tensor, field: str) -> torch.Tensor:
    if field == "epoch":
        return us.to(torch.float64) / 1e6
    days = torch.div(us, _US_DAY, rounding_mode="floor")
    rem = us - days * _US_DAY
    if field == "hour":
        return torch.div(rem, 3_600_000_000, rounding_mode="floor")
    if field == "minute":
        return torch.remainder(torch.div(rem, 60_000_000, rounding_mode="floor"), 60)
    if field == "second":
        return torch.remainder(torch.div(rem, 1_000_000, rounding_mode="floor"), 60)
    if field == "millisecond":
        return torch.remainder(torch.div(rem, 1000, rounding_mode="floor"), 60_000)
    if field == "microsecond":
        return torch.remainder(rem, 60_000_000)
    if field == "week":
        return iso_week(days)
    if field in ("dow", "doy", "quarter"):
        y, m, d = civil_from_days(days)
        if field == "dow":
            return torch.remainder(days + 4, 7)
        if field == "quarter":
            return torch.div(m - 1, 3, rounding_mode="floor") + 1
        return days - days_from_civil(y, torch.ones_like(y), torch.ones_like(y)) + 1
    y, m, d = civil_from_days(days)
    return {"year": y, "month": m, "day": d}[field]


def trunc_ts_py(us: int, unit: str) -> int:
    return int(trunc_ts(torch.tensor([us], dtype=torch.int64), unit)[0])


def ts_part_py(us: int, field: str):
    v = ts_part(torch.tensor([us], dtype=torch.int64), field)[0]
    return float(v) if field == "epoch" else int(v)


def _host_value(c: Column, t: DataType):
    """Engine representation of a one-row column's value (dates in days,
    timestamps in microseconds, decimals unscaled)."""
    if c.valid is not None and not bool(c.valid.cpu()[0]):
        return None
    if t.is_string:
        return c.to_arrow()[0].as_py()
    v = c.data.cpu()[0]
    if t.kind == "bool":
        return bool(v)
    if t.is_float:
        return float(v)
    return int(v)


def add_months(days: torch.Tensor, months: int, extra_days: int = 0) -> torch.Tensor:
    """date32 + INTERVAL 'n' MONTH (+ days) on the device: civil date from
    days (Hinnant), month arithmetic, day clamped to the target month's
    length (Jan 31 + 1 month = Feb 28/29), back to days — integer tensor ops,
    no host round trip."""
    z = days.to(torch.int64) + 719468
    era = torch.div(z, 146097, rounding_mode="floor")      # floor division: no negative-year adjustment
    doe = z - era * 146097
    yoe = torch.div(doe - torch.div(doe, 1460, rounding_mode="floor") + torch.div(doe, 36524, rounding_mode="floor")
                    - torch.div(doe, 146096, rounding_mode="floor"), 365, rounding_mode="floor")
    doy = doe - (365 * yoe + torch.div(yoe, 4, rounding_mode="floor") - torch.div(yoe, 100, rounding_mode="floor"))
    mp = torch.div(5 * doy + 2, 153, rounding_mode="floor")
    d = doy - torch.div(153 * mp + 2, 5, rounding_mode="floor") + 1
    m = torch.where(mp < 10, mp + 3, mp - 9)
    y = yoe + era * 400 + (m <= 2).to(torch.int64)
    k = y * 12 + (m - 1) + months
    y2 = torch.div(k, 12, rounding_mode="floor")
    m2 = k - y2 * 12 + 1
    leap = ((y2 % 4 == 0) & (y2 % 100 != 0)) | (y2 % 400 == 0)
    mdays = torch.tensor([31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31], dtype=torch.int64,
                         device=days.device).index_select(0, m2 - 1) + (leap & (m2 == 2)).to(torch.int64)
    d2 = torch.minimum(d, mdays)
    # days_from_civil
    yy = y2 - (m2 <= 2).to(torch.int64)
    era2 = torch.div(yy, 400, rounding_mode="floor")
    yoe2 = yy - era2 * 400
    doy2 = torch.div(153 * torch.where(m2 > 2, m2 - 3, m2 + 9) + 2, 5, rounding_mode="floor") + d2 - 1
    doe2 = yoe2 * 365 + torch.div(yoe2, 4, rounding_mode="floor") - torch.div(yoe2, 100, rounding_mode="floor") + doy2
    return (era2 * 146097 + doe2 - 719468 + extra_days).to(torch.int32)


# =============================================================== conversions
def _parse_ts_host(v: Column) -> Column:
    from ..ops.strings import note_host_step
    note_host_step("string -> timestamp")
    arr = v.to_arrow()
    try:
        ts = pc.cast(pc.strptime(arr, "%Y-%m-%dT%H:%M:%S", "us", error_is_null=True), pa.timestamp("us"))
        miss = pc.and_(pc.is_null(ts), pc.is_valid(arr))
        if pc.any(miss).as_py():
            ts = pc.cast(arr, pa.timestamp("us"))
    except (pa.ArrowInvalid, pa.ArrowNotImplementedError) as e:
        raise ExecutionError(f"cannot parse timestamp: {e}") from None
    out = Column.from_arrow(ts, device=v.device)
    return Column(T.TIMESTAMP, out.data.to(torch.int64), out.valid)


def _convert_scalar(x, src: DataType, t: DataType):
    if t.is_decimal:
        if src.is_decimal:
            d = t.scale - src.scale
            return x * 10**d if d >= 0 else int(round(x / 10**(-d)))
        if src.is_float:
            return int(round(x * 10**t.scale))
        return int(x) * 10**t.scale
    if t.is_float:
        if src.is_decimal:
            return x / 10**src.scale
        return float(x)
    if t.kind == "bool":
        return bool(x)
    if src.is_decimal and t.is_integer:
        return int(x // 10**src.scale)
    return x


def _convert_tensor(c: Column, t: DataType) -> torch.Tensor:
    src = c.dtype
    x = c.data
    if c.is_wide:
        if t.is_float:
            lo = x[:, 0].to(torch.float64)
            hi = x[:, 1].to(torch.float64)
            lo = torch.where(lo < 0, lo + 18446744073709551616.0, lo)
            v = hi * 18446744073709551616.0 + lo
            return v / 10**src.scale if src.is_decimal else v
        raise ExecutionError("128-bit decimal value used in integer arithmetic (value exceeds 64 bits)")
    if t.is_decimal:
        if src.is_decimal:
            d = t.scale - src.scale
            if d == 0:
                return x
            if d > 0:
                return x * (10**d)
            f = 10**(-d)
            return torch.div(x + torch.sign(x) * (f // 2), f, rounding_mode="trunc")
        if src.is_float:
            return torch.round(x * 10**t.scale).to(torch.int64)
        return x.to(torch.int64) * (10**t.scale)
    if t.is_float:
        if src.is_decimal:
            return x.to(torch.float64) / (10**src.scale)
        return x.to(torch.float64)
    if t.is_integer or t.kind in ("date32", "timestamp"):
        if src.is_decimal:
            return torch.div(x, 10**src.scale, rounding_mode="trunc").to(torch.int64)
        if src.is_float:
            return x.to(torch.int64)
        if src.kind == "bool":
            return x.to(torch.int64)
        return x if x.dtype == t.torch_dtype or t.kind == "int64" and x.dtype in (torch.int32, torch.int64) else x.to(t.torch_dtype)
    return x


def _overflow_guard(a, c):
    """Decimal product whose static precision exceeds 18 digits: verify at run time
    that the int64 product cannot overflow (raises otherwise)."""
    ts = [v for v in (a, c) if isinstance(v, torch.Tensor) and v.numel()]
    dev_max = iter(to_host_ints(torch.stack([v.abs().max().to(torch.int64) for v in ts])) if ts else [])  # one sync

    def mx(v):
        if isinstance(v, torch.Tensor):
            return int(next(dev_max)) if v.numel() else 0
        return abs(int(v))
    if mx(a) * mx(c) >= 2**63:
        raise ExecutionError("decimal multiplication overflows 64-bit fixed point; CAST to DOUBLE")
    return a, c


def _any(m: torch.Tensor) -> bool:
    return bool(to_host_ints(m.any().to(torch.int64))[0]) if m.is_cuda else bool(m.any())


def _bool_parts(v: Column):
    d = v.data if v.data.dtype == torch.bool else v.data != 0
    return d, v.valid


def _full_of(v: Value, t: DataType, n: int, dev):
    if isinstance(v, Scalar):
        if v.value is None:
            td = t.torch_dtype if t.kind != "null" else torch.bool
            return torch.zeros(n, dtype=td, device=dev), torch.zeros(n, dtype=torch.bool, device=dev)
        val = _convert_scalar(v.value, v.dtype, t)
        return torch.full((n,), val, dtype=t.torch_dtype if t.kind != "null" else torch.bool, device=dev), None
    x = _convert_tensor(v, t) if v.dtype != t else v.data
    return x.to(t.torch_dtype) if t.kind != "null" else x, v.valid


def _concat_strings(a: Column, b: Column) -> Column:
    na, nb = len(a), len(b)
    off = torch.cat([a.offsets, b.offsets[1:] + a.offsets[-1]])
    chars = torch.cat([a.data, b.data])
    valid = None
    if a.valid is not None or b.valid is not None:
        va = a.valid if a.valid is not None else torch.ones(na, dtype=torch.bool, device=a.device)
        vb = b.valid if b.valid is not None else torch.ones(nb, dtype=torch.bool, device=b.device)
        valid = torch.cat([va, vb])
    return Column(T.UTF8, chars, valid, offsets=off)
