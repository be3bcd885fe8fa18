"""Code generator for the fused scan kernels: one HIP kernel per scan shape.

Input is the same description ``exec/fused.py`` hands the interpreted
kernels (csrc/kernels/fused.hip): integer columns of 1/2/4/8 bytes, filter
terms (ranges, NOT ranges, dictionary-code sets, column-column ranges, one OR
of conjunctions, an optional precomputed mask), up to two small-domain group
keys and SUM / MIN / MAX of products of affine factors. The generated kernel
has all of it as compile-time constants:

* each thread owns ROWS (4) consecutive rows per iteration and loads each
  column as ONE vector of its exact width (char4 / short4 / int4 / 2 x int4),
  widened to int32 when the width allows;
* filter terms are straight-line compares against literal bounds (a bound
  outside the column's width disappears), the OR of conjunctions is a boolean
  expression, group ids are constant multiply-adds;
* factor arithmetic is typed from static bounds: int32 while |value| < 2^31,
  int64 products (v_mad_i64_i32) after, an overflow check only where the
  bound reaches 2^63 and the SQL type asks for one; shared product prefixes
  are computed once;
* one group: per-thread register accumulators, a wave shuffle reduction and
  one int128 atomic per block and aggregate; 2..16 groups: the interpreted
  kernel's LDS slot scheme (per-lane int64 slots shared by the block's waves)
  with only the halves a value's bound needs;
* SUMs are exact: a sum whose bound could pass 2^63 inside a block is kept as
  unsigned-low / signed-high 32-bit halves and recombined in int128.

The interpreted kernels remain the fallback (and serve the first executions
while hiprtc compiles in the background, see ``ops/jit.py``). Semantics are
identical; tests run both against the CPU engine.
"""
from __future__ import annotations

from ..utils import switches as _sw
import math
import os
from typing import List, Optional, Sequence, Tuple

import torch

from ..ops import jit

I64_MIN, I64_MAX = -(2**63), 2**63 - 1
ENABLED = os.environ.get("IGLOO_JIT", "async").lower() != "off"

_CT = {1: "i8", 2: "i16", 4: "i32", 8: "i64"}
_VT = {1: "i8xR", 2: "i16xR", 4: "i32xR", 8: "i64xR"}

PRELUDE = r"""
typedef signed char i8; typedef short i16; typedef int i32; typedef long long i64;
typedef unsigned char u8; typedef unsigned int u32; typedef unsigned long long u64;
typedef i8 i8xR __attribute__((ext_vector_type(ROWS)));
typedef i16 i16xR __attribute__((ext_vector_type(ROWS)));
typedef i32 i32xR __attribute__((ext_vector_type(ROWS)));
typedef i64 i64xR __attribute__((ext_vector_type(ROWS)));
typedef u8 u8xR __attribute__((ext_vector_type(ROWS)));
#define WG_ADD(p, v) __hip_atomic_fetch_add((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define WG_MIN(p, v) __hip_atomic_fetch_min((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define WG_MAX(p, v) __hip_atomic_fetch_max((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
__device__ __forceinline__ void add128(i64* lo, i64* hi, __int128 v) {
  if (v == 0) return;
  const u64 vl = (u64)v;
  const u64 vh = (u64)(i64)(v >> 64);
  const u64 old = atomicAdd((unsigned long long*)lo, (unsigned long long)vl);
  const u64 carry = (old + vl) < old ? 1ull : 0ull;
  if (vh + carry) atomicAdd((unsigned long long*)hi, (unsigned long long)(vh + carry));
}
__device__ __forceinline__ i64 wsum(i64 v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ i64 wmin(i64 v) {
  for (int o = 32; o > 0; o >>= 1) { const i64 u = __shfl_xor(v, o, 64); v = u < v ? u : v; }
  return v;
}
__device__ __forceinline__ i64 wmax(i64 v) {
  for (int o = 32; o > 0; o >>= 1) { const i64 u = __shfl_xor(v, o, 64); v = u > v ? u : v; }
  return v;
}
"""

BLOCK = 256
# consecutive rows per thread per iteration (one vector load per column)
ROWS = 4
LDS_MAX = 64 * 1024


def _lit(v: int) -> str:
    v = int(v)
    if v == I64_MIN:
        return "(-9223372036854775807LL - 1)"
    return f"{v}LL"


class _Shape:
    """Column widths + typed variable names of one launch."""

    def __init__(self, cols: Sequence[torch.Tensor]):
        self.w = [int(t.element_size()) for t in cols]

    def rng(self, c: int) -> Tuple[int, int]:
        b = 8 * self.w[c] - 1
        return -(1 << b), (1 << b) - 1

    def typ(self, c: int) -> str:
        return "i64" if self.w[c] == 8 else "i32"


def _terms_expr(sh: _Shape, terms, j: int) -> str:
    """Boolean expression of every filter term for row j (AND of top-level
    terms, AND of the OR over conjunction groups). The terms' constants are
    kernel arguments (``_term_args``), not literals: the source depends only
    on the predicate's shape, so a query with other parameter values (a TPC-H
    substitution, an ad-hoc date range) reuses the compiled kernel."""
    top: List[str] = []
    groups: dict = {}
    for t, (col, kindg, lo, hi, bits) in enumerate(terms):
        kind, grp = kindg & 0xFF, kindg >> 8
        x = f"x{col}_{j}"
        mn, mx = sh.rng(col)
        if kind in (0, 1):
            parts = []
            if lo > mn or lo > hi:
                parts.append(f"{x} >= f{t}lo")
            if hi < mx or lo > hi:
                parts.append(f"{x} <= f{t}hi")
            e = "(" + " && ".join(parts) + ")" if parts else "true"
            if kind == 1:
                e = f"!{e}"
        elif kind == 2:
            e = f"((u64){x} < 64ull && ((f{t}bits >> (u32){x}) & 1ull))"
        elif kind == 3:
            c2 = bits & 0xFF
            d = f"((i64){x} - (i64)x{c2}_{j})"
            e = f"({d} >= f{t}lo && {d} <= f{t}hi)"
        else:
            raise ValueError(f"term kind {kind}")
        (groups.setdefault(grp, []) if grp else top).append(e)
    if groups:
        top.append("(" + " || ".join("(" + " && ".join(g) + ")" for _, g in sorted(groups.items())) + ")")
    return " && ".join(top) if top else "true"


def _term_params(terms) -> List[str]:
    """Kernel parameters carrying the filter terms' constants (appended
    after every other parameter)."""
    ps = []
    for t, (col, kindg, lo, hi, bits) in enumerate(terms):
        if kindg & 0xFF == 2:
            ps.append(f"u64 f{t}bits")
        else:
            ps += [f"i64 f{t}lo", f"i64 f{t}hi"]
    return ps


def _term_args(terms) -> List[int]:
    out = []
    for col, kindg, lo, hi, bits in terms:
        if kindg & 0xFF == 2:
            out.append(int(bits) & 0xFFFFFFFFFFFFFFFF)
        else:
            out += [int(lo), int(hi)]
    return out


class _Values:
    """Typed product chains for the aggregate arguments of one row, with
    shared prefixes computed once. Emits C statements; tracks |value| bounds."""

    def __init__(self, sh: _Shape, j: int):
        self.sh, self.j = sh, j
        self.lines: List[str] = []
        self.memo = {}
        self.n = 0
        self.checked_any = False

    def factor(self, c: int, a: int, b: int) -> Tuple[str, int, bool]:
        if c < 0:
            return _lit(a), abs(a), abs(a) < 2**31
        x = f"x{c}_{self.j}"
        mn, mx = self.sh.rng(c)
        bound = abs(a) + abs(b) * max(-mn, mx)
        if bound < 2**31:
            if b == 1:
                e = f"({a} + {x})" if a else x
            elif b == -1:
                e = f"({a} - {x})"
            else:
                e = f"({a} + {b} * {x})" if a else f"({b} * {x})"
            return e, bound, True
        # 64-bit, wrapping like the interpreted kernel (the checked product
        # below catches what the SQL type cannot hold)
        return f"(i64)((u64){_lit(a)} + (u64){_lit(b)} * (u64)(i64){x})", bound, False

    def value(self, fs: Tuple[Tuple[int, int, int], ...], checked: bool) -> Tuple[str, int]:
        key = (tuple(fs), checked)
        if key in self.memo:
            return self.memo[key]
        if len(fs) == 1:
            e, bnd, small = self.factor(*fs[0])
            name = f"v{self.n}_{self.j}"
            self.n += 1
            self.lines.append(f"const {'i32' if small else 'i64'} {name} = {e};")
            self.memo[key] = (name, bnd)
            return name, bnd
        pv, pb = self.value(fs[:-1], checked)
        fe, fb, fsmall = self.factor(*fs[-1])
        name = f"v{self.n}_{self.j}"
        self.n += 1
        nb = pb * fb
        if nb < 2**31:
            self.lines.append(f"const i32 {name} = {pv} * {fe};")
        elif nb < 2**63:
            self.lines.append(f"const i64 {name} = (i64){pv} * (i64){fe};")
        elif checked:
            self.checked_any = True
            self.lines.append(f"i64 {name}; of |= __builtin_mul_overflow((i64){pv}, (i64){fe}, &{name});")
            nb = 2**63
        else:
            self.lines.append(f"const i64 {name} = (i64)((u64)(i64){pv} * (u64)(i64){fe});")
            nb = 2**63
        self.memo[key] = (name, nb)
        return name, nb


def _loads(sh: _Shape, has_mask: bool) -> List[str]:
    L = []
    nc = len(sh.w)
    for c in range(nc):
        for j in range(ROWS):
            L.append(f"{sh.typ(c)} x{c}_{j};")
    for j in range(ROWS):
        L.append(f"bool lv{j};")
        if has_mask:
            L.append(f"bool mk{j};")
    L.append(f"if (r + {ROWS} <= n) {{")
    for c in range(nc):
        L.append(f"  const {_VT[sh.w[c]]} q{c} = *(const {_VT[sh.w[c]]}*)(c{c} + r);")
    if has_mask:
        L.append("  const u8xR mq = *(const u8xR*)(mk + r);")
    for j in range(ROWS):
        for c in range(nc):
            L.append(f"  x{c}_{j} = q{c}[{j}];")
        L.append(f"  lv{j} = true;")
        if has_mask:
            L.append(f"  mk{j} = mq[{j}] != 0;")
    L.append("} else {")
    for j in range(ROWS):
        L.append(f"  lv{j} = r + {j} < n;")
        for c in range(nc):
            L.append(f"  x{c}_{j} = lv{j} ? ({sh.typ(c)})c{c}[r + {j}] : 0;")
        if has_mask:
            L.append(f"  mk{j} = lv{j} && mk[r + {j}] != 0;")
    L.append("}")
    return L


def _params(sh: _Shape, has_mask: bool) -> List[str]:
    ps = [f"const {_CT[w]}* __restrict__ c{c}" for c, w in enumerate(sh.w)]
    if has_mask:
        ps.append("const u8* __restrict__ mk")
    return ps


def _aligned(cols: Sequence[torch.Tensor]) -> bool:
    return all(t.data_ptr() % min(4 * t.element_size(), 16) == 0 and t.is_contiguous() for t in cols)


# ------------------------------------------------------------------ mask
#: rows per select tile (csrc/kernels/select.hip kTile): a tiled mask kernel
#: writes each tile's set-row count with the mask, so the selection that
#: follows skips its count pass over the mask (ops/select.py tile_counts)
SELECT_TILE = 8192
TILE_COUNTS = not _sw.debug("no_mask_counts")


def mask_source(sh: _Shape, terms, has_mask: bool, tiled: bool = False) -> str:
    L = [f"#define ROWS {ROWS}", PRELUDE, f"extern \"C\" __global__ __launch_bounds__({BLOCK}) void igloo_jit_scan_mask("]
    L.append("    " + ", ".join(_params(sh, has_mask) + ["u8* __restrict__ out", "i64 n"]
                            + (["i64* __restrict__ tc"] if tiled else []) + _term_params(terms)) + ") {")
    body = ["    " + s for s in _loads(sh, has_mask)]
    for j in range(ROWS):
        p = f"lv{j} && " + _terms_expr(sh, terms, j) + (f" && mk{j}" if has_mask else "")
        body.append(f"    const bool p{j} = {p};")
    body.append(f"    if (r + {ROWS} <= n) *(u8xR*)(out + r) = u8xR{{" + ", ".join(f"(u8)p{j}" for j in range(ROWS)) + "};")
    body.append("    else { " + " ".join(f"if (lv{j}) out[r + {j}] = p{j};" for j in range(ROWS)) + " }")
    if not tiled:
        L.append(f"  const i64 step = (i64)gridDim.x * {BLOCK * ROWS};")
        L.append(f"  for (i64 r = ((i64)blockIdx.x * {BLOCK} + threadIdx.x) * {ROWS}; r < n; r += step) {{")
        L += body
        L.append("  }")
    else:
        # one workgroup per select tile at a time: the tile's rows in
        # {SELECT_TILE // (BLOCK * ROWS)} block-wide steps, its set rows summed
        # in registers, reduced over the block and stored (no atomics)
        per = SELECT_TILE // (BLOCK * ROWS)
        L.append(f"  __shared__ i32 red[{BLOCK // 64}];")
        L.append(f"  const i64 ntiles = (n + {SELECT_TILE - 1}) / {SELECT_TILE};")
        L.append("  for (i64 t = blockIdx.x; t < ntiles; t += gridDim.x) {")
        L.append("    i32 cnt = 0;")
        L.append(f"    for (int it = 0; it < {per}; ++it) {{")
        L.append(f"    const i64 r = t * {SELECT_TILE} + it * {BLOCK * ROWS} + threadIdx.x * {ROWS};")
        L.append("    if (r >= n) break;")
        L += body
        L.append("    cnt += " + " + ".join(f"(i32)p{j}" for j in range(ROWS)) + ";")
        L.append("    }")
        L.append("    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);")
        L.append("    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;")
        L.append("    __syncthreads();")
        L.append("    if (threadIdx.x == 0) tc[t] = " + " + ".join(f"(i64)red[{w}]" for w in range(BLOCK // 64)) + ";")
        L.append("    __syncthreads();")
        L.append("  }")
    L.append("}")
    return "\n".join(L)


def jit_mask(spec, n: int, out: torch.Tensor, stream: int, tc: Optional[torch.Tensor] = None) -> bool:
    """``tc``: int64 [tiles + 1] to receive the mask's per-select-tile counts
    (the tiled kernel); None: the plain mask kernel."""
    if not (ENABLED and jit.enabled()) or n == 0 or not _aligned(spec.cols):
        return False
    has_mask = spec.mask is not None
    if has_mask and spec.mask.data_ptr() % 4:
        return False
    sh = _Shape(spec.cols)
    k = jit.get(mask_source(sh, spec.terms, has_mask, tc is not None), "igloo_jit_scan_mask")
    if k is None:
        return False
    args = [t.data_ptr() for t in spec.cols] + ([spec.mask.data_ptr()] if has_mask else []) + [out.data_ptr(), n]
    if tc is not None:
        grid = max(1, min(-(-n // SELECT_TILE), 256 * 16))
        args.append(tc.data_ptr())
    else:
        grid = max(1, min(-(-n // (BLOCK * ROWS)), 256 * 16))
    k.launch(grid, BLOCK, 0, stream, args + _term_args(spec.terms))
    return True


# ------------------------------------------------------------- aggregate
def agg_source(sh: _Shape, terms, has_mask: bool, keys, G: int, aggs, split: Sequence[bool], lanes: int) -> str:
    """aggs: [(op, checked, factors)] with op 0 sum / 2 min / 3 max."""
    NA = len(aggs)
    # LDS slot index per (aggregate, half); the row count is the last slot
    slot = []
    ns = 0
    for i, (op, _, _) in enumerate(aggs):
        h = 2 if (op == 0 and split[i]) else 1
        slot.append(list(range(ns, ns + h)))
        ns += h
    cnt_slot = ns
    nslots = ns + 1
    L = [f"#define ROWS {ROWS}", PRELUDE, f"extern \"C\" __global__ __launch_bounds__({BLOCK}) void igloo_jit_scan_agg("]
    ps = _params(sh, has_mask) + ["i64* __restrict__ counts"]
    for i in range(NA):
        ps += [f"i64* __restrict__ d{i}", f"i64* __restrict__ e{i}"]
    ps += ["int* __restrict__ ovf", "i64 n"] + _term_params(terms)
    L.append("    " + ", ".join(ps) + ") {")
    L.append("  int of = 0;")
    if G == 1:
        L.append("  i64 cn = 0;")
        for i, (op, _, _) in enumerate(aggs):
            init = {0: "0", 2: _lit(I64_MAX), 3: _lit(I64_MIN)}[op]
            L.append(f"  i64 s{i} = {init};" + (f" i64 h{i} = 0;" if op == 0 and split[i] else ""))
    else:
        L.append(f"  __shared__ i64 lds[{nslots * G * lanes}];")
        L.append(f"  const int ln = threadIdx.x & {lanes - 1};")
        L.append(f"  for (int s = threadIdx.x; s < {nslots * G * lanes}; s += {BLOCK}) {{")
        L.append(f"    const int k = s / {G * lanes};")
        inits = []
        for i, (op, _, _) in enumerate(aggs):
            if op in (2, 3):
                inits.append(f"k == {slot[i][0]} ? {_lit(I64_MAX if op == 2 else I64_MIN)}")
        L.append("    lds[s] = " + (" : ".join(inits) + " : 0" if inits else "0") + ";")
        L.append("  }")
        L.append("  __syncthreads();")
    L.append(f"  const i64 step = (i64)gridDim.x * {BLOCK * ROWS};")
    L.append(f"  for (i64 r = ((i64)blockIdx.x * {BLOCK} + threadIdx.x) * {ROWS}; r < n; r += step) {{")
    L += ["    " + s for s in _loads(sh, has_mask)]
    for j in range(ROWS):
        p = f"lv{j} && " + _terms_expr(sh, terms, j) + (f" && mk{j}" if has_mask else "")
        L.append(f"    const bool p{j} = {p};")
        V = _Values(sh, j)
        vals = [V.value(tuple(fs), bool(chk)) for _, chk, fs in aggs]
        body = list(V.lines)
        if G == 1:
            body.append("cn += 1;")
            for i, (op, _, _) in enumerate(aggs):
                v, _ = vals[i]
                if op == 0:
                    if split[i]:
                        body.append(f"s{i} += (i64)(u32)(u64)(i64){v}; h{i} += (i64){v} >> 32;")
                    else:
                        body.append(f"s{i} += (i64){v};")
                elif op == 2:
                    body.append(f"s{i} = (i64){v} < s{i} ? (i64){v} : s{i};")
                else:
                    body.append(f"s{i} = (i64){v} > s{i} ? (i64){v} : s{i};")
        else:
            g = " + ".join(f"(i32)(x{k}_{j} - {_lit(lo)}) * {mul}" if lo else f"(i32)x{k}_{j} * {mul}"
                           for k, lo, mul in keys) or "0"
            body.append(f"const int b_ = ({g}) * {lanes} + ln;")
            body.append(f"WG_ADD(&lds[{cnt_slot * G * lanes} + b_], (i64)1);")
            for i, (op, _, _) in enumerate(aggs):
                v, _ = vals[i]
                base = slot[i][0] * G * lanes
                if op == 0:
                    if split[i]:
                        body.append(f"WG_ADD(&lds[{base} + b_], (i64)(u32)(u64)(i64){v});")
                        body.append(f"WG_ADD(&lds[{slot[i][1] * G * lanes} + b_], (i64){v} >> 32);")
                    else:
                        body.append(f"WG_ADD(&lds[{base} + b_], (i64){v});")
                elif op == 2:
                    body.append(f"WG_MIN(&lds[{base} + b_], (i64){v});")
                else:
                    body.append(f"WG_MAX(&lds[{base} + b_], (i64){v});")
        L.append(f"    if (p{j}) {{")
        L += ["      " + s for s in body]
        L.append("    }")
    L.append("  }")
    # ---- epilogue
    if G == 1:
        accs = ["cn"] + [f"s{i}" for i in range(NA)] + [f"h{i}" for i in range(NA) if aggs[i][0] == 0 and split[i]]
        red = {a: "wsum" for a in accs}
        for i, (op, _, _) in enumerate(aggs):
            if op == 2:
                red[f"s{i}"] = "wmin"
            elif op == 3:
                red[f"s{i}"] = "wmax"
        L.append(f"  __shared__ i64 red[{BLOCK // 64}][{len(accs)}];")
        L.append("  const int w_ = threadIdx.x >> 6;")
        for ai, a in enumerate(accs):
            L.append(f"  {{ const i64 t_ = {red[a]}({a}); if ((threadIdx.x & 63) == 0) red[w_][{ai}] = t_; }}")
        L.append("  __syncthreads();")
        L.append("  if (threadIdx.x == 0) {")
        for ai, a in enumerate(accs):
            f = red[a]
            comb = {"wsum": "t_ += red[w][{ai}];", "wmin": "t_ = red[w][{ai}] < t_ ? red[w][{ai}] : t_;",
                    "wmax": "t_ = red[w][{ai}] > t_ ? red[w][{ai}] : t_;"}[f].format(ai=ai)
            L.append(f"    i64 {a}_b = red[0][{ai}]; {{ i64 t_ = {a}_b; for (int w = 1; w < {BLOCK // 64}; ++w) {comb} {a}_b = t_; }}")
        L.append("    if (cn_b) atomicAdd((unsigned long long*)counts, (unsigned long long)cn_b);")
        for i, (op, _, _) in enumerate(aggs):
            if op == 0:
                tot = f"(__int128)s{i}_b" + (f" + ((__int128)h{i}_b << 32)" if split[i] else "")
                L.append(f"    add128(d{i}, e{i}, {tot});")
            elif op == 2:
                L.append(f"    if (cn_b) atomicMin((long long*)d{i}, (long long)s{i}_b);")
            else:
                L.append(f"    if (cn_b) atomicMax((long long*)d{i}, (long long)s{i}_b);")
        L.append("  }")
    else:
        L.append("  __syncthreads();")
        L.append(f"  for (int s = threadIdx.x; s < {G * (NA + 1)}; s += {BLOCK}) {{")
        L.append(f"    const int g = s / {NA + 1}, o = s % {NA + 1};")
        L.append("    __int128 t = 0;")
        L.append(f"    if (o == {NA}) {{")
        L.append(f"      for (int l = 0; l < {lanes}; ++l) t += lds[{cnt_slot * G * lanes} + g * {lanes} + l];")
        L.append("      if (t) atomicAdd((unsigned long long*)&counts[g], (unsigned long long)(i64)t);")
        L.append("      continue;")
        L.append("    }")
        for i, (op, _, _) in enumerate(aggs):
            b0 = slot[i][0] * G * lanes
            L.append(f"    if (o == {i}) {{")
            if op == 0:
                L.append(f"      for (int l = 0; l < {lanes}; ++l) t += lds[{b0} + g * {lanes} + l];")
                if split[i]:
                    b1 = slot[i][1] * G * lanes
                    L.append(f"      __int128 u = 0; for (int l = 0; l < {lanes}; ++l) u += lds[{b1} + g * {lanes} + l];")
                    L.append("      t += u << 32;")
                L.append(f"      add128(&d{i}[g], &e{i}[g], t);")
            else:
                cmp = "<" if op == 2 else ">"
                L.append(f"      i64 m = lds[{b0} + g * {lanes}];")
                L.append(f"      for (int l = 1; l < {lanes}; ++l) {{ const i64 x = lds[{b0} + g * {lanes} + l]; m = x {cmp} m ? x : m; }}")
                fn = "atomicMin" if op == 2 else "atomicMax"
                L.append(f"      {fn}((long long*)&d{i}[g], (long long)m);")
            L.append("    }")
        L.append("  }")
    L.append("  if (of) atomicOr(ovf, 1);")
    L.append("}")
    return "\n".join(L)


# Off by default: SF100 kernel A/B (profiles/r2_ab_jit_mfma{0,1}_q1q6.txt) measured
# the generated MFMA aggregation at 1.45 ms for Q1 against 1.23 ms for the
# generated LDS-atomic kernel - the scan is bound by loads / filter / value
# arithmetic, not by the per-row accumulation the matrix cores take over.
MFMA = _sw.debug("ff_jit_mfma")
MFMA_COL = 272   # LDS bytes per limb column: 256 rows + 16 (spreads a ds_read_b128 over all banks)

MFMA_PRELUDE = r"""
typedef int v4i __attribute__((ext_vector_type(4)));
// byte b of each of x0..x3 packed into one dword (v_perm_b32 pairs + merge)
__device__ __forceinline__ u32 limb_dword(u32 x0, u32 x1, u32 x2, u32 x3, u32 b) {
  const u32 sel = b | ((b + 4) << 8);
  const u32 p01 = __builtin_amdgcn_perm(x1, x0, sel);
  const u32 p23 = __builtin_amdgcn_perm(x3, x2, sel);
  return __builtin_amdgcn_perm(p23, p01, 0x05040100u);
}
// 0x01 in each byte of x equal to the matching byte of g4
__device__ __forceinline__ u32 bytes_eq(u32 x, u32 g4) {
  const u32 d = x ^ g4;
  const u32 y = ~(((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d | 0x7f7f7f7fu);
  return y >> 7;
}
"""


def mfma_agg_source(sh: _Shape, terms, has_mask: bool, keys, G: int, aggs) -> Tuple[str, int]:
    """SUM / COUNT over 2..16 groups as one-hot x byte-limb products on the
    matrix cores (v_mfma_i32_16x16x64_i8), the generated-kernel form of
    csrc/kernels/fused.hip ff_mfma_agg_kernel (see its comment for the
    fragment maps and the biased lower limbs). Limb counts come from the
    static value bounds. Returns (source, LDS bytes per block)."""
    assert ROWS == 4 and 1 < G <= 16
    NA = len(aggs)
    lines: List[str] = []
    vals_per_row = []
    for j in range(ROWS):
        V = _Values(sh, j)
        vals_per_row.append([V.value(tuple(fs), bool(chk)) for _, chk, fs in aggs])
        lines.append(V.lines)
    col0, nlimb, col = [], [], 0
    for i in range(NA):
        bnd = max(v[i][1] for v in vals_per_row)
        nbits = min(64, max(1, int(bnd).bit_length()) + 1)
        nl = (nbits + 7) // 8
        col0.append(col)
        nlimb.append(nl)
        col += nl
    cnt_col = col
    ncols = col + 1
    NT = (ncols + 15) // 16
    if NT > 4:
        raise ValueError("too many limb columns")
    NC = NT * 16
    tile_bytes = (NC + 1) * MFMA_COL
    L = [f"#define ROWS {ROWS}", PRELUDE, MFMA_PRELUDE,
         f"extern \"C\" __global__ __launch_bounds__({BLOCK}) void igloo_jit_scan_agg_mfma("]
    ps = _params(sh, has_mask) + ["i64* __restrict__ counts"]
    for i in range(NA):
        ps += [f"i64* __restrict__ d{i}", f"i64* __restrict__ e{i}"]
    ps += ["int* __restrict__ ovf", "i64 n"] + _term_params(terms)
    L.append("    " + ", ".join(ps) + ") {")
    L.append(f"  __shared__ __attribute__((aligned(16))) u8 tile[{BLOCK // 64}][{tile_bytes}];")
    L.append("  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;")
    L.append("  u8* T = tile[wave];")
    L.append(f"  u8* gidb = T + {NC * MFMA_COL};")
    L.append(f"  for (int c = 0; c < {NC}; ++c) *(u32*)(T + c * {MFMA_COL} + 4 * lane) = c == {cnt_col} ? 0x01010101u : 0u;")
    L.append(f"  v4i acc[{NT}];")
    L.append(f"  i64 acc64[{NT}][4];")
    L.append(f"  for (int t = 0; t < {NT}; ++t) {{ acc[t] = v4i{{0, 0, 0, 0}}; for (int i = 0; i < 4; ++i) acc64[t][i] = 0; }}")
    L.append("  int of = 0, steps = 0;")
    L.append("  const u32 g4 = (u32)(lane & 15) * 0x01010101u;")
    L.append("  const int q16 = 16 * (lane >> 4);")
    L.append(f"  const i64 step = (i64)gridDim.x * {BLOCK * ROWS};")
    # wave-uniform loop: every lane of a wave runs every MFMA
    L.append(f"  for (i64 wbase = (i64)blockIdx.x * {BLOCK * ROWS} + (i64)wave * {64 * ROWS}; wbase < n; wbase += step) {{")
    L.append("    const i64 r = wbase + 4 * lane;")
    L += ["    " + x for x in _loads(sh, has_mask)]
    for j in range(ROWS):
        p = f"lv{j} && " + _terms_expr(sh, terms, j) + (f" && mk{j}" if has_mask else "")
        g = " + ".join(f"(i32)(x{k}_{j} - {_lit(lo)}) * {mul}" if lo else f"(i32)x{k}_{j} * {mul}"
                       for k, lo, mul in keys) or "0"
        L.append(f"    const bool p{j} = {p};")
        L.append(f"    const u32 g{j} = p{j} ? (u32)({g}) & 0xffu : 0xffu;")
        L += ["    " + x for x in lines[j]]
    L.append(f"    *(u32*)(gidb + 4 * lane) = g0 | (g1 << 8) | (g2 << 16) | (g3 << 24);")
    for i in range(NA):
        v = [vals_per_row[j][i][0] for j in range(ROWS)]
        L.append(f"    {{ const i64 a0 = (i64){v[0]}, a1 = (i64){v[1]}, a2 = (i64){v[2]}, a3 = (i64){v[3]};")
        for l in range(nlimb[i]):
            half = "" if l < 4 else " >> 32"
            xs = ", ".join(f"(u32)((u64)a{j}{half})" for j in range(ROWS))
            flip = " ^ 0x80808080u" if l != nlimb[i] - 1 else ""
            L.append(f"      *(u32*)(T + {(col0[i] + l) * MFMA_COL} + 4 * lane) = limb_dword({xs}, {l % 4}u){flip};")
        L.append("    }")
    L.append("    __builtin_amdgcn_wave_barrier();")
    L.append("#pragma unroll")
    L.append("    for (int s = 0; s < 4; ++s) {")
    L.append("      const uint4 gv = *(const uint4*)(gidb + 64 * s + q16);")
    L.append("      v4i af;")
    L.append("      af[0] = (int)bytes_eq(gv.x, g4); af[1] = (int)bytes_eq(gv.y, g4);")
    L.append("      af[2] = (int)bytes_eq(gv.z, g4); af[3] = (int)bytes_eq(gv.w, g4);")
    L.append("#pragma unroll")
    L.append(f"      for (int t = 0; t < {NT}; ++t) {{")
    L.append(f"        const uint4 bw = *(const uint4*)(T + (16 * t + (lane & 15)) * {MFMA_COL} + 64 * s + q16);")
    L.append("        const v4i bf = v4i{(int)bw.x, (int)bw.y, (int)bw.z, (int)bw.w};")
    L.append("        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, acc[t], 0, 0, 0);")
    L.append("      }")
    L.append("    }")
    L.append("    __builtin_amdgcn_wave_barrier();")
    L.append("    if (++steps == 4096) {")
    L.append(f"      steps = 0;")
    L.append(f"      for (int t = 0; t < {NT}; ++t) {{ for (int i = 0; i < 4; ++i) acc64[t][i] += acc[t][i]; acc[t] = v4i{{0, 0, 0, 0}}; }}")
    L.append("    }")
    L.append("  }")
    L.append(f"  for (int t = 0; t < {NT}; ++t) for (int i = 0; i < 4; ++i) acc64[t][i] += acc[t][i];")
    L.append("  __syncthreads();")
    L.append(f"  long long (*red)[{NC}][16] = reinterpret_cast<long long (*)[{NC}][16]>(&tile[0][0]);")
    L.append(f"  for (int t = 0; t < {NT}; ++t) for (int i = 0; i < 4; ++i) red[wave][16 * t + (lane & 15)][4 * (lane >> 4) + i] = acc64[t][i];")
    L.append("  __syncthreads();")
    L.append(f"  for (int s = threadIdx.x; s < {G * (NA + 1)}; s += {BLOCK}) {{")
    L.append(f"    const int g = s / {NA + 1}, o = s % {NA + 1};")
    L.append(f"    i64 cnt = 0; for (int w = 0; w < {BLOCK // 64}; ++w) cnt += red[w][{cnt_col}][g];")
    L.append(f"    if (o == {NA}) {{ if (cnt) atomicAdd((unsigned long long*)&counts[g], (unsigned long long)cnt); continue; }}")
    for i in range(NA):
        L.append(f"    if (o == {i}) {{")
        L.append("      __int128 tot = 0;")
        for l in range(nlimb[i]):
            bias = " + 128 * cnt" if l != nlimb[i] - 1 else ""
            L.append(f"      {{ i64 x = 0; for (int w = 0; w < {BLOCK // 64}; ++w) x += red[w][{col0[i] + l}][g];"
                     f" tot += (__int128)(x{bias}) << {8 * l}; }}")
        L.append(f"      add128(&d{i}[g], &e{i}[g], tot);")
        L.append("    }")
    L.append("  }")
    L.append("  if (of) atomicOr(ovf, 1);")
    L.append("}")
    return "\n".join(L), (BLOCK // 64) * tile_bytes


def jit_aggregate(spec, keys, G: int, kaggs, counts: torch.Tensor, ovf: torch.Tensor, n: int, stream: int) -> bool:
    """kaggs: the interpreted kernel's aggregate tuples
    (op, checked, factors, dst, dst2, shared, vbits)."""
    if not (ENABLED and jit.enabled()) or n == 0 or not _aligned(spec.cols):
        return False
    if any(op not in (0, 2, 3) for op, *_ in kaggs):
        return False
    has_mask = spec.mask is not None
    if has_mask and spec.mask.data_ptr() % 4:
        return False
    sh = _Shape(spec.cols)
    aggs = [(op, chk, tuple(tuple(f) for f in fs)) for op, chk, fs, *_ in kaggs]
    nslots_hint = sum(2 if op == 0 else 1 for op, *_ in aggs) + 1
    lanes = 64
    while lanes > 1 and nslots_hint * G * lanes * 8 > LDS_MAX:
        lanes //= 2
    if G == 1:
        grid = max(1, min(-(-n // (BLOCK * ROWS)), 256 * 8))
        per_acc = grid * BLOCK                        # threads; a block sums BLOCK of them
        rows_per = -(-n // per_acc) * BLOCK
    else:
        lds = nslots_hint * G * lanes * 8
        per_cu = max(1, min(8, (160 * 1024) // max(lds, 1)))
        grid = max(1, min(-(-n // (BLOCK * ROWS)), 256 * per_cu))
        rows_per = -(-n // (grid * lanes))            # rows one LDS slot can receive
    lg = max(1, math.ceil(math.log2(rows_per + 1)))
    split = []
    for op, chk, fs, d, d2, shared, vbits in kaggs:
        vb = vbits if 0 < vbits <= 64 else 64
        split.append(op == 0 and vb + lg + 1 > 63)
    name = "igloo_jit_scan_agg"
    if MFMA and 1 < G <= 16 and all(op == 0 for op, *_ in aggs) and ROWS == 4:
        try:
            src, lds = mfma_agg_source(sh, spec.terms, has_mask, keys, G, aggs)
            name = "igloo_jit_scan_agg_mfma"
            per_cu = max(1, min(4, (160 * 1024) // lds))
            grid = max(1, min(-(-n // (BLOCK * ROWS)), 256 * per_cu))
        except ValueError:
            src = agg_source(sh, spec.terms, has_mask, keys, G, aggs, split, lanes)
    else:
        src = agg_source(sh, spec.terms, has_mask, keys, G, aggs, split, lanes)
    k = jit.get(src, name)
    if k is None:
        return False
    args = [t.data_ptr() for t in spec.cols] + ([spec.mask.data_ptr()] if has_mask else []) + [counts.data_ptr()]
    for op, chk, fs, d, d2, shared, vbits in kaggs:
        args += [d, d2 or d]
    args += [ovf.data_ptr(), n]
    k.launch(grid, BLOCK, 0, stream, args + _term_args(spec.terms))
    return True
