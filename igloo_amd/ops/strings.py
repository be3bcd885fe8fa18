"""String operators (csrc/kernels/strings.hip, strexpr.hip).

Dictionary-encoded columns (low cardinality, e.g. p_type, l_shipmode) are
evaluated once per distinct value — on the GPU by running the plain-string
kernel over the dictionary's own device column — and mapped to rows through a
code lookup table; plain columns (comments, names) run per-row HIP kernels on
the GPU and pyarrow.compute on the CPU (the CPU engine's reference path).
What still leaves the GPU (non-ASCII case mapping, float text formatting) is
counted by ``note_host_step`` and reported by EXPLAIN ANALYZE.
"""
from __future__ import annotations

import re
from typing import List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

from .. import types as T
from ..columnar import Column
from .gather import gather_tensor
from ._lib import capture_hold, capturing, check_not_capturing, device_ints, is_gpu, launch, note_host_step, ptr, stream, to_host_int
from .gather import take
from .hashing import group_ids
from .select import offsets_from_lengths

CMP_OPS = {"=": 0, "<>": 1, "<": 2, "<=": 3, ">": 4, ">=": 5}


# --------------------------------------------------------------------- helpers
def tokenize_like(pattern: str, escape: Optional[str] = "\\") -> Tuple[bytes, bytes]:
    """LIKE pattern -> (bytes, kinds) with kinds 0=literal byte, 1='_', 2='%'."""
    out, kinds = bytearray(), bytearray()
    i = 0
    while i < len(pattern):
        ch = pattern[i]
        if escape and ch == escape and i + 1 < len(pattern):
            for b in pattern[i + 1].encode("utf-8"):
                out.append(b)
                kinds.append(0)
            i += 2
            continue
        if ch == "%":
            if not (kinds and kinds[-1] == 2):  # collapse %%
                out.append(0)
                kinds.append(2)
        elif ch == "_":
            out.append(0)
            kinds.append(1)
        else:
            for b in ch.encode("utf-8"):
                out.append(b)
                kinds.append(0)
        i += 1
    return bytes(out), bytes(kinds)


def _like_segments(pat: bytes, kinds: bytes):
    """'%'-separated literal segments of a tokenized LIKE pattern, or None when
    the pattern has '_' wildcards / too many or too long segments.
    Returns (concatenated bytes, offsets, anchored_start, anchored_end)."""
    if 1 in kinds:
        return None
    segs, cur = [], bytearray()
    for b, k in zip(pat, kinds):
        if k == 2:
            if cur:
                segs.append(bytes(cur))
                cur = bytearray()
        else:
            cur.append(b)
    if cur:
        segs.append(bytes(cur))
    a0 = not kinds or kinds[0] != 2
    a1 = not kinds or kinds[-1] != 2
    if len(segs) > 4 or sum(map(len, segs)) > 256 or (not segs and (a0 or a1)):
        return None   # empty pattern '' (matches only empty strings) keeps the generic matcher
    off = [0]
    for sg in segs:
        off.append(off[-1] + len(sg))
    return b"".join(segs), off, a0, a1


def like_regex(pattern: str, ci: bool = False, escape: Optional[str] = "\\") -> "re.Pattern":
    parts = []
    i = 0
    while i < len(pattern):
        ch = pattern[i]
        if escape and ch == escape and i + 1 < len(pattern):
            parts.append(re.escape(pattern[i + 1]))
            i += 2
            continue
        parts.append(".*" if ch == "%" else "." if ch == "_" else re.escape(ch))
        i += 1
    return re.compile("".join(parts), re.DOTALL | (re.IGNORECASE if ci else 0))


def _lut_apply(col: Column, lut_vals, key=None) -> torch.Tensor:
    """Map dictionary codes through a per-dictionary-entry lookup table.
    ``lut_vals``: the table, or (with ``key``) a callable building it; keyed
    tables are kept on the dictionary, so a repeated predicate reuses its
    device table instead of rebuilding and uploading it every query."""
    cache = col.dictionary.derived() if key is not None else None
    lut = cache.get(key) if cache is not None else None
    if lut is None:
        check_not_capturing("dictionary lookup-table upload")
        lut = torch.tensor(list(lut_vals() if callable(lut_vals) else lut_vals), device=col.device)
        if cache is not None:
            cache[key] = lut
    if lut.numel() == 0:
        return torch.zeros(len(col), dtype=lut.dtype, device=col.device)
    return gather_tensor(lut, col.data)


def _dict_lut_dev(col: Column, key, plain_fn) -> torch.Tensor:
    """Per-code result of ``plain_fn`` evaluated over the dictionary's own
    (plain, device) string column — the dictionary never leaves the GPU —
    then gathered by the codes. The table is kept on the dictionary (not
    while a graph is being captured: its contents would only exist inside
    that graph's replays)."""
    from ._lib import capturing
    d = col.dictionary
    cache = d.derived()
    lut = cache.get(key)
    if lut is None:
        dp = decode(d) if d.is_dict else d
        lut = plain_fn(dp)
        if dp.valid is not None:
            lut = lut & dp.valid if lut.dtype == torch.bool else torch.where(dp.valid, lut, torch.zeros_like(lut))
        if not capturing():
            cache[key] = lut
    if lut.numel() == 0:
        return torch.zeros(len(col), dtype=lut.dtype, device=col.device)
    return gather_tensor(lut, col.data)


_CONSTS: dict = {}


def _consts(key, build):
    """Device copies of small per-pattern constants (LIKE segments, comparison
    bytes), uploaded once per pattern and device."""
    v = _CONSTS.get(key)
    if v is None:
        check_not_capturing("pattern constant upload")
        if len(_CONSTS) > 4096:
            _CONSTS.clear()
        v = _CONSTS[key] = build()
    # a captured graph reads it by address: it must outlive a later clear()
    capture_hold(v)
    return v


def _with_valid(values: torch.Tensor, col: Column) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    return values, col.valid


# ------------------------------------------------------------------------ LIKE
def like(col: Column, pattern: str, ci: bool = False, negate: bool = False, escape: Optional[str] = "\\") -> torch.Tensor:
    """Bool tensor (NULL rows are False; callers combine ``col.valid``)."""
    if col.is_dict:
        if is_gpu(col.data):
            return _dict_lut_dev(col, ("like", pattern, ci, negate, escape),
                                 lambda d: like(d, pattern, ci, negate, escape))
        def build():
            rx = like_regex(pattern, ci, escape)
            return [(v is not None and rx.fullmatch(v) is not None) != negate for v in col.dict_values()]
        return _lut_apply(col, build, ("like", pattern, ci, negate, escape)).to(torch.bool)
    n = len(col)
    if not is_gpu(col.data):
        arr = col.to_arrow()
        r = pc.match_like(arr, pattern, ignore_case=ci)
        if negate:
            r = pc.invert(r)
        return torch.from_numpy(r.fill_null(False).to_numpy(zero_copy_only=False).astype(np.bool_))
    pat, kinds = tokenize_like(pattern, escape)
    dev = col.device
    segs = None if ci else _like_segments(pat, kinds)
    if segs is not None:
        seg_bytes, seg_off, a0, a1 = segs
        sb, so = _consts(("seg", pattern, escape, dev), lambda: (
            torch.tensor(list(seg_bytes) or [0], dtype=torch.uint8).to(dev),
            torch.tensor(seg_off, dtype=torch.int32).to(dev)))
        out = torch.empty(n, dtype=torch.bool, device=dev)
        launch("str_like_segments").str_like_segments(ptr(col.offsets), ptr(col.data), n, ptr(sb), ptr(so),
                                                      len(seg_off) - 1, a0, a1, negate, ptr(out), col.data.numel(),
                                                      min((b - a for a, b in zip(seg_off, seg_off[1:])), default=0),
                                                      stream(out))
        return out
    pt, kt = _consts(("pat", pattern, escape, dev), lambda: (
        torch.tensor(list(pat) or [0], dtype=torch.uint8).to(dev),
        torch.tensor(list(kinds) or [0], dtype=torch.uint8).to(dev)))
    out = torch.empty(n, dtype=torch.bool, device=dev)
    launch("str_like").str_like(ptr(col.offsets), ptr(col.data), n, ptr(pt), ptr(kt), len(pat), ci, negate, ptr(out),
                                stream(out))
    return out


# --------------------------------------------------------------- comparisons
def compare_const(col: Column, op: str, value: str) -> torch.Tensor:
    if col.is_dict:
        if is_gpu(col.data):
            return _dict_lut_dev(col, ("cmp", op, value), lambda d: compare_const(d, op, value))
        import operator as o
        f = {"=": o.eq, "<>": o.ne, "<": o.lt, "<=": o.le, ">": o.gt, ">=": o.ge}[op]
        vb = value.encode("utf-8")
        return _lut_apply(col, lambda: [(v is not None and f(v.encode("utf-8"), vb)) for v in col.dict_values()],
                          ("cmp", op, value)).to(torch.bool)
    n = len(col)
    if not is_gpu(col.data):
        arr = col.to_arrow()
        fn = {"=": pc.equal, "<>": pc.not_equal, "<": pc.less, "<=": pc.less_equal, ">": pc.greater,
              ">=": pc.greater_equal}[op]
        r = fn(arr, pa.scalar(value, pa.large_string()))
        return torch.from_numpy(r.fill_null(False).to_numpy(zero_copy_only=False).astype(np.bool_))
    vb = value.encode("utf-8")
    ct = _consts(("bytes", value, col.device), lambda: torch.tensor(list(vb) or [0], dtype=torch.uint8).to(col.device))
    out = torch.empty(n, dtype=torch.bool, device=col.device)
    launch("str_cmp_const").str_cmp_const(ptr(col.offsets), ptr(col.data), n, ptr(ct), len(vb), CMP_OPS[op], ptr(out),
                                          stream(out))
    return out


def in_set(col: Column, values: Sequence[str], prefix_chars: Optional[int] = None) -> torch.Tensor:
    """bool per row of a plain string column: the row is one of ``values``;
    with ``prefix_chars`` L: ``substr(row, 1, L)`` is (a constant of L code
    points is a byte prefix of the row, a shorter one the whole row). One
    pass on the GPU (strings.hip in_set_kernel), no substring copy."""
    vals, modes = [], []
    for v in dict.fromkeys(values):
        nch = len(v)
        if prefix_chars is not None and nch > prefix_chars:
            continue                     # longer than the substring: never equal
        vals.append(v.encode("utf-8"))
        modes.append(1 if prefix_chars is not None and nch == prefix_chars else 0)
    n = len(col)
    if not is_gpu(col.data):
        base = substr(col, 1, prefix_chars) if prefix_chars is not None else col
        return in_list(base, [v.decode("utf-8") for v in vals]) if vals else torch.zeros(n, dtype=torch.bool)
    out = torch.empty(n, dtype=torch.bool, device=col.device)
    key = ("in_set", tuple(vals), tuple(modes), col.device)
    vb = _consts(key + ("b",), lambda: torch.tensor(list(b"".join(vals)) or [0], dtype=torch.uint8).to(col.device))
    voff = _consts(key + ("o",), lambda: torch.tensor(np.cumsum([0] + [len(v) for v in vals]).tolist(),
                                                      dtype=torch.int32).to(col.device))
    vm = _consts(key + ("m",), lambda: torch.tensor(modes or [0], dtype=torch.uint8).to(col.device))
    launch("str_in_set").str_in_set(ptr(col.offsets), ptr(col.data), n, ptr(vb), ptr(voff), ptr(vm), len(vals),
                                    ptr(out), stream(out))
    return out


def in_list(col: Column, values: Sequence[str]) -> torch.Tensor:
    if not col.is_dict and is_gpu(col.data) and len(values) > 1:
        return in_set(col, values)
    if col.is_dict:
        if is_gpu(col.data):
            return _dict_lut_dev(col, ("in", tuple(values)), lambda d: in_list(d, values))
        s = set(values)
        return _lut_apply(col, lambda: [v in s for v in col.dict_values()], ("in", tuple(values))).to(torch.bool)
    out = None
    for v in values:
        m = compare_const(col, "=", v)
        out = m if out is None else (out | m)
    return out if out is not None else torch.zeros(len(col), dtype=torch.bool, device=col.device)


# ------------------------------------------------------------ transformations
def _dict_transform(col: Column, fn, plain_fn=None) -> Column:
    """A string -> string function over a dictionary column: applied to the
    dictionary's values only. On the GPU (``plain_fn`` = the same function
    over a plain device column) the transformed values are re-encoded on the
    device (equal results share one code) and the codes remapped by a gather."""
    if plain_fn is not None and is_gpu(col.data):
        d = col.dictionary
        dp = decode(d) if d.is_dict else d
        enc = dict_encode(plain_fn(dp))
        remap = enc.data.to(torch.int32)
        codes = gather_tensor(remap, col.data) if len(dp) else col.data
        return Column(T.UTF8, codes, col.valid, dictionary=enc.dictionary)
    vals = [None if v is None else fn(v) for v in col.dict_values()]
    uniq, remap = {}, []
    for v in vals:
        if v not in uniq:
            uniq[v] = len(uniq)
        remap.append(uniq[v])
    new_dict = Column.from_arrow(pa.array(list(uniq.keys()), pa.large_string()), device=col.device, dict_encode=False)
    codes = _lut_apply(col, remap).to(torch.int32) if remap else col.data
    return Column(T.UTF8, codes, col.valid, dictionary=new_dict)


def _host_roundtrip(col: Column, fn_arrow) -> Column:
    arr = col.to_arrow()
    if fn_arrow in (pc.utf8_upper, pc.utf8_lower) and not pc.all(pc.string_is_ascii(arr)).as_py():
        # full Unicode case mapping with Rust/Python semantics ('ß' -> 'SS'),
        # which is what the reference's String::to_uppercase produces
        f = str.upper if fn_arrow is pc.utf8_upper else str.lower
        arr = pa.array([None if v is None else f(v) for v in arr.to_pylist()], pa.large_string())
    else:
        arr = fn_arrow(arr)
    return Column.from_arrow(arr, device=col.device, dict_encode=False)


def upper(col: Column) -> Column:
    return _case(col, True)


def lower(col: Column) -> Column:
    return _case(col, False)


def _case(col: Column, up: bool) -> Column:
    if col.is_dict:
        return _dict_transform(col, str.upper if up else str.lower, lambda d: _case(d, up))
    if not is_gpu(col.data):
        return _host_roundtrip(col, pc.utf8_upper if up else pc.utf8_lower)
    out = torch.empty_like(col.data)
    flag = torch.zeros(1, dtype=torch.int32, device=col.device)
    launch("str_case").str_case(ptr(col.data), col.data.numel(), up, ptr(out), ptr(flag), stream(out))
    if to_host_int(flag):
        # non-ASCII bytes present: full Unicode case mapping can change byte
        # lengths ('ß' -> 'SS'), so take the exact host path.
        note_host_step("upper/lower of non-ASCII text")
        return _host_roundtrip(col, pc.utf8_upper if up else pc.utf8_lower)
    return Column(T.UTF8, out, col.valid, offsets=col.offsets)


def _py_substr(s: str, start: int, length: Optional[int]) -> str:
    first = max(start, 1)
    last = None if length is None else start + length
    if last is not None and last <= first:
        return ""
    return s[first - 1: None if last is None else last - 1]


def substr(col: Column, start: int, length: Optional[int]) -> Column:
    if col.is_dict:
        return _dict_transform(col, lambda s: _py_substr(s, start, length), lambda d: substr(d, start, length))
    n = len(col)
    if not is_gpu(col.data):
        vals = [None if v is None else _py_substr(v, start, length) for v in col.to_pylist()]
        c = Column.from_arrow(pa.array(vals, pa.large_string()), device=col.device, dict_encode=False)
        c.valid = col.valid
        return c
    N = launch("str_substr")
    s = stream(col.data)
    has_len = length is not None
    lens = torch.empty(n, dtype=torch.int64, device=col.device)
    N.str_substr_lengths(ptr(col.offsets), ptr(col.data), n, start, length or 0, has_len, ptr(lens), s)
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(total, dtype=torch.uint8, device=col.device)
    if total:
        N.str_substr_copy(ptr(col.offsets), ptr(col.data), n, start, length or 0, has_len, ptr(off), ptr(chars), s)
    return Column(T.UTF8, chars, col.valid, offsets=off)


def char_length(col: Column) -> torch.Tensor:
    """Characters (UTF-8 code points) per row, int32 (NULL rows: 0)."""
    if col.is_dict:
        if is_gpu(col.data):
            return _dict_lut_dev(col, ("char_length",), char_length).to(torch.int32)
        return _lut_apply(col, lambda: [0 if v is None else len(v) for v in col.dict_values()],
                          ("char_length",)).to(torch.int32)
    if not is_gpu(col.data):
        arr = col.to_arrow()
        r = pc.utf8_length(arr).fill_null(0).to_numpy(zero_copy_only=False)
        return torch.from_numpy(r.astype(np.int32)).to(col.device)
    n = len(col)
    out = torch.empty(n, dtype=torch.int32, device=col.device)
    launch("str_char_length").str_char_length(ptr(col.offsets), ptr(col.data), n, ptr(out), stream(out))
    return out


def const_column(value: str, device) -> Column:
    """One-row plain string column (a constant operand broadcast by the kernels)."""
    b = value.encode("utf-8")
    key = ("const_col", value, str(device))
    def build():
        return (torch.tensor(list(b) or [0], dtype=torch.uint8).to(device)[:len(b)],
                torch.tensor([0, len(b)], dtype=torch.int64).to(device))
    chars, off = _consts(key, build)
    return Column(T.UTF8, chars, None, offsets=off)


def concat(a: Column, b: Column, n: Optional[int] = None) -> Column:
    """a || b (NULL when either side is NULL). Either side may be a one-row
    constant column broadcast over ``n`` rows."""
    n = n if n is not None else max(len(a), len(b))
    if not is_gpu(a.data if len(a) else b.data):
        aa, bb = a.to_arrow().cast(pa.large_string()), b.to_arrow().cast(pa.large_string())
        if len(aa) == 1 and n != 1:
            aa = pa.array([aa[0].as_py()] * n, pa.large_string())
        if len(bb) == 1 and n != 1:
            bb = pa.array([bb[0].as_py()] * n, pa.large_string())
        return Column.from_arrow(pc.binary_join_element_wise(aa, bb, pa.scalar("", pa.large_string())), device=a.device)
    a, b = decode(a), decode(b)
    ba, bb_ = len(a) == 1 and n != 1, len(b) == 1 and n != 1
    N = launch("str_concat")
    s = stream(a.offsets)
    lens = torch.empty(n, dtype=torch.int64, device=a.device)
    N.str_concat2_lengths(ptr(a.offsets), ba, ptr(b.offsets), bb_, n, ptr(lens), s)
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(total, dtype=torch.uint8, device=a.device)
    if total:
        N.str_concat2_copy(ptr(a.offsets), ptr(a.data), ba, ptr(b.offsets), ptr(b.data), bb_, n, ptr(off), ptr(chars), s)
    va = None if a.valid is None else (a.valid.expand(n) if ba else a.valid)
    vb = None if b.valid is None else (b.valid.expand(n) if bb_ else b.valid)
    valid = va if vb is None else (vb if va is None else va & vb)
    return Column(T.UTF8, chars, valid.contiguous() if valid is not None else None, offsets=off)


#: fmt / parse kinds of the strexpr kernels
_FMT_FIXED, _FMT_I32, _FMT_DATE, _FMT_BOOL = 0, 1, 2, 3


def to_string(col: Column) -> Column:
    """CAST(x AS VARCHAR) on the GPU for integers, decimals (text at the
    type's scale), dates (ISO) and booleans. Floats keep the host formatter
    (shortest round-trip text), reported as a host step."""
    t = col.dtype
    n = len(col)
    x = col.data
    if t.is_decimal and col.is_wide:
        kind = None
    elif t.is_decimal or t.kind in ("int64",) or (t.is_integer and x.dtype == torch.int64):
        kind, scale, x = _FMT_FIXED, (t.scale if t.is_decimal else 0), x.to(torch.int64).contiguous()
    elif t.is_integer:
        kind, scale, x = _FMT_I32, 0, x.to(torch.int32).contiguous()
    elif t.kind == "date32":
        kind, scale, x = _FMT_DATE, 0, x.to(torch.int32).contiguous()
    elif t.kind == "bool":
        kind, scale, x = _FMT_BOOL, 0, x.to(torch.uint8).contiguous()
    else:
        kind = None
    if kind is None or not is_gpu(x):
        if is_gpu(x):
            note_host_step(f"CAST({t} AS VARCHAR)")
        return Column.from_arrow(pc.cast(col.to_arrow(), pa.large_string()), device=col.device, dict_encode=False)
    N = launch("fmt")
    s = stream(x)
    valid = col.valid.to(torch.uint8).contiguous() if col.valid is not None else None
    lens = torch.empty(n, dtype=torch.int64, device=x.device)
    N.fmt_lengths(ptr(x), kind, n, scale, ptr(valid), ptr(lens), s)
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(total, dtype=torch.uint8, device=x.device)
    if total:
        N.fmt_write(ptr(x), kind, n, scale, ptr(valid), ptr(off), ptr(chars), s)
    return Column(T.UTF8, chars, col.valid, offsets=off)


def parse(col: Column, t) -> Column:
    """CAST(varchar AS t) on the GPU: integers, decimals (exact at t's scale),
    dates, doubles and booleans; a malformed value raises ExecutionError."""
    from ..utils.errors import ExecutionError
    c = decode(col)
    n = len(c)
    if not is_gpu(c.data):
        return Column.from_arrow(pc.cast(c.to_arrow(), t.to_arrow()), device=c.device, dtype=t)
    if t.is_decimal:
        kind, scale, dt = 2, t.scale, torch.int64
    elif t.kind == "date32":
        kind, scale, dt = 3, 0, torch.int32
    elif t.is_float:
        kind, scale, dt = 4, 0, torch.float64
    elif t.kind == "bool":
        kind, scale, dt = 5, 0, torch.uint8
    elif t.is_integer:
        kind, scale, dt = (0, 0, torch.int64) if t.torch_dtype == torch.int64 else (1, 0, torch.int32)
    else:
        note_host_step(f"CAST(VARCHAR AS {t})")
        return Column.from_arrow(pc.cast(c.to_arrow(), t.to_arrow()), device=c.device, dtype=t)
    out = torch.empty(n, dtype=dt, device=c.device)
    err = torch.zeros(1, dtype=torch.int32, device=c.device)
    valid = c.valid.to(torch.uint8).contiguous() if c.valid is not None else None
    launch("str_parse").str_parse(ptr(c.offsets), ptr(c.data), n, ptr(valid), kind, scale, ptr(out), ptr(err),
                                  stream(out))
    if to_host_int(err):
        raise ExecutionError(f"cannot cast string value to {t}")
    if dt == torch.uint8:
        out = out.to(torch.bool)
    elif t.torch_dtype != dt and t.kind != "date32":
        out = out.to(t.torch_dtype)
    return Column(t, out, c.valid)


def select_rows(branches: Sequence[Column], choice: torch.Tensor, n: int) -> Column:
    """Row i takes row i of ``branches[choice[i]]`` (a one-row branch is a
    constant). Every branch is appended into one plain column and a single
    device string gather picks the rows: CASE / COALESCE over strings."""
    parts, base = [], []
    pos = 0
    for br in branches:
        p = decode(br)
        if p.valid is None:
            p = Column(T.UTF8, p.data, torch.ones(len(p), dtype=torch.bool, device=p.device), offsets=p.offsets)
        parts.append(p)
        base.append(pos)
        pos += len(p)
    offs = [parts[0].offsets]
    shift = parts[0].offsets[-1:]
    for p in parts[1:]:
        offs.append(p.offsets[1:] + shift)
        shift = shift + p.offsets[-1:]
    allc = Column(T.UTF8, torch.cat([p.data for p in parts]), torch.cat([p.valid for p in parts]),
                  offsets=torch.cat(offs))
    rows = torch.arange(n, dtype=torch.int64, device=choice.device)
    starts = device_ints(base, choice.device)
    single = device_ints([int(len(p) == 1 and n != 1) for p in parts], choice.device).bool()
    ch = choice.to(torch.int64)
    idx = starts.index_select(0, ch) + torch.where(single.index_select(0, ch), torch.zeros_like(rows), rows)
    return take(allc, idx)


# ------------------------------------------------------------------ encoding
def hash64(col: Column) -> torch.Tensor:
    n = len(col)
    if not is_gpu(col.data):
        import xxhash
        vals = col.to_pylist()
        return torch.tensor([(xxhash.xxh64_intdigest(v.encode()) - 2**63) if v is not None else 0 for v in vals],
                            dtype=torch.int64)
    out = torch.empty(n, dtype=torch.int64, device=col.device)
    launch("str_hash64").str_hash64(ptr(col.offsets), ptr(col.data), n, ptr(col.valid), ptr(out), stream(out))
    out._igloo_hashed = True     # spread over 64 bits: group_ids goes straight to its hash table
    return out


def decode(col: Column) -> Column:
    """Dictionary column -> plain column."""
    if not col.is_dict:
        return col
    if col.valid is not None:
        # codes under NULL rows are unspecified: never dereference them
        idx = torch.where(col.valid, col.data, torch.full_like(col.data, -1))
        c = take(col.dictionary, idx, neg=True)
    else:
        c = take(col.dictionary, col.data)
    c.valid = col.valid
    return c


def dict_encode(col: Column) -> Column:
    """Plain column -> dictionary column (exact: hash collisions are verified)."""
    if col.is_dict:
        return col
    n = len(col)
    if not is_gpu(col.data):
        return Column.from_arrow(pc.dictionary_encode(col.to_arrow()), device=col.device)
    h = hash64(col)
    gid, g, rep = group_ids(h)
    # verify every row equals its group's representative (no 64-bit collision)
    mism = torch.zeros(1, dtype=torch.int32, device=col.device)
    rep_of_row = gather_tensor(rep, gid)
    ri = rep_of_row.to(torch.int32)
    ai = torch.arange(n, dtype=torch.int32, device=col.device)
    launch("str_eq_rows").str_eq_rows(ptr(col.offsets), ptr(col.data), ptr(ai), ptr(col.offsets), ptr(col.data),
                                      ptr(ri), False, n, ptr(mism), stream(mism))
    if to_host_int(mism):
        return Column.from_arrow(pc.dictionary_encode(col.to_arrow()), device=col.device)
    dictionary = take(col, rep)
    dictionary.valid = None
    return Column(T.UTF8, gid, col.valid, dictionary=dictionary)


def sort_ranks(col: Column) -> torch.Tensor:
    """Order-preserving int64 rank per row (byte-wise UTF-8 order)."""
    c = dict_encode(col) if not col.is_dict else col
    cache = c.dictionary.derived()
    lut = cache.get("rank")
    dd = c.dictionary
    if lut is None and is_gpu(dd.data) and dd.valid is None and dd.offsets is not None:
        lut = _device_ranks(dd)
        if not capturing():     # a rank computed inside a graph lives in its pool: never cache it
            cache["rank"] = lut
    if lut is None:
        check_not_capturing("dictionary rank upload")
        d = c.dictionary.to_arrow()
        if len(d) == 0:
            return torch.zeros(len(c), dtype=torch.int64, device=c.device)
        # Arrow orders strings byte-wise (UTF-8 code point order), NULL entries last
        order = pc.array_sort_indices(d, null_placement="at_end").to_numpy()
        rank = np.empty(len(order), dtype=np.int64)
        rank[order] = np.arange(len(order), dtype=np.int64)
        lut = cache["rank"] = torch.from_numpy(rank).to(c.device)
    return gather_tensor(lut, c.data)


def _device_ranks(d: Column) -> torch.Tensor:
    """Byte-wise UTF-8 order rank of every entry of a plain-string dictionary,
    on the device: an LSD radix argsort over 8-byte big-endian chunks
    (``str_prefix_keys``, last chunk first; ops/sort.py). The only host value is
    the longest entry's length (a replayable readback)."""
    from .sort import argsort
    n = len(d)
    dev = d.data.device
    if n == 0:
        return torch.zeros(0, dtype=torch.int64, device=dev)
    lens = d.offsets[1:] - d.offsets[:-1]
    chunks = max(1, (to_host_int(lens.max()) + 7) // 8)
    keys = torch.empty(chunks * n, dtype=torch.int64, device=dev)
    launch("str_prefix_keys").str_prefix_keys(ptr(d.offsets), ptr(d.data), n, chunks, ptr(keys), stream(keys))
    perm = argsort([(keys[k * n:(k + 1) * n], False, False, None) for k in range(chunks)], n, dev)
    rank = torch.empty(n, dtype=torch.int64, device=dev)
    rank.index_copy_(0, perm.long(), torch.arange(n, dtype=torch.int64, device=dev))
    return rank


def group_codes(col: Column) -> Tuple[torch.Tensor, Column]:
    """(int32 codes, dictionary-encoded column) for GROUP BY / join on strings."""
    c = dict_encode(col)
    return c.data, c
