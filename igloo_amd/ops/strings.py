"""String operators (csrc/kernels/strings.hip).

Dictionary-encoded columns (low cardinality, e.g. p_type, l_shipmode) are
evaluated once per distinct value on the host dictionary and mapped to rows
through a code lookup table; plain columns (comments, names) run per-row HIP
kernels on the GPU and pyarrow.compute on the CPU.
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
from ._lib import capturing, check_not_capturing, is_gpu, launch, ptr, stream, to_host_int
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
    return v


def _with_valid(values: torch.Tensor, col: Column) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    return values, col.valid


# ------------------------------------------------------------------------ LIKE
def like(col: Column, pattern: str, ci: bool = False, negate: bool = False, escape: Optional[str] = "\\") -> torch.Tensor:
    """Bool tensor (NULL rows are False; callers combine ``col.valid``)."""
    if col.is_dict:
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
                                                      len(seg_off) - 1, a0, a1, negate, ptr(out), stream(out))
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


def in_list(col: Column, values: Sequence[str]) -> torch.Tensor:
    if col.is_dict:
        s = set(values)
        return _lut_apply(col, lambda: [v in s for v in col.dict_values()], ("in", tuple(values))).to(torch.bool)
    out = None
    for v in values:
        m = compare_const(col, "=", v)
        out = m if out is None else (out | m)
    return out if out is not None else torch.zeros(len(col), dtype=torch.bool, device=col.device)


# ------------------------------------------------------------ transformations
def _dict_transform(col: Column, fn) -> Column:
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
        return _dict_transform(col, str.upper if up else str.lower)
    if not is_gpu(col.data):
        return _host_roundtrip(col, pc.utf8_upper if up else pc.utf8_lower)
    out = torch.empty_like(col.data)
    flag = torch.zeros(1, dtype=torch.int32, device=col.device)
    launch("str_case").str_case(ptr(col.data), col.data.numel(), up, ptr(out), ptr(flag), stream(out))
    if to_host_int(flag):
        # non-ASCII bytes present: full Unicode case mapping can change byte
        # lengths ('ß' -> 'SS'), so take the exact host path.
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
        return _dict_transform(col, lambda s: _py_substr(s, start, length))
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
    if col.is_dict:
        return _lut_apply(col, lambda: [0 if v is None else len(v) for v in col.dict_values()],
                          ("char_length",)).to(torch.int32)
    arr = col.to_arrow()
    r = pc.utf8_length(arr).fill_null(0).to_numpy(zero_copy_only=False)
    return torch.from_numpy(r.astype(np.int32)).to(col.device)


def concat(a: Column, b: Column) -> Column:
    arr = pc.binary_join_element_wise(a.to_arrow(), b.to_arrow(), "")
    return Column.from_arrow(arr, device=a.device)


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
