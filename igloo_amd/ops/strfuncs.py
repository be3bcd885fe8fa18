"""Scalar string functions (csrc/kernels/strfunc.hip): btrim / ltrim / rtrim,
replace, lpad / rpad, reverse, repeat, left / right, initcap, translate,
split_part, strpos, ascii, octet_length; regexp_like / regexp_replace /
regexp_count (host regex engine, reported as a host step).

Plain device columns run the two-pass kernels; dictionary columns apply the
function to their dictionary only (ops/strings.py ``_dict_transform``); CPU
columns use the Python definitions below, which are also the numerics oracle
of the GPU tests. Parity: DataFusion's string functions (reference
Cargo.lock:1062 datafusion-functions 48.0.0) behind SessionContext::sql
(reference crates/engine/src/lib.rs:54-57).
"""
from __future__ import annotations

import re
from typing import Callable, Optional

import pyarrow as pa
import pyarrow.compute as pc
import torch

from .. import types as T
from ..columnar import Column
from ._lib import is_gpu, launch, native, ptr, stream
from .select import offsets_from_lengths

CODES = {"trim": 0, "replace": 1, "lpad": 2, "rpad": 3, "reverse": 4, "repeat": 5, "left": 6, "right": 7,
         "initcap": 8, "translate": 9, "split_part": 10}
INT_CODES = {"strpos": 20, "ascii": 21, "octet_length": 22}


# ------------------------------------------------------------ Python semantics
def py_fn(name: str, opts: tuple) -> Callable[[str], object]:
    if name == "trim":
        mode, chars = opts
        if mode == 3:
            return lambda s: s.strip(chars)
        return (lambda s: s.lstrip(chars)) if mode == 1 else (lambda s: s.rstrip(chars))
    if name == "replace":
        a, b = opts
        return (lambda s: s) if a == "" else (lambda s: s.replace(a, b))
    if name in ("lpad", "rpad"):
        n, fill = opts
        n = max(int(n), 0)

        def pad(s):
            if len(s) >= n:
                return s[:n]
            if not fill:
                return s
            k = n - len(s)
            f = (fill * (k // len(fill) + 1))[:k]
            return f + s if name == "lpad" else s + f
        return pad
    if name == "reverse":
        return lambda s: s[::-1]
    if name == "repeat":
        n = max(int(opts[0]), 0)
        return lambda s: s * n
    if name == "left":
        n = int(opts[0])
        return lambda s: s[:n] if n >= 0 else s[:max(len(s) + n, 0)]
    if name == "right":
        n = int(opts[0])
        return lambda s: (s[max(len(s) - n, 0):] if n >= 0 else s[min(-n, len(s)):])
    if name == "initcap":
        def initcap(s):
            out, start = [], True
            for ch in s:
                if ch.isascii():
                    out.append(ch.upper() if start else ch.lower())
                else:
                    out.append(ch)
                start = not (ch.isalnum() or not ch.isascii())
            return "".join(out)
        return initcap
    if name == "translate":
        a, b = opts

        def tr(s):
            out = []
            for ch in s:
                k = a.find(ch)
                if k < 0:
                    out.append(ch)
                elif k < len(b):
                    out.append(b[k])
            return "".join(out)
        return tr
    if name == "split_part":
        d, n = opts
        n = int(n)

        def sp(s):
            parts = s.split(d) if d else [s]
            idx = n - 1 if n > 0 else len(parts) + n
            return parts[idx] if 0 <= idx < len(parts) and n != 0 else ""
        return sp
    if name == "strpos":
        sub = opts[0]
        return lambda s: s.find(sub) + 1
    if name == "ascii":
        return lambda s: ord(s[0]) if s else 0
    if name == "octet_length":
        return lambda s: len(s.encode("utf-8"))
    raise KeyError(name)


def _dev_bytes(s: str, device) -> torch.Tensor:
    from .strings import _consts
    b = s.encode("utf-8")
    key = ("strfn_arg", s, str(device))
    return _consts(key, lambda: torch.tensor(list(b) or [0], dtype=torch.uint8).to(device))


def apply(col: Column, name: str, opts: tuple) -> Column:
    """string -> string function ``name`` with constant options."""
    from .strings import _dict_transform, decode
    fn = py_fn(name, opts)
    if col.is_dict:
        return _dict_transform(col, fn, lambda d: apply(d, name, opts))
    if not is_gpu(col.data):
        vals = [None if v is None else fn(v) for v in col.to_arrow().to_pylist()]
        c = Column.from_arrow(pa.array(vals, pa.large_string()), device=col.device, dict_encode=False)
        c.valid = col.valid
        return c
    n = len(col)
    code = CODES[name]
    n1, a, b = 0, "", ""
    if name == "trim":
        n1, a = opts
    elif name == "replace":
        a, b = opts
    elif name in ("lpad", "rpad"):
        n1, a = int(opts[0]), opts[1]
    elif name in ("repeat", "left", "right"):
        n1 = int(opts[0])
    elif name == "translate":
        a, b = opts
    elif name == "split_part":
        a, n1 = opts[0], int(opts[1])
    ta, tb = _dev_bytes(a, col.device), _dev_bytes(b, col.device)
    la, lb = len(a.encode("utf-8")), len(b.encode("utf-8"))
    N = launch("str_fn")
    s = stream(col.data)
    lens = torch.empty(n, dtype=torch.int64, device=col.device)
    N.str_fn_lengths(code, n1, ptr(ta), la, ptr(tb), lb, ptr(col.offsets), ptr(col.data), n, ptr(lens), s)
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(max(total, 1), dtype=torch.uint8, device=col.device)[:total]
    if total:
        N.str_fn_copy(code, n1, ptr(ta), la, ptr(tb), lb, ptr(col.offsets), ptr(col.data), n, ptr(off),
                      ptr(chars), int(chars.numel()), s)
    return Column(T.UTF8, chars, col.valid, offsets=off)


def apply_int(col: Column, name: str, opts: tuple) -> torch.Tensor:
    """string -> int32 function (NULL rows: 0; the caller keeps the validity)."""
    from .strings import _dict_lut_dev, _lut_apply
    fn = py_fn(name, opts)
    if col.is_dict:
        key = ("strfn_int", name) + tuple(opts)
        if is_gpu(col.data):
            return _dict_lut_dev(col, key, lambda d: apply_int(d, name, opts)).to(torch.int32)
        return _lut_apply(col, lambda: [0 if v is None else fn(v) for v in col.dict_values()], key).to(torch.int32)
    if not is_gpu(col.data):
        vals = [0 if v is None else fn(v) for v in col.to_arrow().to_pylist()]
        return torch.tensor(vals, dtype=torch.int32, device=col.device)
    n = len(col)
    pat = opts[0] if name == "strpos" else ""
    tp = _dev_bytes(pat, col.device)
    out = torch.empty(n, dtype=torch.int32, device=col.device)
    launch("str_fn_int").str_fn_int(INT_CODES[name], ptr(tp), len(pat.encode("utf-8")), ptr(col.offsets),
                                    ptr(col.data), n, ptr(out), stream(out))
    return out


# --------------------------------------------------------------------- regexps
def _re_flags(flags: str) -> str:
    return "".join(f for f in flags if f in "imsx")


def regexp(col: Column, name: str, pattern: str, repl: Optional[str] = None, flags: str = ""):
    """regexp_like (bool tensor), regexp_count (int64 tensor), regexp_replace
    (Column): evaluated by the host regex engine over the column's values
    (dictionary columns: over the dictionary only)."""
    from .strings import note_host_step
    from ..utils.errors import PlanError
    try:
        re.compile(pattern)
    except re.error as e:
        raise PlanError(f"invalid regular expression {pattern!r}: {e}") from None
    if name == "regexp_like" and set(flags) <= {"i", "c"} and col.data.is_cuda:
        m = _regexp_like_gpu(col, pattern, "i" in flags and not flags.endswith("c"))
        if m is not None:
            return m
    note_host_step(name)
    fl = _re_flags(flags)
    pat = f"(?{fl}){pattern}" if fl else pattern
    if col.is_dict:
        vals = col.dict_values()
        d = col.dictionary
        arr = pa.array(vals, pa.large_string())
        res = _regexp_arrow(arr, name, pat, repl, flags)
        if name == "regexp_replace":
            from .strings import _lut_apply
            uniq, remap = {}, []
            for v in res.to_pylist():
                remap.append(uniq.setdefault(v, len(uniq)))
            nd = Column.from_arrow(pa.array(list(uniq), pa.large_string()), device=col.device, dict_encode=False)
            codes = _lut_apply(col, remap, ("re_remap", pattern, repl, flags)).to(torch.int32)
            return Column(T.UTF8, codes, col.valid, dictionary=nd)
        lut = torch.tensor([0 if v is None else int(v) for v in res.to_pylist()] or [0], dtype=torch.int64,
                           device=col.device)
        out = lut.index_select(0, col.data.to(torch.int64).clamp(min=0)) if len(col) else lut[:0]
        return out.to(torch.bool) if name == "regexp_like" else out
    arr = col.to_arrow()
    res = _regexp_arrow(arr, name, pat, repl, flags)
    if name == "regexp_replace":
        c = Column.from_arrow(res.cast(pa.large_string()), device=col.device, dict_encode=False)
        c.valid = col.valid
        return c
    t = torch.tensor(res.cast(pa.int64()).fill_null(0).to_numpy(zero_copy_only=False), device=col.device)
    return t.to(torch.bool) if name == "regexp_like" else t


def _regexp_like_gpu(col: Column, pattern: str, icase: bool) -> Optional[torch.Tensor]:
    """regexp_like on the device: the pattern as a byte DFA (ops/regex_dfa.py)
    walked by csrc/kernels/regex.hip, one lane per string (dictionary columns:
    per dictionary entry, then the codes gather the flags). None when the
    pattern needs the host engine."""
    from . import regex_dfa as RD
    from .gather import gather_tensor
    from .strings import decode
    try:
        d = RD.compile_dfa(pattern, icase)
    except (RD.Unsupported, RecursionError):
        return None
    if native().regex_lds_bytes(d.nstates, d.nclasses) > 64 * 1024:
        return None
    dev = col.device
    src = col.dictionary if col.is_dict else (col if col.is_plain_string else decode(col))
    n = len(src)
    table = torch.tensor([x for row in d.table for x in row], dtype=torch.int32).to(torch.int16).to(dev)
    cls = torch.tensor(d.cls, dtype=torch.uint8).to(dev)
    flg = torch.tensor(d.accept, dtype=torch.uint8).to(dev)
    out = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)[:n]
    launch("regex_dfa").regex_dfa_match(ptr(src.offsets), ptr(src.data), n, ptr(table), ptr(cls), ptr(flg),
                                        d.nstates, d.nclasses, d.start, d.anchored_end, False, ptr(out),
                                        stream(out))
    m = out.view(torch.bool)
    if col.is_dict:
        m = gather_tensor(m, col.data) if len(col) else m[:0]
    return m


def _regexp_arrow(arr, name, pat, repl, flags):
    if name == "regexp_like":
        return pc.match_substring_regex(arr, pat)
    if name == "regexp_count":
        return pc.count_substring_regex(arr, pat)
    # Rust-regex replacement syntax ${1} / $1 -> RE2 \1
    r = re.sub(r"\$\{(\d+)\}|\$(\d+)", lambda m: "\\" + (m.group(1) or m.group(2)), repl or "")
    return pc.replace_substring_regex(arr, pat, r, max_replacements=None if "g" in flags else 1)
