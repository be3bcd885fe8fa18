"""md5 / sha224 / sha256 / sha384 / sha512 / digest(), uuid() and to_char()
(csrc/kernels/digest.hip, csrc/kernels/strfmt.hip).

Parity: DataFusion's crypto / datetime string functions (reference
Cargo.lock:1062-1090 datafusion-functions with md-5 and sha2; chrono's
strftime for to_char). DataFusion returns Binary for sha224..sha512 and
digest(); here every digest is the lowercase hex text (md5's type) -- the
bytes a client would hex-encode, parity unpinned for the column type. On the
CPU the host hashlib / strftime give the same values (the GPU tests compare
the kernels against hashlib).
"""
from __future__ import annotations

import datetime
import hashlib
import os
import uuid as _uuid

import pyarrow as pa
import torch

from .. import types as T
from ..columnar import Column
from ._lib import is_gpu, launch, native, ptr, stream

ALGOS = {"md5": 0, "sha224": 1, "sha256": 2, "sha384": 3, "sha512": 4}
WIDTH = {"md5": 32, "sha224": 56, "sha256": 64, "sha384": 96, "sha512": 128}


def _fixed_width(chars: torch.Tensor, n: int, w: int, valid) -> Column:
    off = torch.arange(n + 1, dtype=torch.int64, device=chars.device) * w
    return Column(T.UTF8, chars, valid, offsets=off)


def hex_digest(col: Column, algo: str) -> Column:
    """Hex digest of every string of ``col`` (NULL stays NULL)."""
    from . import strings as S
    algo = algo.lower()
    if algo not in ALGOS:
        from ..utils.errors import PlanError
        raise PlanError(f"digest(): unsupported algorithm '{algo}' (md5, sha224, sha256, sha384, sha512)")
    w = WIDTH[algo]
    if col.is_dict:
        # each distinct value once, the codes pick the digests
        from .gather import take
        d = hex_digest(col.dictionary, algo)
        out = take(d, col.data)
        out.valid = col.valid
        return out
    n = len(col)
    if not is_gpu(col.data):
        vals = col.to_arrow().to_pylist()
        out = [None if v is None else hashlib.new(algo, v.encode("utf-8")).hexdigest() for v in vals]
        return Column.from_arrow(pa.array(out, pa.large_string()), device=col.device, dict_encode=False)
    col = S.decode(col) if not col.is_plain_string else col
    chars = torch.empty(max(n * w, 1), dtype=torch.uint8, device=col.device)[:n * w]
    launch("digest_hex").digest_hex(ALGOS[algo], ptr(col.offsets), ptr(col.data), n, ptr(chars), stream(chars))
    return _fixed_width(chars, n, w, col.valid)


def uuid_column(n: int, device) -> Column:
    """uuid(): a random version-4 UUID per row."""
    device = torch.device(device)
    if device.type != "cuda":
        return Column.from_arrow(pa.array([str(_uuid.uuid4()) for _ in range(n)], pa.large_string()), device=device,
                                 dict_encode=False)
    chars = torch.empty(max(n * 36, 1), dtype=torch.uint8, device=device)[:n * 36]
    seed = int.from_bytes(os.urandom(8), "little")
    launch("uuid_v4").uuid_v4(seed, n, ptr(chars), stream(chars))
    return _fixed_width(chars, n, 36, None)


def py_strftime(us: int, fmt: str) -> str:
    """Host twin of strfmt.hip (chrono's subset used by to_char)."""
    t = datetime.datetime(1970, 1, 1) + datetime.timedelta(microseconds=int(us))
    out, i = [], 0
    days = ["Sunday", "Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday"]
    months = ["January", "February", "March", "April", "May", "June", "July", "August", "September", "October",
              "November", "December"]
    dow = (t.weekday() + 1) % 7
    while i < len(fmt):
        ch = fmt[i]
        if ch != "%" or i + 1 >= len(fmt):
            out.append(ch)
            i += 1
            continue
        s = fmt[i + 1]
        i += 2
        if s == "." and i <= len(fmt):
            if fmt[i:i + 1] == "f":
                out.append("." + f"{t.microsecond * 1000:09d}")
                i += 1
                continue
            if fmt[i:i + 2] in ("3f", "6f", "9f"):
                k = int(fmt[i])
                out.append("." + f"{t.microsecond * 1000:09d}"[:k])
                i += 2
                continue
            out.append("%.")
            continue
        h12 = t.hour % 12 or 12
        m = {"Y": f"{t.year:04d}", "C": f"{t.year // 100:02d}", "y": f"{t.year % 100:02d}", "m": f"{t.month:02d}",
             "d": f"{t.day:02d}", "e": f"{t.day:2d}", "j": f"{t.timetuple().tm_yday:03d}", "H": f"{t.hour:02d}",
             "k": f"{t.hour:2d}", "I": f"{h12:02d}", "l": f"{h12:2d}", "M": f"{t.minute:02d}",
             "S": f"{t.second:02d}", "p": "AM" if t.hour < 12 else "PM", "P": "am" if t.hour < 12 else "pm",
             "f": f"{t.microsecond * 1000:09d}", "a": days[dow][:3], "A": days[dow], "b": months[t.month - 1][:3],
             "h": months[t.month - 1][:3], "B": months[t.month - 1], "u": str(dow or 7), "w": str(dow),
             "F": f"{t.year:04d}-{t.month:02d}-{t.day:02d}", "T": f"{t.hour:02d}:{t.minute:02d}:{t.second:02d}",
             "R": f"{t.hour:02d}:{t.minute:02d}", "D": f"{t.month:02d}/{t.day:02d}/{t.year % 100:02d}",
             "s": str(us // 1_000_000), "%": "%"}.get(s)
        out.append(m if m is not None else "%" + s)
    return "".join(out)


def to_char(col: Column, fmt: str) -> Column:
    """to_char(date | timestamp, format) with chrono's strftime syntax."""
    from .select import offsets_from_lengths
    is_date = col.dtype.kind == "date32"
    n = len(col)
    if not is_gpu(col.data):
        vals = col.data.tolist()
        mult = 86_400_000_000 if is_date else 1
        ok = col.valid.tolist() if col.valid is not None else [True] * n
        out = [py_strftime(v * mult, fmt) if k else None for v, k in zip(vals, ok)]
        return Column.from_arrow(pa.array(out, pa.large_string()), device=col.device, dict_encode=False)
    v = col.data.contiguous()
    b = fmt.encode("utf-8")
    N = native()
    s = stream(v)
    lens = torch.empty(max(n, 1), dtype=torch.int64, device=v.device)
    launch("strfmt").strfmt_lengths(b, is_date, ptr(v), n, ptr(lens), s)
    off, total = offsets_from_lengths(lens[:n])
    chars = torch.empty(max(total, 1), dtype=torch.uint8, device=v.device)[:total]
    if total:
        N.strfmt_write(b, is_date, ptr(v), n, ptr(off), int(chars.numel()), ptr(chars), s)
    return Column(T.UTF8, chars, col.valid, offsets=off)
