"""LIST / STRUCT column operations (csrc/kernels/nested.hip + the gather and
range-expansion kernels).

Parity: DataFusion's nested functions (reference Cargo.lock:1125
datafusion-functions-nested: make_array / ``[..]`` literals, array_length,
cardinality, array_element / ``l[i]``, unnest, array_agg, struct /
named_struct / get_field), reached through ``SessionContext::sql``
(reference crates/engine/src/lib.rs:54-57).

Layout (types.py): a LIST row is an (start, length) int64 pair into
``col.nested.child``; a STRUCT row is an int64 row id into each of
``col.nested.children``. Row movement (filters, joins, sorts) therefore
gathers 16 / 8 bytes per row and never touches the children; functions turn
into index arithmetic plus one child gather.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import pyarrow as pa
import torch

from .. import types as T
from ..columnar import Column, Nested
from ..utils.errors import ExecutionError, NotSupported
from ._lib import is_gpu, launch, ptr, stream, to_host_int


def _cat_children(children: List[Column]) -> Column:
    from ..exec.joins import concat_columns
    return concat_columns(children) if len(children) > 1 else children[0]


def concat(cols: Sequence[Column], valid: Optional[torch.Tensor]) -> Column:
    """Rows of ``cols`` end to end (UNION ALL, INSERT): children concatenated,
    each part's starts / row ids shifted by the child rows before it."""
    c0 = cols[0]
    dt = c0.dtype
    datas, base = [], 0
    if dt.kind == "list":
        kids = [c.nested.child for c in cols]
        for c, ch in zip(cols, kids):
            d = c.data.clone()
            d[:, 0] += base
            datas.append(d)
            base += len(ch)
        return Column(dt, torch.cat(datas), valid, dictionary=Nested(child=_cat_children(kids)))
    kids: Dict[str, List[Column]] = {n: [] for n, _ in dt.fields}
    for c in cols:
        datas.append(c.data + base)
        for n, _ in dt.fields:
            kids[n].append(c.nested.children[n])
        base += len(c.nested)
    return Column(dt, torch.cat(datas), valid,
                  dictionary=Nested(children={n: _cat_children(v) for n, v in kids.items()}))


def scalar_to_column(value, dtype: T.DataType, n: int, device) -> Column:
    return Column.full(value, dtype, n, device)


def make_list(cols: Sequence[Column], n: int, dtype: T.DataType, device) -> Column:
    """make_array(c0, .., ck-1): row r = [c0[r], .., ck-1[r]]. The child is
    the k columns concatenated, read back interleaved (one gather)."""
    from .gather import take
    k = len(cols)
    device = torch.device(device)
    if k == 0:
        child = Column.full(None, dtype.child if dtype.child.kind != "null" else T.INT64, 0, device)
        se = torch.zeros((n, 2), dtype=torch.int64, device=device)
        return Column(dtype, se, None, dictionary=Nested(child=child))
    flat = _cat_children(list(cols))
    idx = torch.empty(n * k, dtype=torch.int64, device=device)
    se = torch.empty((n, 2), dtype=torch.int64, device=device)
    if is_gpu(idx):
        s = stream(idx)
        launch("interleave_idx").interleave_idx(n, k, ptr(idx), s)
        launch("list_slots").list_slots(n, k, ptr(se), s)
    else:
        r = torch.arange(n, dtype=torch.int64)
        idx = (torch.arange(k, dtype=torch.int64).view(1, k) * n + r.view(n, 1)).reshape(-1)
        se = torch.stack([r * k, torch.full_like(r, k)], 1)
    child = take(flat, idx) if n * k else flat
    return Column(dtype, se, None, dictionary=Nested(child=child))


def lengths(col: Column) -> torch.Tensor:
    return col.data[:, 1].contiguous() if len(col) else torch.zeros(0, dtype=torch.int64, device=col.device)


def element(col: Column, pos, pos_valid: Optional[torch.Tensor] = None) -> Column:
    """l[i] / array_element(l, i): 1-based, negative from the end, NULL when
    out of range. ``pos``: an int constant or an int64 tensor per row."""
    from .gather import take
    n = len(col)
    child = col.nested.child
    dev = col.device
    out = torch.empty(n, dtype=torch.int64, device=dev)
    ptensor = pos.to(torch.int64).contiguous() if isinstance(pos, torch.Tensor) else None
    if is_gpu(out):
        launch("list_element_idx").list_element_idx(ptr(col.data.contiguous()), ptr(col.valid), ptr(ptensor),
                                                    ptr(pos_valid), 0 if ptensor is not None else int(pos), n,
                                                    len(child), ptr(out), stream(out))
    else:
        st, ln = col.data[:, 0], col.data[:, 1]
        i = ptensor if ptensor is not None else torch.full((n,), int(pos), dtype=torch.int64)
        k = torch.where(i > 0, i - 1, ln + i)
        ok = (i != 0) & (k >= 0) & (k < ln)
        if col.valid is not None:
            ok &= col.valid
        if pos_valid is not None:
            ok &= pos_valid
        out = torch.where(ok, st + k, torch.full_like(st, -1))
    return take(child, out, neg=True)


def unnest_rows(col: Column) -> Tuple[torch.Tensor, Column]:
    """One output row per list element: (parent row per output row, the
    elements). NULL and empty lists produce no rows (DataFusion's unnest)."""
    from .gather import take
    from .hashing import expand_ranges
    n = len(col)
    lo = col.data[:, 0].contiguous() if n else torch.zeros(0, dtype=torch.int64, device=col.device)
    cnt = lengths(col)
    if col.valid is not None:
        cnt = torch.where(col.valid, cnt, torch.zeros_like(cnt))
    parent, cidx = expand_ranges(lo, cnt, len(col.nested.child))
    return parent, take(col.nested.child, cidx)


def unnest_values(col: Column, device) -> Column:
    return unnest_rows(col)[1]


def from_groups(child: Column, starts: torch.Tensor, counts: torch.Tensor, dtype: T.DataType,
                valid: Optional[torch.Tensor]) -> Column:
    """A list per group over a child already ordered by group (array_agg)."""
    se = torch.stack([starts.to(torch.int64), counts.to(torch.int64)], 1).contiguous()
    return Column(dtype, se, valid, dictionary=Nested(child=child))


def make_struct(names: Sequence[str], cols: Sequence[Column], n: int, dtype: T.DataType, device) -> Column:
    rid = torch.arange(n, dtype=torch.int64, device=torch.device(device))
    return Column(dtype, rid, None, dictionary=Nested(children=dict(zip(names, cols))))


def field(col: Column, name: str) -> Column:
    """get_field(s, 'name') / s['name']: NULL where the struct row is NULL."""
    from .gather import take
    ch = col.nested.children.get(name)
    if ch is None:
        raise ExecutionError(f"struct has no field '{name}'")
    idx = col.data
    if col.valid is not None:
        idx = torch.where(col.valid, idx, torch.full_like(idx, -1))
        return take(ch, idx, neg=True)
    return take(ch, idx)


def to_string(col: Column, sep: str, null_str: Optional[str] = None) -> Column:
    """array_to_string(l, sep [, null_str]) via the host (Arrow)."""
    vals = col.to_arrow().to_pylist()
    out = []
    for v in vals:
        if v is None:
            out.append(None)
            continue
        parts = [("" if x is None else str(x)) if null_str is not None or x is not None else None for x in v]
        if null_str is None:
            parts = [p for p, x in zip(parts, v) if x is not None]
        else:
            parts = [null_str if x is None else p for p, x in zip(parts, v)]
        out.append(sep.join(parts))
    return Column.from_arrow(pa.array(out, pa.large_string()), device=col.device)


def has(col: Column, value) -> Column:
    """array_has(l, x): some element equals x (NULL row -> NULL)."""
    from .hashing import expand_ranges
    n = len(col)
    dev = col.device
    child = col.nested.child
    if value is None:
        return Column(T.BOOL, torch.zeros(n, dtype=torch.bool, device=dev), torch.zeros(n, dtype=torch.bool,
                                                                                            device=dev))
    if child.dtype.is_string:
        from . import strings as S
        eq = S.in_list(child, [str(value)])
    else:
        eq = child.data == torch.as_tensor(value, dtype=child.data.dtype, device=dev)
    if child.valid is not None:
        eq = eq & child.valid
    cnt = lengths(col)
    if col.valid is not None:
        cnt = torch.where(col.valid, cnt, torch.zeros_like(cnt))
    p, c = expand_ranges(col.data[:, 0].contiguous() if n else cnt, cnt, len(child))
    hit = torch.zeros(n, dtype=torch.int64, device=dev)
    if p.numel():
        hit.index_add_(0, p.long(), eq.index_select(0, c.long()).to(torch.int64))
    return Column(T.BOOL, hit > 0, col.valid)
