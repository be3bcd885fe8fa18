"""Exchange operators for SPMD execution (one fragment slice per GPU).

Every operator of a query runs on every rank over that rank's slice; rows
move only at exchanges:

* hash shuffle — stable hash-partition kernel (csrc/kernels/partition.hip)
  + one RCCL all-to-all-v per column (co-locates join / group keys);
* broadcast — all-gather-v of the (small) build side of a join (SURVEY §2.4
  P6: hash-join build side replicated over xGMI);
* two-phase aggregation — local partial aggregate, shuffle of the (small)
  partial states by group key, final merge;
* gather — final results / sort inputs collected on every rank.

Distribution of a Batch is tracked in ``Batch.dist``: ``("hash", cid, ...)``
(rows placed by mix64(key) % world; after a co-partitioned equi-join every
column equal to the key is listed), ``("replicated",)`` or ``None``
(arbitrary).
Every decision is taken from globally reduced values, so all ranks issue the
same collectives in the same order.

Reference parity: FragmentType::Shuffle and GetDataForTask are declared but
unimplemented (reference crates/coordinator/src/fragment.rs:12,
crates/worker/src/service.rs:26-32); the DistributedPlanner places whole
tables on workers and runs joins centrally (distributed_planner.rs:44-92).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import torch

from .. import types as T
from ..columnar import Batch, Column
from ..ops.gather import gather_tensor
from ..ops import misc as M
from ..ops import strings as S
from ..ops.gather import take_many
from ..ops._lib import device_ints, to_host_ints
from ..sql import logical as L
from ..sql.expr import AggCall, ColRef, Expr
from ..utils.errors import NotSupported
from ..utils.log import get_logger

log = get_logger("exchange")
REPLICATED = ("replicated",)
DEFAULT_BROADCAST_ROWS = 4_000_000


def dist_of(b: Batch):
    return getattr(b, "dist", None)


def materialized(b: Batch) -> Batch:
    """A plain Batch for an exchange: late-materialised join results and lazy
    filtered scans (exec/operators.py LateBatch / _LazyScanBatch) gather their
    columns first."""
    if hasattr(b, "materialize"):
        return b.materialize()
    if type(b).__name__ == "_LazyScanBatch":
        return Batch(dict(b.columns.items()), b.num_rows, b.dist)
    return b


def hashed_on(d, cid) -> bool:
    """Rows placed by the hash of column ``cid`` (or a column equal to it)."""
    return cid is not None and bool(d) and d[0] == "hash" and cid in d[1:]


def with_dist(b: Batch, d) -> Batch:
    b.dist = d
    return b


# ------------------------------------------------------------------ key hashing
def partition_keys(c: Column) -> torch.Tensor:
    """Int64 per row whose mix64 decides the destination; identical for equal
    SQL values whatever the column representation (plain / dictionary)."""
    if c.dtype.is_string:
        if c.is_dict:
            dh = S.hash64(c.dictionary)
            k = gather_tensor(dh, c.data)
        else:
            k = S.hash64(c)
        if c.valid is not None:
            k = torch.where(c.valid, k, torch.zeros_like(k))
        return k.contiguous()
    x = c.data
    if x.dtype in (torch.float32, torch.float64):
        x = x.to(torch.float64)
        x = torch.where(x == 0, torch.zeros_like(x), x).view(torch.int64)
    elif x.dim() == 2:
        x = x[:, 0]
    elif x.dtype != torch.int64 and x.dtype != torch.int32:
        x = x.to(torch.int64)
    if c.valid is not None:
        x = torch.where(c.valid, x, torch.zeros_like(x))
    return x.contiguous()


# -------------------------------------------------------------- dictionary sync
def _dict_digest(d: Column) -> int:
    """Order-sensitive 63-bit digest of a dictionary's values (cached on it)."""
    h = d._unified
    if h is None:
        import hashlib
        hh = hashlib.blake2b(digest_size=8)
        for v in d.to_arrow().to_pylist():
            hh.update(b"\x00" if v is None else (v.encode() + b"\x01"))
        h = int.from_bytes(hh.digest(), "little") >> 1
        d._unified = h
    return h


def unify_dictionaries(cols: List[Column], comm, digests=None) -> List[Column]:
    """Make the codes of every dictionary column meaningful on every rank.
    One tiny all-gather of content digests for ALL dictionary columns (or the
    caller's, ``digests[rank][j]`` for the j-th dictionary column); only a
    column whose dictionaries differ between ranks gathers them (as a plain
    string column: offsets + bytes over the device collectives, no pickling)
    and re-codes through the union built on the device."""
    idx = [i for i, c in enumerate(cols) if c.is_dict]
    if not idx:
        return cols
    if digests is None:
        digests = comm.allgather_ints([_dict_digest(cols[i].dictionary) for i in idx])
    out = list(cols)
    for j, i in enumerate(idx):
        if all(d[j] == digests[0][j] for d in digests):
            continue
        c = cols[i]
        d = c.dictionary
        # same structure on every rank for the packed gather: plain, no validity
        mine = Column(T.UTF8, d.data, None, offsets=d.offsets) if d.is_plain_string else \
            Column(T.UTF8, S.decode(d).data, None, offsets=S.decode(d).offsets)
        counts = [x[0] for x in comm.allgather_ints([len(mine)])]
        every = _gather_column(mine, counts, comm)      # concatenation of all ranks' dictionaries
        enc = S.dict_encode(every)                      # union: codes into a deduplicated dictionary
        start = sum(counts[:comm.rank])
        remap = enc.data[start:start + len(mine)].to(torch.int32)
        codes = gather_tensor(remap, c.data) if len(mine) else c.data
        out[i] = Column(T.UTF8, codes, c.valid, dictionary=enc.dictionary)
    return out


def unify_dictionary(c: Column, comm) -> Column:
    return unify_dictionaries([c], comm)[0]


# ------------------------------------------------------ structural agreement
def _sig(c: Column) -> tuple:
    return (c.valid is not None, c.is_dict, c.is_plain_string, c.is_wide)


def normalize_structure(b: Batch, comm, extra: Sequence[int] = ()) -> Batch:
    """Make every rank's columns structurally identical (validity present,
    dictionary vs plain strings, 64- vs 128-bit decimals) so the packed
    collectives that follow line up across ranks, and give dictionary columns
    one shared code space. ONE all-gather carries every column's structure
    bits, every dictionary's content digest and the caller's ``extra`` ints
    (e.g. row counts); they come back as ``b.preamble[rank]``."""
    keys = list(b.columns)
    cols = [b.columns[k] for k in keys]
    bits = [sum(int(f) << i for i, f in enumerate(_sig(c))) for c in cols]
    digs = [_dict_digest(c.dictionary) if c.is_dict else 0 for c in cols]
    rows = comm.allgather_ints(list(extra) + bits + digs)
    ne, nk = len(extra), len(keys)
    sigs = [r[ne:ne + nk] for r in rows]
    out = {}
    for j, k in enumerate(keys):
        c = cols[j]
        if any(s[j] != sigs[0][j] for s in sigs):
            any_valid = any(s[j] & 1 for s in sigs)
            any_plain = any(s[j] & 4 for s in sigs)
            any_wide = any(s[j] & 8 for s in sigs)
            if any_plain and c.is_dict:
                c = S.decode(c)
            if any_wide and not c.is_wide and c.dtype.is_decimal:
                c = Column(c.dtype, torch.stack([c.data, c.data >> 63], 1), c.valid)
            if any_valid and c.valid is None:
                c = Column(c.dtype, c.data, torch.ones(len(c), dtype=torch.bool, device=c.device), c.offsets,
                           c.dictionary)
        out[k] = c
    # dictionary columns that stayed dictionary-coded everywhere
    dict_js = [j for j in range(nk) if out[keys[j]].is_dict]
    if dict_js:
        digests = [[r[ne + nk + j] for j in dict_js] for r in rows]
        unified = unify_dictionaries([out[keys[j]] for j in dict_js], comm, digests)
        for j, c in zip(dict_js, unified):
            out[keys[j]] = c
    nb = Batch(out, b.num_rows, b.dist)
    nb.preamble = [r[:ne] for r in rows]
    return nb


# --------------------------------------------------------------------- shuffle
def _fixed_parts(cols: List[Column]):
    """Per column the tensors that travel packed in one row matrix:
    validity bytes, dictionary codes / values, plain-string row lengths."""
    tensors, spec = [], []
    for c in cols:
        vi = None
        if c.valid is not None:
            vi = len(tensors)
            tensors.append(c.valid)
        di = len(tensors)
        if c.is_plain_string:
            tensors.append((c.offsets[1:] - c.offsets[:-1]).contiguous())
        else:
            tensors.append(c.data)
        spec.append((di, vi))
    return tensors, spec


def _rebuild(cols: List[Column], spec, parts: List[torch.Tensor], chars: Dict[int, torch.Tensor]) -> List[Column]:
    out = []
    for j, (c, (di, vi)) in enumerate(zip(cols, spec)):
        valid = parts[vi] if vi is not None else None
        if c.is_plain_string:
            lens = parts[di]
            if lens.numel():
                from ..ops.select import offsets_from_lengths
                off, _ = offsets_from_lengths(lens)
            else:
                off = torch.zeros(1, dtype=torch.int64, device=lens.device)
            out.append(Column(c.dtype, chars[j], valid, offsets=off))
        else:
            out.append(Column(c.dtype, parts[di], valid, dictionary=c.dictionary))
    return out


def shuffle(b: Batch, key: torch.Tensor, ctx, key_cid=None) -> Batch:
    """Hash-repartition rows of ``b`` by ``key`` across all ranks.

    Collectives: one all-to-all of the [rank x (rows, string bytes...)] count
    matrix, ONE all-to-all-v of every fixed-width column packed row-wise
    (gathered into destination order by the pack kernel itself), and one
    all-to-all-v of bytes per plain-string column."""
    from ..ops.gather import take
    from ..ops.pack import pack_rows, unpack_rows
    comm = ctx.comm
    W = comm.world_size
    b = normalize_structure(materialized(b), comm)
    perm, send = M.hash_partition(key, W)
    keys = list(b.columns)
    cols = [b.columns[k] for k in keys]
    tensors, spec = _fixed_parts(cols)
    # string bytes per destination (strings gathered into destination order)
    bounds = np.cumsum([0] + list(send)).tolist()
    sgath, sbytes = {}, []
    for j, c in enumerate(cols):
        if c.is_plain_string:
            g = take(c, perm)
            sgath[j] = g
            offs = to_host_ints(g.offsets.index_select(0, device_ints(bounds, g.offsets.device)))
            sbytes.append([offs[r + 1] - offs[r] for r in range(W)])
    mat = [[send[r]] + [sb[r] for sb in sbytes] for r in range(W)]
    rmat = comm.all_to_all_matrix(mat)
    recv = [r[0] for r in rmat]
    parts: List[torch.Tensor] = []
    if tensors:
        packed, lay = pack_rows(tensors, perm, b.num_rows)
        rpacked, _ = comm.all_to_all_v(packed, send, recv)
        parts = unpack_rows(rpacked, lay, tensors)
    chars = {}
    for k, (j, g) in enumerate(sgath.items()):
        chars[j], _ = comm.all_to_all_v(g.data, sbytes[k], [r[1 + k] for r in rmat])
    out = dict(zip(keys, _rebuild(cols, spec, parts, chars)))
    return with_dist(Batch(out, sum(recv)), ("hash", key_cid) if key_cid is not None else None)


def local_slice(b: Batch, key: torch.Tensor, ctx, key_cid=None) -> Batch:
    """This rank's hash partition of a REPLICATED batch, with no
    communication: every rank holds all rows, so each keeps those whose
    ``mix64(key) % world`` is its rank (the partition function of ``shuffle``).
    The result is co-partitioned with any batch shuffled on the same key."""
    from ..ops.gather import take_many as _take_many
    from ..ops.select import mask_to_indices
    comm = ctx.comm
    b = materialized(b)
    d = ("hash", key_cid) if key_cid is not None else None
    if comm.world_size == 1:
        return Batch(dict(b.columns), b.num_rows, d)
    idx = mask_to_indices(M.partition_ids(key, comm.world_size) == comm.rank)
    keys = list(b.columns)
    cols = _take_many([b.columns[k] for k in keys], idx)
    return Batch(dict(zip(keys, cols)), idx.numel(), d)


def _gather_column(c: Column, counts: List[int], comm) -> Column:
    """All-gather of one column (dictionaries must already agree)."""
    return _gather_columns([c], counts, comm)[0]


def _str_bytes(c: Column) -> int:
    return int(c.data.numel())


def _gather_columns(cols: List[Column], counts: List[int], comm,
                    str_bytes: Optional[List[List[int]]] = None) -> List[Column]:
    """All-gather of columns with agreeing structure: one packed all-gather-v
    of the fixed-width parts and ONE all-gather-v of every plain-string
    column's bytes concatenated (``str_bytes[rank][k]``: byte count of the
    k-th string column per rank, exchanged here when not given)."""
    from ..ops.pack import pack_rows, unpack_rows
    n = len(cols[0]) if cols else 0
    tensors, spec = _fixed_parts(cols)
    parts: List[torch.Tensor] = []
    if tensors:
        packed, lay = pack_rows(tensors, None, n)
        rpacked, _ = comm.all_gather_v(packed, counts)
        parts = unpack_rows(rpacked, lay, tensors)
    sj = [j for j, c in enumerate(cols) if c.is_plain_string]
    chars = {}
    if sj:
        if str_bytes is None:
            str_bytes = comm.allgather_ints([_str_bytes(cols[j]) for j in sj])
        local = cols[sj[0]].data if len(sj) == 1 else torch.cat([cols[j].data for j in sj])
        allb, _ = comm.all_gather_v(local, [sum(r) for r in str_bytes])
        pieces = {j: [] for j in sj}
        pos = 0
        for r in range(len(str_bytes)):
            for k, j in enumerate(sj):
                pieces[j].append(allb[pos:pos + str_bytes[r][k]])
                pos += str_bytes[r][k]
        for j in sj:
            chars[j] = pieces[j][0] if len(pieces[j]) == 1 else torch.cat(pieces[j])
    return _rebuild(cols, spec, parts, chars)


def gather_all(b: Batch, ctx) -> Batch:
    """Every rank receives the concatenation of all ranks' rows (one packed
    all-gather-v for the fixed-width columns)."""
    comm = ctx.comm
    if comm is None or not comm.spmd or dist_of(b) == REPLICATED:
        return b
    b = materialized(b)
    keys = list(b.columns)
    # string byte counts ride along in the preamble (-1: not a plain string
    # here; same length on every rank)
    pre = [b.num_rows] + [_str_bytes(b.columns[k]) if b.columns[k].is_plain_string else -1 for k in keys]
    b = normalize_structure(b, comm, pre)
    counts = [p[0] for p in b.preamble]
    cols = [b.columns[k] for k in keys]
    sj = [j for j, c in enumerate(cols) if c.is_plain_string]
    sb = [[p[1 + j] for j in sj] for p in b.preamble]
    if any(x < 0 for r in sb for x in r):
        sb = None   # a dictionary column was decoded by normalisation: exchange its byte counts
    out = dict(zip(keys, _gather_columns(cols, counts, comm, sb))) if keys else {}
    return with_dist(Batch(out, sum(counts)), REPLICATED)


# ----------------------------------------------------------------------- joins
def _cid(e: Expr):
    return e.cid if isinstance(e, ColRef) else None


def prepare_join(lb: Batch, rb: Batch, join: L.Join, ctx, rows: Optional[Tuple[int, int]] = None):
    """Move rows so the join can run rank-locally; returns (lb, rb) with the
    output distribution stored in ``lb.out_dist``. ``rows``: the inputs'
    global row counts when the caller already reduced them."""
    from ..exec.operators import _pair_key
    comm = ctx.comm
    kind, on = join.kind, join.on
    ld, rd = dist_of(lb), dist_of(rb)
    rep_l, rep_r = ld == REPLICATED, rd == REPLICATED
    limit = int(ctx.engine.session.get("broadcast_rows", DEFAULT_BROADCAST_ROWS)) if ctx.engine else DEFAULT_BROADCAST_ROWS

    def done(l, r, d):
        l.out_dist = d
        return l, r

    if rep_l and rep_r:
        return done(lb, rb, REPLICATED)
    if on:
        for le, re_ in on:
            lc, rc = _cid(le), _cid(re_)
            if hashed_on(ld, lc) and hashed_on(rd, rc):
                # co-partitioned: rank-local; the output is placed by both keys
                return done(lb, rb, ld + tuple(c for c in rd[1:] if c not in ld))
    if kind in ("inner", "cross") and (rep_l or rep_r):
        return done(lb, rb, rd if rep_l else ld)
    if kind in ("left", "semi", "anti") and rep_r:
        return done(lb, rb, ld)
    # global sizes decide broadcast vs shuffle (a replicated side counts once)
    if rows is not None:
        nl, nr = rows
    else:
        nl, nr = comm.allreduce_ints([lb.num_rows if not rep_l else 0, rb.num_rows if not rep_r else 0])
    if rep_l:
        nl = lb.num_rows
    if rep_r:
        nr = rb.num_rows
    null_aware = getattr(join, "null_aware", False)
    if kind in ("inner", "cross"):
        if rep_r:
            return done(lb, rb, ld)
        if rep_l:
            return done(lb, rb, rd)
        if not on or min(nl, nr) <= limit:
            if nr <= nl:
                return done(lb, gather_all(rb, ctx), ld)
            return done(gather_all(lb, ctx), rb, rd)
    if kind in ("left", "semi", "anti"):
        if rep_r and not rep_l:
            return done(lb, rb, ld)
        if (nr <= limit or null_aware or not on) and not rep_l:
            return done(lb, gather_all(rb, ctx), ld)
        if rep_l and (nr <= limit or null_aware or not on):
            # preserved side replicated, small other side: bring everything together
            return done(lb, gather_all(rb, ctx), REPLICATED)
        # preserved side replicated, large other side (TPC-H Q13 / Q22:
        # customer against orders): each rank keeps its hash slice of the
        # replicated side (no exchange) and the other side is shuffled below
    if not on:
        return done(gather_all(lb, ctx), gather_all(rb, ctx), REPLICATED)
    # hash shuffle both sides on the first key pair (a replicated side is
    # sliced locally instead: shuffling it would multiply its rows)
    ev = ctx.evaluator
    le, re_ = on[0]
    lcol, rcol = ev.column(le, lb), ev.column(re_, rb)
    if lcol.dtype.is_string or rcol.dtype.is_string:
        lk, rk = partition_keys(lcol), partition_keys(rcol)
    else:
        lk, rk = _pair_key(lcol, rcol)
        lk, rk = lk.to(torch.int64).contiguous(), rk.to(torch.int64).contiguous()
    lc, rc = _cid(le), _cid(re_)
    if rep_l:
        lb = local_slice(lb, lk, ctx, lc)
    elif not (hashed_on(ld, lc) and lcol.dtype == rcol.dtype):
        lb = shuffle(lb, lk, ctx, lc)
    if rep_r:
        rb = local_slice(rb, rk, ctx, rc)
    elif not (hashed_on(rd, rc) and lcol.dtype == rcol.dtype):
        rb = shuffle(rb, rk, ctx, rc)
    return done(lb, rb, ("hash",) + tuple(c for c in (lc, rc) if c is not None) if lc is not None else None)


#: largest global key span a semi / anti join filters through a dense
#: key-presence table (bytes, all-reduced)
KEYSET_MAX_SPAN = 1 << 27


def semi_by_key_set(lb: Batch, rb: Batch, join: L.Join, ctx) -> Optional[Batch]:
    """SEMI / ANTI join of a REPLICATED left side against a partitioned right
    side (TPC-H Q22: customer NOT EXISTS orders) with no row movement: every
    rank marks the keys of its right rows in a dense presence table over the
    global key range, ONE all-reduce (max) makes it the global key set, and
    each rank filters its replicated left rows locally — the result stays
    replicated. Two collectives (key range, presence table) instead of
    slicing the left side and shuffling the right side. None when the shape
    does not apply."""
    from ..exec.operators import _pair_key
    from ..ops.select import mask_to_indices
    comm = ctx.comm
    if join.kind not in ("semi", "anti") or len(join.on or []) != 1 or join.residual is not None \
            or getattr(join, "null_aware", False):
        return None
    if dist_of(lb) != REPLICATED or dist_of(rb) == REPLICATED:
        return None
    ev = ctx.evaluator
    le, re_ = join.on[0]
    lcol, rcol = ev.column(le, lb), ev.column(re_, rb)
    if lcol.dtype.is_string or rcol.dtype.is_string or lcol.data.dim() != 1 or rcol.data.dim() != 1 \
            or not (lcol.dtype.is_integer or lcol.dtype.kind == "date32") \
            or not (rcol.dtype.is_integer or rcol.dtype.kind == "date32"):
        return None
    lk, rk = _pair_key(lcol, rcol)
    lk, rk = lk.to(torch.int64), rk.to(torch.int64)
    if rcol.valid is not None:
        rk = gather_tensor(rk, mask_to_indices(rcol.valid))
    from ..ops import hashing as H
    rng = H.key_range(rk) if rk.numel() else None
    lo_hi = comm.allgather_ints([rng[0], rng[1]] if rng else [2**62, -2**62])
    g0, g1 = min(r[0] for r in lo_hi), max(r[1] for r in lo_hi)
    span = g1 - g0 + 1 if g0 <= g1 else 0
    if span > KEYSET_MAX_SPAN:
        return None     # every rank decides alike (global range)
    present = torch.zeros(max(span, 1), dtype=torch.uint8, device=ctx.device)
    if rk.numel():
        present.index_fill_(0, rk - g0, 1)
    present = comm.allreduce_tensor(present, "max")
    li = lk - g0
    inr = (li >= 0) & (li < span)
    hit = inr & (present.index_select(0, torch.where(inr, li, torch.zeros_like(li))) > 0)
    if lcol.valid is not None:
        hit &= lcol.valid
    keep = mask_to_indices(hit if join.kind == "semi" else ~hit)
    keys = list(lb.columns)
    out = Batch(dict(zip(keys, take_many([lb.columns[k] for k in keys], keep))), int(keep.numel()), REPLICATED)
    return out


# ------------------------------------------------------------------ aggregation
DECOMPOSABLE = {"sum", "count", "min", "max", "avg", "bool_and", "bool_or"}


def distributed_aggregate(lg: L.Aggregate, b: Batch, ctx, local=None) -> Batch:
    """``local(groups, partial_aggs) -> Batch | None`` may compute the phase-1
    partial states directly from the scan (fused VM kernel)."""
    from ..exec.operators import aggregate
    groups, aggs = lg.groups, lg.aggs
    d = dist_of(b)
    if d == REPLICATED:
        return with_dist(aggregate(groups, aggs, b, ctx), REPLICATED)
    if d and d[0] == "hash":
        for ci, e in groups:
            if isinstance(e, ColRef) and hashed_on(d, e.cid):
                return with_dist(aggregate(groups, aggs, b, ctx), ("hash", ci.cid))
    ev = ctx.evaluator
    if not decomposable(aggs):
        if groups:
            k = partition_keys(ev.column(groups[0][1], b))
            sb = shuffle(b, k, ctx)
            return with_dist(aggregate(groups, aggs, sb, ctx), ("hash", groups[0][0].cid))
        return with_dist(aggregate(groups, aggs, gather_all(b, ctx), ctx), REPLICATED)
    # ---- phase 1: partial states
    ids = _TmpIds()
    partial, plan = partial_plan(aggs, ids)
    pb = local(groups, partial) if local is not None else None
    if pb is None:
        pb = aggregate(groups, partial, b, ctx)
    # ---- exchange partial states: all-reduce over a small dense key domain
    # (global aggregates, dictionary-coded group keys) else hash shuffle
    rb = _dense_allreduce(groups, partial, pb, ctx)
    out_dist = REPLICATED if rb is not None else None
    if rb is None and groups:
        g0 = groups[0][0]
        rb = shuffle(pb, partition_keys(pb.columns[g0.cid]), ctx, g0.cid)
    elif rb is None:
        rb = gather_all(pb, ctx)
        out_dist = REPLICATED
    # ---- phase 2: merge
    res = merge_partials(groups, plan, rb, ids, ctx)
    return with_dist(res, out_dist if out_dist is not None else ("hash", groups[0][0].cid))


def decomposable(aggs) -> bool:
    """Every aggregate merges from partial states (two-phase aggregation)."""
    return all(a.func in DECOMPOSABLE and not a.distinct for _, a in aggs)


def partial_plan(aggs, ids):
    """Phase-1 aggregates whose states merge into ``aggs`` (AVG -> SUM + COUNT)
    and the plan ``merge_partials`` follows. Shared by the SPMD exchange and the
    morsel pipeline (exec/morsel.py), whose partial states come from ranks and
    morsels respectively."""
    partial, plan = [], []
    for ci, a in aggs:
        if a.func == "avg":
            st = _sum_type(a.arg.dtype)
            s_ci = L.ColInfo(ids(), "__ps", st)
            c_ci = L.ColInfo(ids(), "__pc", T.INT64)
            partial += [(s_ci, AggCall("sum", a.arg, False, st, a.filter)), (c_ci, AggCall("count", a.arg, False, T.INT64, a.filter))]
            plan.append(("avg", ci, a, s_ci, c_ci))
        else:
            p_ci = L.ColInfo(ids(), "__p", a.dtype)
            partial.append((p_ci, AggCall(a.func, a.arg, False, a.dtype, a.filter)))
            plan.append((a.func, ci, a, p_ci, None))
    return partial, plan


def merge_partials(groups, plan, rb: Batch, ids, ctx) -> Batch:
    """Phase 2: merge the partial states in ``rb`` (rows = partial groups) into
    the final aggregates of ``plan`` (see ``partial_plan``)."""
    from ..exec.operators import _avg, aggregate
    fgroups = [(ci, ColRef(ci.cid, ci.name, ci.dtype, ci.nullable)) for ci, _ in groups]
    # 128-bit partial sums (wide decimals: SF100 charges) merge as three
    # int64 sums — high word, and the low word's two 32-bit halves — that
    # cannot overflow, recombined into 128 bits after the merge
    rb, wide_parts = _split_wide_partials(rb, plan, ids)
    final, post = [], []
    for func, ci, a, p1, p2 in plan:
        if func == "avg":
            fs = L.ColInfo(ids(), "__fs", p1.dtype)
            fc = L.ColInfo(ids(), "__fc", T.INT64)
            final += [(fs, AggCall("sum", p1.ref(), False, p1.dtype)), (fc, AggCall("sum", p2.ref(), False, T.INT64))]
            post.append(("avg", ci, a, fs, fc))
        elif func == "count":
            final.append((ci, AggCall("sum", p1.ref(), False, T.INT64)))
            post.append(("count", ci, a, None, None))
        else:
            merge = {"sum": "sum", "min": "min", "max": "max", "bool_and": "bool_and", "bool_or": "bool_or"}[func]
            final.append((ci, AggCall(merge, p1.ref(), False, a.dtype)))
            post.append((func, ci, a, None, None))
    final, recombine = _wide_finals(final, wide_parts, ids)
    fb = aggregate(fgroups, final, rb, ctx)
    fb = _join_wide_finals(fb, recombine)
    out = {ci.cid: fb.columns[ci.cid] for ci, _ in groups}
    for func, ci, a, fs, fc in post:
        if func == "avg":
            s, c = fb.columns[fs.cid], fb.columns[fc.cid]
            cnt = c.data if c.valid is None else torch.where(c.valid, c.data, torch.zeros_like(c.data))
            out[ci.cid] = Column(a.dtype, _avg(s.data, cnt, a.arg.dtype, a.dtype), cnt > 0)
        elif func == "count":
            c = fb.columns[ci.cid]
            data = c.data if c.valid is None else torch.where(c.valid, c.data, torch.zeros_like(c.data))
            out[ci.cid] = Column(T.INT64, data)
        else:
            out[ci.cid] = fb.columns[ci.cid]
    return Batch(out, fb.num_rows)


#: largest dense group-key domain whose partial states are all-reduced
DENSE_ALLREDUCE_MAX = 4096
_I64_MAX, _I64_MIN = 2**63 - 1, -2**63


def _dense_allreduce(groups, partial, pb: Batch, ctx) -> Optional[Batch]:
    """Two-phase aggregation over a small dense key domain (no GROUP BY, or
    dictionary-coded / boolean group keys whose dictionary sizes multiply to
    at most DENSE_ALLREDUCE_MAX, e.g. TPC-H Q1's returnflag x linestatus):
    every rank scatters its partial states into dense per-key arrays and ONE
    all-reduce per reduction op (SUM / MIN / MAX) merges them — no shuffle,
    and the result is replicated on every rank (so a following ORDER BY needs
    no gather). Returns the merged partial-state batch or None when the shape
    does not apply (128-bit sums, strings, large domains)."""
    comm = ctx.comm
    dev = ctx.device
    cols = [pb.columns[ci.cid] for ci, _ in partial]
    for (ci, a), c in zip(partial, cols):
        if a.func not in ("sum", "count", "min", "max", "bool_and", "bool_or") or c.is_wide or c.dtype.is_string \
                or c.data.dim() != 1:
            return None
    # group keys -> dense index (structure agreement first: every rank decides alike)
    keys = [pb.columns[ci.cid] for ci, _ in groups]
    if any(not (k.is_dict or k.dtype.kind == "bool") for k in keys):
        return None
    sig = comm.allgather_ints([int(k.valid is not None) for k in keys] + [int(pb.num_rows)])
    nullable = [any(r[j] for r in sig) for j in range(len(keys))]
    keys = unify_dictionaries(keys, comm) if keys else keys
    sizes = [(len(k.dictionary) if k.is_dict else 2) + (1 if nullable[j] else 0) for j, k in enumerate(keys)]
    domain = 1
    for z in sizes:
        domain *= max(z, 1)
    if domain > DENSE_ALLREDUCE_MAX:
        return None
    n = pb.num_rows
    idx = torch.zeros(n, dtype=torch.int64, device=dev)
    for j, k in enumerate(keys):
        code = k.data.to(torch.int64)
        if nullable[j] and k.valid is not None:
            code = torch.where(k.valid, code, torch.full_like(code, sizes[j] - 1))
        idx = idx * sizes[j] + code
    isum, fsum, imin, imax, fmin, fmax = [], [], [], [], [], []

    def dense(vals, fill, dtype):
        d = torch.full((domain,), fill, dtype=dtype, device=dev)
        if n:
            d.index_put_((idx,), vals.to(dtype), accumulate=False)
        return d

    presence = dense(torch.ones(n, dtype=torch.int64, device=dev), 0, torch.int64)
    isum.append(presence)
    slots = []
    for (ci, a), c in zip(partial, cols):
        isf = c.data.dtype in (torch.float32, torch.float64)
        valid = c.valid if c.valid is not None else torch.ones(n, dtype=torch.bool, device=dev)
        vcount = dense(valid.to(torch.int64), 0, torch.int64)
        isum.append(vcount)
        if a.func in ("sum", "count"):
            v = torch.where(valid, c.data, torch.zeros_like(c.data))
            lst = fsum if isf else isum
            lst.append(dense(v, 0, torch.float64 if isf else torch.int64))
        else:
            is_min = a.func in ("min", "bool_and")
            fill = (float("inf") if is_min else float("-inf")) if isf else (_I64_MAX if is_min else _I64_MIN)
            v = torch.where(valid, c.data.to(torch.float64 if isf else torch.int64),
                            torch.full((n,), fill, dtype=torch.float64 if isf else torch.int64, device=dev))
            lst = (fmin if is_min else fmax) if isf else (imin if is_min else imax)
            lst.append(dense(v, fill, torch.float64 if isf else torch.int64))
        slots.append((lst, len(lst) - 1, len(isum) - 1))
    red = {}
    for name, lst, op in (("isum", isum, "sum"), ("fsum", fsum, "sum"), ("imin", imin, "min"), ("imax", imax, "max"),
                          ("fmin", fmin, "min"), ("fmax", fmax, "max")):
        if lst:
            red[id(lst)] = comm.allreduce_tensor(torch.stack(lst), op)
    present = mask_idx = None
    tot = red[id(isum)]
    from ..ops.select import mask_to_indices
    mask_idx = mask_to_indices(tot[0] > 0)
    m = mask_idx.numel()
    out = {}
    rest = mask_idx.to(torch.int64)
    for j in range(len(keys) - 1, -1, -1):
        code = rest % sizes[j]
        rest = rest // sizes[j]
        k = keys[j]
        valid = None
        if nullable[j]:
            valid = code != sizes[j] - 1
            code = torch.where(valid, code, torch.zeros_like(code))
        ci = groups[j][0]
        if k.is_dict:
            out[ci.cid] = Column(k.dtype, code.to(torch.int32), valid, dictionary=k.dictionary)
        else:
            out[ci.cid] = Column(k.dtype, code.to(torch.bool), valid)
    for ((ci, a), c), (lst, li, vi) in zip(zip(partial, cols), slots):
        vals = gather_tensor(red[id(lst)][li], mask_idx)
        has = gather_tensor(tot[vi], mask_idx) > 0
        if a.func == "count":
            out[ci.cid] = Column(c.dtype, vals.to(torch.int64))
        else:
            data = vals.to(c.data.dtype) if c.dtype.kind != "bool" else vals != 0
            out[ci.cid] = Column(c.dtype, torch.where(has, data, torch.zeros_like(data)), has)
    return Batch(out, m)


def _split_wide_partials(rb: Batch, plan, ids):
    """Replace every 128-bit partial-sum column of ``rb`` by three int64
    columns (hi, lo >> 32, lo & 0xFFFFFFFF as unsigned halves); returns
    (batch, {partial cid: (hi, mid, low) ColInfos})."""
    wide = {}
    cols = None
    for func, ci, a, p1, p2 in plan:
        c = rb.columns.get(p1.cid)
        if c is None or not c.is_wide:
            continue
        if cols is None:
            cols = dict(rb.columns)
        lo, hi = c.data[:, 0], c.data[:, 1]
        parts = (L.ColInfo(ids(), "__whi", T.INT64), L.ColInfo(ids(), "__wmid", T.INT64),
                 L.ColInfo(ids(), "__wlow", T.INT64))
        for pc, t in zip(parts, (hi, (lo >> 32) & 0xFFFFFFFF, lo & 0xFFFFFFFF)):
            cols[pc.cid] = Column(T.INT64, t.contiguous(), c.valid)
        wide[p1.cid] = parts
    if cols is None:
        return rb, wide
    return Batch(cols, rb.num_rows, rb.dist), wide


def _wide_finals(final, wide, ids):
    """Merge aggregates with every SUM over a wide partial replaced by the
    three int64 SUMs of its parts; returns (aggregates, recombination list)."""
    if not wide:
        return final, []
    out, rec = [], []
    for ci, call in final:
        arg = call.arg
        if call.func == "sum" and isinstance(arg, ColRef) and arg.cid in wide:
            fs = [L.ColInfo(ids(), n, T.INT64) for n in ("__mhi", "__mmid", "__mlow")]
            out += [(f, AggCall("sum", p.ref(), False, T.INT64)) for f, p in zip(fs, wide[arg.cid])]
            rec.append((ci, fs))
        else:
            out.append((ci, call))
    return out, rec


def _join_wide_finals(fb: Batch, rec) -> Batch:
    """hi * 2^64 + mid * 2^32 + low -> one 128-bit (lo, hi) column per merged
    wide sum (mid, low >= 0 and < 2^63: sums of fewer than 2^31 32-bit halves)."""
    if not rec:
        return fb
    cols = dict(fb.columns)
    sign = -(2**63)
    for ci, (fh, fm, fl) in rec:
        hc = cols.pop(fh.cid)
        mid, low = cols.pop(fm.cid).data, cols.pop(fl.cid).data
        hi = hc.data
        lo = low + ((mid & 0xFFFFFFFF) << 32)                     # wraps as uint64
        carry = ((lo ^ sign) < (low ^ sign)).to(torch.int64)      # unsigned overflow of that add
        cols[ci.cid] = Column(ci.dtype, torch.stack([lo, hi + (mid >> 32) + carry], 1).contiguous(), hc.valid)
    return Batch(cols, fb.num_rows, fb.dist)


def _sum_type(t):
    if t.is_decimal:
        return T.DECIMAL(min(38, t.precision + 10), t.scale)
    if t.is_float:
        return T.FLOAT64
    return T.INT64


class _TmpIds:
    """Temporary column ids for partial states (negative: never collide with binder ids)."""
    _n = 0

    def __call__(self) -> int:
        _TmpIds._n -= 1
        return _TmpIds._n
