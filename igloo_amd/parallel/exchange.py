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
    filtered scans (exec/joins.py LateBatch, exec/scan.py _LazyScanBatch) gather their
    columns first."""
    if hasattr(b, "materialize"):
        return b.materialize()
    if type(b).__name__ == "_LazyScanBatch":
        return Batch(dict(b.columns.items()), b.num_rows, b.dist)
    return b


def hashed_on(d, cid) -> bool:
    """Rows placed by the hash of column ``cid`` (or a column equal to it)."""
    return cid is not None and bool(d) and d[0] == "hash" and cid in d[1:]


def keyed(d) -> bool:
    """A placement by the value of its key columns ``d[1:]``: hash
    (("hash", cid, ...)) or key range ((("range", world, kmin, chunk), cid,
    ...), parallel/slicing.py)."""
    return bool(d) and (d[0] == "hash" or (isinstance(d[0], tuple) and d[0][0] == "range"))


def placed_on(d, cid) -> bool:
    """All rows with one value of column ``cid`` live on one rank."""
    return cid is not None and keyed(d) and cid in d[1:]


def copartitioned(ld, lc, rd, rc) -> bool:
    """Equal values of ``lc`` (left) and ``rc`` (right) live on the same rank:
    both placed by those columns with the same mapping."""
    return placed_on(ld, lc) and placed_on(rd, rc) and ld[0] == rd[0]


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
_GOLDEN = -0x61C8864680B583EB          # 0x9E3779B97F4A7C15 as int64
_MIX1, _MIX2 = -0x40A7B892E31B1A47, -0x6B2FB644ECCEEE15


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 (wrapping arithmetic, logical shifts)."""
    m = (1 << 64) - 1
    def srl(v, k):
        return (v >> k) & ((m >> k) if k else m)
    x = (x ^ srl(x, 30)) * _MIX1
    x = (x ^ srl(x, 27)) * _MIX2
    return x ^ srl(x, 31)


def _dict_digest(d: Column) -> int:
    """Order-sensitive 63-bit digest of a dictionary's values (cached on it):
    the per-entry string hashes (ops/strings.py hash64: the str_hash64 kernel
    on the GPU) mixed with their positions and summed on the device -- one
    8-byte readback, no host copy of the dictionary."""
    h = d._unified
    if h is None:
        from ..ops._lib import unlogged
        n = len(d)
        if n == 0:
            h = 0
        else:
            if d.is_dict:
                d = S.decode(d)
            hv = S.hash64(d)
            if d.valid is not None:
                hv = torch.where(d.valid, hv, torch.full_like(hv, 0x5bd1e995))
            pos = torch.arange(n, dtype=torch.int64, device=hv.device) * _GOLDEN
            tot = _mix64(hv ^ pos).sum().reshape(1) + n
            with unlogged():
                h = to_host_ints(tot)[0] & ((1 << 63) - 1)
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


def _no_nested(cols) -> None:
    """LIST / STRUCT rows are views into per-rank child columns: they do not
    travel in the packed collectives (single-rank engines evaluate them)."""
    for c in cols:
        if c.dtype.is_nested:
            raise NotSupported(f"{c.dtype} columns cannot be exchanged between ranks")


def normalize_structure(b: Batch, comm, extra: Sequence[int] = ()) -> Batch:
    """Make every rank's columns structurally identical (validity present,
    dictionary vs plain strings, 64- vs 128-bit decimals) so the packed
    collectives that follow line up across ranks, and give dictionary columns
    one shared code space. ONE all-gather carries every column's structure
    bits, every dictionary's content digest and the caller's ``extra`` ints
    (e.g. row counts); they come back as ``b.preamble[rank]``."""
    keys = wire_order(b)
    cols = [b.columns[k] for k in keys]
    _no_nested(cols)
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
                off, _ = offsets_from_lengths(lens, host_total=False)
            else:
                off = torch.zeros(1, dtype=torch.int64, device=lens.device)
            out.append(Column(c.dtype, chars[j], valid, offsets=off))
        else:
            out.append(Column(c.dtype, parts[di], valid, dictionary=c.dictionary))
    return out


def _split_bytes(buf: torch.Tensor, sizes: List[int]) -> List[torch.Tensor]:
    """Consecutive pieces of a byte buffer (views)."""
    out, pos = [], 0
    for z in sizes:
        out.append(buf[pos:pos + z])
        pos += z
    return out


class ShufflePlan:
    """Where this rank's rows go: the stable permutation grouping them by
    destination, rows per destination, the plain-string columns gathered into
    that order and their byte counts per destination. Built before the
    structure all-gather when the caller can ship it in that all-gather's
    preamble (``preamble``/``receive``): the shuffle then needs no count
    exchange of its own."""

    def __init__(self, b: Batch, key: torch.Tensor, W: int):
        from ..ops.gather import take
        self.W = W
        n = key.numel()
        self.perm, self.send = M.hash_partition(key, W) if n else \
            (torch.zeros(0, dtype=torch.int32, device=key.device), [0] * W)
        cols = [b.columns[k] for k in wire_order(b)]       # (positions j: the shuffle's column order)
        self.bounds = np.cumsum([0] + list(self.send)).tolist()
        self.sgath = {j: take(c, self.perm) for j, c in enumerate(cols) if c.is_plain_string}
        self.sbytes: List[List[int]] = []
        if self.sgath and not n:
            self.sbytes = [[0] * W for _ in self.sgath]
        elif self.sgath:
            bidx = device_ints(self.bounds, key.device)
            offs = to_host_ints(torch.cat([g.offsets.index_select(0, bidx).to(torch.int64)
                                           for g in self.sgath.values()]))
            for k in range(len(self.sgath)):
                o = offs[k * (W + 1):(k + 1) * (W + 1)]
                self.sbytes.append([o[r + 1] - o[r] for r in range(W)])
        self.str_cols = [j for j, c in enumerate(cols) if c.dtype.is_string]
        self.rmat: Optional[List[List[int]]] = None
        self.full_max: Optional[int] = None

    def matrix(self) -> List[List[int]]:
        return [[self.send[r]] + [sb[r] for sb in self.sbytes] for r in range(self.W)]

    def preamble(self) -> List[int]:
        """Fixed-length ints (same on every rank): per destination the row
        count and every string column's bytes (-1: dictionary here)."""
        by = {j: sb for j, sb in zip(self.sgath, self.sbytes)}
        out = []
        for r in range(self.W):
            out.append(self.send[r])
            out += [by[j][r] if j in by else -1 for j in self.str_cols]
        return out

    @staticmethod
    def width(b: Batch, W: int) -> int:
        return W * (1 + sum(1 for c in b.columns.values() if c.dtype.is_string))

    def receive(self, pre: List[List[int]], rank: int, nb: Batch) -> bool:
        """The count matrix from every rank's ``preamble`` (``pre[r]``);
        False when a string column is plain on some ranks and dictionary-
        coded on others (normalisation decoded it: byte counts unknown)."""
        ns = len(self.str_cols)
        cols = [nb.columns[k] for k in wire_order(nb)]
        plain_now = [j for j in self.str_cols if cols[j].is_plain_string]
        if plain_now != list(self.sgath):
            return False
        rmat = []
        # every rank's rows per destination (the whole count matrix, known
        # alike on every rank: a pipelined exchange sizes its chunks from it)
        self.full_max = max((pre[r][d * (1 + ns)] for r in range(self.W) for d in range(self.W)), default=0)
        for r in range(self.W):
            blk = pre[r][rank * (1 + ns):(rank + 1) * (1 + ns)]
            bys = [blk[1 + t] for t, j in enumerate(self.str_cols) if j in self.sgath]
            if any(x < 0 for x in bys):
                return False
            rmat.append([blk[0]] + bys)
        self.rmat = rmat
        return True


def shuffle(b: Batch, key: torch.Tensor, ctx, key_cid=None, normalized: bool = False,
            plan: Optional[ShufflePlan] = None) -> Batch:
    """Hash-repartition rows of ``b`` by ``key`` across all ranks.

    Collectives: the structure all-gather (skipped when the caller already
    ``normalized`` the batch; otherwise it also carries every rank's count
    matrix row), one all-to-all of the [rank x (rows, string bytes...)] count
    matrix only when neither did (or a string column changed representation
    in the normalisation), and ONE all-to-all-v of bytes:
    per destination the packed fixed-width rows (gathered into destination
    order by the pack kernel itself) followed by every plain-string column's
    bytes."""
    from ..ops.pack import pack_rows, unpack_rows
    comm = ctx.comm
    W = comm.world_size
    if not normalized:
        # the count matrix rides in the structure all-gather's preamble
        b = materialized(b)
        plan = ShufflePlan(b, key, W)
        b = normalize_structure(b, comm, plan.preamble())
        if not plan.receive(b.preamble, comm.rank, b):
            plan = None
    if plan is None or plan.rmat is None:
        plan = ShufflePlan(b, key, W)
        plan.rmat = comm.all_to_all_matrix(plan.matrix())
    perm, send, bounds, sgath, sbytes, rmat = plan.perm, plan.send, plan.bounds, plan.sgath, plan.sbytes, plan.rmat
    keys = wire_order(b)
    cols = [b.columns[k] for k in keys]
    tensors, spec = _fixed_parts(cols)
    recv = [r[0] for r in rmat]
    if not sgath and tensors and plan.full_max is not None and W > 1 and \
            plan.full_max * sum(t.element_size() * (t.shape[1] if t.dim() == 2 else 1) for t in tensors) \
            > PIPELINE_MIN_BYTES:
        from ..ops._lib import capturing
        if not capturing():
            parts = _pipelined_exchange(tensors, plan, comm)
            out = dict(zip(keys, _rebuild(cols, spec, parts, {})))
            return with_dist(Batch(out, sum(recv)), ("hash", key_cid) if key_cid is not None else None)
    packed, lay = pack_rows(tensors, perm, b.num_rows) if tensors else (None, (0, []))
    rb = lay[0]
    if not sgath:
        parts: List[torch.Tensor] = []
        if tensors:
            rpacked, _ = comm.all_to_all_v(packed, send, recv)
            parts = unpack_rows(rpacked, lay, tensors)
        out = dict(zip(keys, _rebuild(cols, spec, parts, {})))
        return with_dist(Batch(out, sum(recv)), ("hash", key_cid) if key_cid is not None else None)
    # one byte stream per destination: [rows | string column 1 | string column 2 ...]
    flat = packed.reshape(-1) if packed is not None else None
    pieces, send_b = [], []
    for r in range(W):
        if flat is not None:
            pieces.append(flat[bounds[r] * rb:bounds[r + 1] * rb])
        for k, g in enumerate(sgath.values()):
            lo = sum(sbytes[k][:r])
            pieces.append(g.data[lo:lo + sbytes[k][r]])
        send_b.append(send[r] * rb + sum(sb[r] for sb in sbytes))
    recv_b = [rmat[r][0] * rb + sum(rmat[r][1:]) for r in range(W)]
    buf, _ = comm.all_to_all_v(torch.cat(pieces) if pieces else torch.zeros(0, dtype=torch.uint8, device=key.device),
                               send_b, recv_b)
    row_parts, str_parts = [], [[] for _ in sgath]
    for r, blk in enumerate(_split_bytes(buf, recv_b)):
        sizes = [rmat[r][0] * rb] + list(rmat[r][1:])
        sp = _split_bytes(blk, sizes)
        row_parts.append(sp[0])
        for k in range(len(sgath)):
            str_parts[k].append(sp[1 + k])
    parts = []
    if tensors:
        rows = torch.cat(row_parts) if len(row_parts) > 1 else row_parts[0]
        parts = unpack_rows(rows.view(-1, rb) if rb else rows.view(0, 0), lay, tensors)
    chars = {j: (torch.cat(str_parts[k]) if len(str_parts[k]) > 1 else str_parts[k][0])
             for k, j in enumerate(sgath)}
    out = dict(zip(keys, _rebuild(cols, spec, parts, chars)))
    return with_dist(Batch(out, sum(recv)), ("hash", key_cid) if key_cid is not None else None)


#: a fixed-width shuffle whose largest (sender, destination) block exceeds this
#: many bytes is pipelined in chunks of PIPELINE_CHUNK_BYTES per rank
PIPELINE_MIN_BYTES = 256 << 20
PIPELINE_CHUNK_BYTES = 64 << 20


def _pipelined_exchange(tensors: List[torch.Tensor], plan: ShufflePlan, comm) -> List[torch.Tensor]:
    """The rows of a large fixed-width shuffle in chunks: chunk j carries rows
    [j*C, (j+1)*C) of every (sender, destination) block. While chunk j moves
    (an asynchronous all-to-all-v), chunk j+1 is packed and chunk j-1 is
    placed into the assembled receive buffer -- pack, transfer and unpack of
    consecutive chunks overlap instead of running as three full-size
    barriers. The chunk count follows from the whole count matrix (the
    structure all-gather carried it), so every rank issues the same
    collectives. Rows come out in the unchunked order (by sender, then send
    order). Returns the unpacked tensors."""
    from ..ops.pack import layout, pack_rows, unpack_rows
    W = plan.W
    lay = layout(tensors)
    rb = lay[0]
    send, recv = plan.send, [r[0] for r in plan.rmat]
    C = max(1, PIPELINE_CHUNK_BYTES // max(rb * W, 1))
    nchunks = -(-plan.full_max // C)
    comm.chunk_calls += max(0, nchunks - 1)
    dev = tensors[0].device
    total = sum(recv)
    assembled = torch.empty((total, rb), dtype=torch.uint8, device=dev)
    roff = np.cumsum([0] + recv).tolist()
    perm = plan.perm
    pending = []

    def land(j, out, work, r_j):
        work.wait()
        out = out.to(dev)
        pos = 0
        for r in range(W):
            if r_j[r]:
                assembled[roff[r] + j * C:roff[r] + j * C + r_j[r]].copy_(out[pos:pos + r_j[r]])
            pos += r_j[r]

    for j in range(nchunks):
        s_j = [max(0, min(C, send[r] - j * C)) for r in range(W)]
        r_j = [max(0, min(C, recv[r] - j * C)) for r in range(W)]
        sl = [perm[plan.bounds[r] + j * C:plan.bounds[r] + j * C + s_j[r]] for r in range(W) if s_j[r]]
        idx = torch.cat(sl) if sl else perm[:0]
        packed, _ = pack_rows(tensors, idx, idx.numel(), lay)
        out, work = comm.all_to_all_v_async(packed, s_j, r_j)
        pending.append((j, out, work, r_j))
        if len(pending) > 1:
            land(*pending.pop(0))
    for item in pending:
        land(*item)
    return unpack_rows(assembled, lay, tensors)


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
    keys = wire_order(b)
    cols = _take_many([b.columns[k] for k in keys], idx)
    return Batch(dict(zip(keys, cols)), idx.numel(), d)


def _gather_column(c: Column, counts: List[int], comm) -> Column:
    """All-gather of one column (dictionaries must already agree)."""
    return _gather_columns([c], counts, comm)[0]


def _str_bytes(c: Column) -> int:
    return int(c.data.numel())


def _gather_columns(cols: List[Column], counts: List[int], comm,
                    str_bytes: Optional[List[List[int]]] = None) -> List[Column]:
    """All-gather of columns with agreeing structure: ONE all-gather-v of
    bytes carrying every rank's packed fixed-width rows followed by its
    plain-string columns' bytes (``str_bytes[rank][k]``: byte count of the
    k-th string column per rank, exchanged here when not given)."""
    _no_nested(cols)
    from ..ops.pack import pack_rows, unpack_rows
    n = len(cols[0]) if cols else 0
    tensors, spec = _fixed_parts(cols)
    sj = [j for j, c in enumerate(cols) if c.is_plain_string]
    packed, lay = pack_rows(tensors, None, n) if tensors else (None, (0, []))
    rb = lay[0]
    if not sj:
        parts: List[torch.Tensor] = []
        if tensors:
            rpacked, _ = comm.all_gather_v(packed, counts)
            parts = unpack_rows(rpacked, lay, tensors)
        return _rebuild(cols, spec, parts, {})
    if str_bytes is None:
        str_bytes = comm.allgather_ints([_str_bytes(cols[j]) for j in sj])
    local = [packed.reshape(-1)] if packed is not None else []
    local += [cols[j].data for j in sj]
    sizes = [counts[r] * rb + sum(str_bytes[r]) for r in range(len(counts))]
    allb, _ = comm.all_gather_v(torch.cat(local) if len(local) > 1 else local[0], sizes)
    row_parts, pieces = [], {j: [] for j in sj}
    for r, blk in enumerate(_split_bytes(allb, sizes)):
        sp = _split_bytes(blk, [counts[r] * rb] + list(str_bytes[r]))
        row_parts.append(sp[0])
        for k, j in enumerate(sj):
            pieces[j].append(sp[1 + k])
    parts = []
    if tensors:
        rows = torch.cat(row_parts) if len(row_parts) > 1 else row_parts[0]
        parts = unpack_rows(rows.view(-1, rb), lay, tensors)
    chars = {j: (pieces[j][0] if len(pieces[j]) == 1 else torch.cat(pieces[j])) for j in sj}
    return _rebuild(cols, spec, parts, chars)


def gather_all(b: Batch, ctx, max_rows: Optional[int] = None, normalized: bool = False) -> Optional[Batch]:
    """Every rank receives the concatenation of all ranks' rows (one packed
    all-gather-v for the fixed-width columns). ``max_rows``: return None
    (on every rank alike) when the rows of all ranks exceed it -- decided
    from the structure preamble, before any data moves."""
    comm = ctx.comm
    if comm is None or not comm.spmd or dist_of(b) == REPLICATED:
        return b if max_rows is None or b.num_rows <= max_rows else None
    b = materialized(b)
    keys = wire_order(b)
    # string byte counts ride along in the preamble (-1: not a plain string
    # here; same length on every rank)
    if normalized:
        # the caller's structure all-gather happened: only the counts (and
        # string byte counts) travel, in one tiny all-gather
        sj = [k for k in keys if b.columns[k].is_plain_string]
        rows = comm.allgather_ints([b.num_rows] + [_str_bytes(b.columns[k]) for k in sj])
        counts = [r[0] for r in rows]
        if max_rows is not None and sum(counts) > max_rows:
            return None
        out = dict(zip(keys, _gather_columns([b.columns[k] for k in keys], counts, comm,
                                             [r[1:] for r in rows] if sj else None))) if keys else {}
        return with_dist(Batch(out, sum(counts)), REPLICATED)
    pre = [b.num_rows] + [_str_bytes(b.columns[k]) if b.columns[k].is_plain_string else -1 for k in keys]
    b = normalize_structure(b, comm, pre)
    counts = [p[0] for p in b.preamble]
    if max_rows is not None and sum(counts) > max_rows:
        return None
    cols = [b.columns[k] for k in keys]
    sj = [j for j, c in enumerate(cols) if c.is_plain_string]
    sb = [[p[1 + j] for j in sj] for p in b.preamble]
    if any(x < 0 for r in sb for x in r):
        sb = None   # a dictionary column was decoded by normalisation: exchange its byte counts
    out = dict(zip(keys, _gather_columns(cols, counts, comm, sb))) if keys else {}
    return with_dist(Batch(out, sum(counts)), REPLICATED)


#: string bytes per row and string column a small gather reserves per rank
SMALL_GATHER_STR_BYTES = 160
#: largest per-rank row count ``gather_small`` serves (ORDER BY ... LIMIT k)
SMALL_GATHER_ROWS = 4096


def gather_small(b: Batch, ctx, cap_rows: int) -> Batch:
    """``gather_all`` for a batch of at most ``cap_rows`` rows per rank (the
    local top-k of a distributed ORDER BY ... LIMIT k) in ONE collective: a
    fixed-size all-gather of per-rank slots whose layout follows from the
    schema and ``cap_rows`` alone -- [header | packed rows | string bytes per
    column] with validity always present, strings plain and decimals 128-bit
    -- so no structure or count exchange precedes it. The header carries the
    row count, the string byte counts and the local structure bits (validity
    and 128-bit sums are dropped again when no rank had them). A rank whose
    rows or string bytes exceed the slot flags it there; every rank then sees
    the flag and falls back to ``gather_all`` alike."""
    from ..ops.pack import pack_rows, unpack_rows
    from ..ops.select import offsets_from_lengths
    comm = ctx.comm
    if comm is None or not comm.spmd or dist_of(b) == REPLICATED:
        return b
    b = materialized(b)
    W = comm.world_size
    keys = wire_order(b)
    n = b.num_rows
    dev = ctx.device
    cap_s = cap_rows * SMALL_GATHER_STR_BYTES
    flags, tensors, chars = [], [], []
    over = n > cap_rows
    for k in keys:
        c = b.columns[k]
        flags.append((1 if c.valid is not None else 0) | (2 if c.is_wide else 0))
        if c.is_dict:
            c = S.decode(c)
        tensors.append(c.valid if c.valid is not None else torch.ones(len(c), dtype=torch.bool, device=dev))
        if c.is_plain_string:
            tensors.append((c.offsets[1:] - c.offsets[:-1]).to(torch.int64))
            chars.append(c.data)
            over = over or c.data.numel() > cap_s
        elif c.dtype.is_decimal and not c.is_wide:
            x = c.data.to(torch.int64)
            tensors.append(torch.stack([x, x >> 63], 1))
        else:
            tensors.append(c.data)
    sbytes = [int(x.numel()) for x in chars]
    hdr = [n, int(over)] + flags + sbytes
    H = 8 * len(hdr)
    packed, lay = pack_rows(tensors, None, n)
    rb = lay[0]
    slot = H + cap_rows * rb + len(chars) * cap_s
    pieces = [device_ints(hdr, dev).view(torch.uint8)]
    if not over:
        pieces.append(packed.reshape(-1))
        pieces.append(torch.zeros((cap_rows - n) * rb, dtype=torch.uint8, device=dev))
        for x in chars:
            pieces += [x.view(torch.uint8), torch.zeros(cap_s - x.numel(), dtype=torch.uint8, device=dev)]
    else:
        pieces.append(torch.zeros(slot - H, dtype=torch.uint8, device=dev))
    allb = comm.allgather_tensor(torch.cat(pieces)).view(W, slot)
    hv = to_host_ints(allb[:, :H].contiguous().view(torch.int64).reshape(-1))
    hd = [hv[r * len(hdr):(r + 1) * len(hdr)] for r in range(W)]
    if any(h[1] for h in hd):
        log.debug("small gather overflowed its slot: falling back to the counted gather")
        return gather_all(b, ctx)
    counts = [h[0] for h in hd]
    total = sum(counts)
    rows = torch.cat([allb[r, H:H + counts[r] * rb] for r in range(W)]).view(total, rb)
    parts = unpack_rows(rows, lay, tensors)
    out, t, sc = {}, 0, 0
    for j, k in enumerate(keys):
        c0 = b.columns[k]
        anyf = 0
        for h in hd:
            anyf |= h[2 + j]
        valid = parts[t] if anyf & 1 else None
        t += 1
        if c0.dtype.is_string:
            lens = parts[t]
            t += 1
            base = H + cap_rows * rb + sc * cap_s
            data = torch.cat([allb[r, base:base + hd[r][2 + len(keys) + sc]] for r in range(W)])
            sc += 1
            off = offsets_from_lengths(lens, host_total=False)[0] if total else \
                torch.zeros(1, dtype=torch.int64, device=dev)
            out[k] = Column(c0.dtype, data, valid, offsets=off)
            continue
        data = parts[t]
        t += 1
        if c0.dtype.is_decimal and not anyf & 2:
            data = data[:, 0].contiguous().to(c0.data.dtype)
        out[k] = Column(c0.dtype, data, valid, dictionary=None)
    return with_dist(Batch(out, total), REPLICATED)


# ----------------------------------------------------------------------- joins
def _cid(e: Expr):
    return e.cid if isinstance(e, ColRef) else None


def join_out_dist(kind: str, ld, rd):
    """Placement of a rank-local join's output given the placement keys of
    its inputs (``ld``/``rd``: ("hash", cid, ...) or None). A key column
    describes the output's placement only when it can never be NULL-padded:
    an outer join pads the non-preserved side with NULLs on whatever rank
    the preserved row lives, so GROUP BY that column would form one NULL
    group per rank. Inner / semi / anti keep both sides' keys (semi and anti
    output only left columns anyway), LEFT only the left side's, RIGHT only
    the right side's, FULL none."""
    scheme = ld[0] if keyed(ld) else (rd[0] if keyed(rd) else None)
    lk = tuple(ld[1:]) if keyed(ld) and ld[0] == scheme else ()
    rk = tuple(rd[1:]) if keyed(rd) and rd[0] == scheme else ()
    if kind in ("inner", "cross", "semi", "anti"):
        keys = lk + tuple(c for c in rk if c not in lk)
    elif kind == "left":
        keys = lk
    elif kind == "right":
        keys = rk
    else:
        keys = ()
    return (scheme,) + keys if keys else None


def prepare_join(lb: Batch, rb: Batch, join: L.Join, ctx, rows: Optional[Tuple[int, int]] = None):
    """Move rows so the join can run rank-locally; returns (lb, rb) with the
    output distribution stored in ``lb.out_dist``. ``rows``: the inputs'
    global row counts when the caller already reduced them."""
    from ..exec.joins import _pair_key
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
            if copartitioned(ld, lc, rd, rc):
                # co-partitioned: rank-local; the output is placed by the keys
                # of the sides that are never NULL-padded
                return done(lb, rb, join_out_dist(kind, ld, rd))
    if kind in ("inner", "cross") and (rep_l or rep_r):
        return done(lb, rb, rd if rep_l else ld)
    if kind in ("left", "semi", "anti") and rep_r:
        return done(lb, rb, ld)
    null_aware = getattr(join, "null_aware", False)
    if rows is None and kind in ("left", "semi", "anti") and on and not (rep_l or rep_r or null_aware):
        # only the non-preserved side's global size matters here: the gather's
        # own structure preamble decides it (None when it is too big to
        # broadcast, on every rank alike), one collective fewer than counting
        # first; a big side is shuffled below
        g = gather_all(rb, ctx, max_rows=limit)
        if g is not None:
            return done(lb, g, ld)
        nl, nr = lb.num_rows, limit + 1      # (not read again on this path)
    # global sizes decide broadcast vs shuffle (a replicated side counts once)
    elif rows is not None:
        nl, nr = rows
    else:
        nl, nr = comm.allreduce_ints([lb.num_rows if not rep_l else 0, rb.num_rows if not rep_r else 0])
    if rep_l:
        nl = lb.num_rows
    if rep_r:
        nr = rb.num_rows
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
    # a key converted to a common type (decimal scales) is no longer placed by
    # the hash of its own column's values
    same = lcol.dtype == rcol.dtype
    return done(lb, rb, join_out_dist(kind, ("hash", lc) if lc is not None and same else None,
                                      ("hash", rc) if rc is not None and same else None))


def semi_by_key_set(lb: Batch, rb: Batch, join: L.Join, ctx) -> Optional[Batch]:
    """SEMI / ANTI join of a REPLICATED left side against a partitioned right
    side (TPC-H Q22: customer NOT EXISTS orders) with no row movement: each
    rank builds a hash table on the (small, replicated) left keys, streams
    its own right rows through it marking the left rows that found a partner,
    and ONE all-reduce (max) of those per-left-row marks -- the left side is
    identical on every rank, so mark i means the same row everywhere -- gives
    the global answer; each rank then filters its replicated left rows
    locally and the result stays replicated. One collective of n_left bytes,
    no key-range exchange, no shuffle. None when the shape does not apply."""
    from ..exec.joins import _pair_key
    from ..ops import hashing as H
    from ..ops.select import mask_to_indices
    comm = ctx.comm
    if join.kind not in ("semi", "anti") or len(join.on or []) != 1 or join.residual is not None \
            or getattr(join, "null_aware", False):
        return None
    if dist_of(rb) == REPLICATED:
        return None
    if dist_of(lb) != REPLICATED:
        return _semi_by_range_marks(lb, rb, join, ctx)
    ev = ctx.evaluator
    le, re_ = join.on[0]
    lcol, rcol = ev.column(le, lb), ev.column(re_, rb)
    if lcol.dtype.is_string or rcol.dtype.is_string or lcol.data.dim() != 1 or rcol.data.dim() != 1 \
            or not (lcol.dtype.is_integer or lcol.dtype.kind == "date32") \
            or not (rcol.dtype.is_integer or rcol.dtype.kind == "date32"):
        return None
    lk, rk = _pair_key(lcol, rcol)
    n_l = lb.num_rows
    matched = torch.zeros(n_l, dtype=torch.bool, device=ctx.device)
    if n_l and rk.numel():
        with ctx.span("join.semi_marks"):
            H.JoinTable(lk.contiguous(), lcol.valid).probe_first(rk.contiguous(), rcol.valid, build_matched=matched)
    marks = comm.allreduce_tensor(matched.to(torch.uint8), "max") if n_l else matched.to(torch.uint8)
    hit = marks > 0
    keep = mask_to_indices(hit if join.kind == "semi" else ~hit)
    keys = list(lb.columns)
    return Batch(dict(zip(keys, take_many([lb.columns[k] for k in keys], keep))), int(keep.numel()), REPLICATED)


#: largest key domain (bytes of marks per rank) of the range-sliced semi join
RANGE_MARKS_MAX = 1 << 28


def _semi_by_range_marks(lb: Batch, rb: Batch, join: L.Join, ctx) -> Optional[Batch]:
    """SEMI / ANTI join of a left side sliced by key range ON THE JOIN KEY
    (parallel/slicing.py: TPC-H Q22's customer, every rank a contiguous
    c_custkey chunk) against a partitioned right side: every rank marks the
    right keys it holds in a dense byte array over the whole key domain
    [kmin, kmin + world * chunk), and ONE reduce-scatter (max) hands rank r
    the marks of its own chunk -- the keys of its left rows. (world - 1) /
    world of the domain's bytes move per rank; no row moves. None when the
    shape does not apply (the caller exchanges rows instead)."""
    from ..ops.gather import take_many as _take_many
    from ..ops.select import mask_to_indices
    comm = ctx.comm
    d = dist_of(lb)
    le, re_ = join.on[0]
    if not (keyed(d) and isinstance(d[0], tuple) and d[0][0] == "range" and isinstance(le, ColRef)
            and placed_on(d, le.cid)):
        return None
    _tag, W, kmin, chunk = d[0]
    if W != comm.world_size or W * chunk > RANGE_MARKS_MAX:
        return None
    ev = ctx.evaluator
    lcol, rcol = ev.column(le, lb), ev.column(re_, rb)
    for c in (lcol, rcol):
        if c.dtype.is_string or c.data.dim() != 1 or not (c.dtype.is_integer or c.dtype.kind == "date32") \
                or c.dtype.is_decimal:
            return None
    dev = ctx.device
    dom = W * chunk
    gpu = dev.type == "cuda"
    marks = torch.zeros(dom + (0 if gpu else 1), dtype=torch.uint8, device=dev)
    if rb.num_rows:
        if gpu:
            # one pass over the keys (ops/_lib: the mark_keys kernel), no temporaries
            from ..ops._lib import launch, ptr, stream
            rk = rcol.data if rcol.data.dtype in (torch.int32, torch.int64) else rcol.data.to(torch.int64)
            if rcol.valid is None and getattr(rk, "_igloo_resident", False) and rk.numel() >= (1 << 20):
                # a resident key column: its sorted secondary index (built once,
                # kept with the column) makes the mark stores ascending --
                # coalesced, instead of one random byte store per row (Q22:
                # 150M o_custkey into a 15 MB mark array, 2.6 -> ~0.2 ms)
                from ..ops import hashing as H
                rk = H.perm_index(rk)[0]
            rk = rk.contiguous()
            launch("mark_keys").mark_keys(ptr(rk), rk.dtype == torch.int64, ptr(rcol.valid), rk.numel(), kmin, dom,
                                          ptr(marks), stream(marks))
        else:
            rk = rcol.data.to(torch.int64) - kmin
            ok = (rk >= 0) & (rk < dom)
            if rcol.valid is not None:
                ok = ok & rcol.valid
            marks.index_fill_(0, torch.where(ok, rk, torch.full_like(rk, dom)), 1)   # [dom]: no mark
    mine = comm.reduce_scatter_tensor(marks[:dom].view(W, chunk), "max")
    n_l = lb.num_rows
    base = kmin + comm.rank * chunk
    if n_l and gpu:
        from ..ops._lib import launch, ptr, stream
        lk = lcol.data if lcol.data.dtype in (torch.int32, torch.int64) else lcol.data.to(torch.int64)
        lk = lk.contiguous()
        keepm = torch.empty(n_l, dtype=torch.bool, device=dev)
        launch("probe_marks").probe_marks(ptr(lk), lk.dtype == torch.int64, ptr(lcol.valid), n_l, base, chunk,
                                          ptr(mine.contiguous()), join.kind == "anti", ptr(keepm), stream(keepm))
    elif n_l:
        lk = lcol.data.to(torch.int64) - base
        inr = (lk >= 0) & (lk < chunk)
        if lcol.valid is not None:
            inr = inr & lcol.valid
        hit = (mine.index_select(0, lk.clamp(0, chunk - 1)) > 0) & inr
        keepm = hit if join.kind == "semi" else ~hit
    else:
        keepm = torch.zeros(0, dtype=torch.bool, device=dev)
    keep = mask_to_indices(keepm)
    keys = list(lb.columns)
    return Batch(dict(zip(keys, _take_many([lb.columns[k] for k in keys], keep))), int(keep.numel()), d)


# ------------------------------------------------------------------ aggregation
DECOMPOSABLE = {"sum", "count", "min", "max", "avg", "bool_and", "bool_or"}


def distributed_aggregate(lg: L.Aggregate, b: Batch, ctx, local=None) -> Batch:
    """``local(groups, partial_aggs) -> Batch | None`` may compute the phase-1
    partial states directly from the scan (fused VM kernel)."""
    from ..exec.aggregate import aggregate
    groups, aggs = lg.groups, lg.aggs
    d = dist_of(b)
    if d == REPLICATED:
        return with_dist(aggregate(groups, aggs, b, ctx), REPLICATED)
    if keyed(d):
        for ci, e in groups:
            if isinstance(e, ColRef) and placed_on(d, e.cid):
                # every group lives on one rank: the local aggregate is final
                return with_dist(aggregate(groups, aggs, b, ctx), (d[0], ci.cid))
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
    pb = local(groups, partial, plan) if local is not None else None
    restore = None
    if pb is None:
        pb, groups, restore = _partial_by_rows(groups, partial, b, ids, ctx)
    # ---- exchange partial states. A global aggregate (no GROUP BY) is ONE
    # all-reduce of dense state matrices (every partial column carries a
    # validity count, so no structure agreement is needed). Otherwise ONE
    # all-gather agrees on the structure of the partial batch (validity,
    # dictionary vs plain, 64 vs 128-bit sums, shared dictionary codes) and
    # carries in its preamble: the local ranges of the integer group keys,
    # the partial row count and string bytes, and -- where a hash shuffle is
    # certain to follow -- the shuffle's count matrix row. From that, alike on
    # every rank, one of:
    #   * an all-reduce over a small dense key domain (dictionary / boolean /
    #     small-range integer keys: TPC-H Q1, Q4, Q9's year x nation, Q13);
    #   * few partial groups in all (<= SMALL_AGG_GATHER): ONE all-gather-v
    #     and a replicated merge (a following join or ORDER BY needs no
    #     exchange: Q17's per-part averages, Q20's per-(part, supplier) sums);
    #   * a hash shuffle by the group key: ONE all-to-all-v.
    comm = ctx.comm
    W = comm.world_size
    dense_plan = _dense_candidate(groups, partial)
    unique = False
    if dense_plan and not groups:
        pbn = _with_validity(materialized(pb))
        pbn.preamble = [[] for _ in range(W)]
        rb = _dense_allreduce(groups, partial, pbn, ctx)
        log.debug("aggregate exchange: global, dense all-reduce")
        unique, out_dist = True, REPLICATED
    else:
        pm = materialized(pb)
        extra = _int_key_ranges(groups, pm) if dense_plan else []
        nr = len(extra)
        strs = [k for k, c in pm.columns.items() if c.dtype.is_string]
        extra += [pm.num_rows] + [_str_bytes(pm.columns[k]) if pm.columns[k].is_plain_string else -1 for k in strs]
        # a shuffle plan travels with the preamble when this rank already
        # knows the dense domain is too large (its local ranges exceed it)
        splan, key, kcid = None, None, None
        if groups and (not dense_plan or pm.num_rows == 0 or
                       _local_domain(groups, pm, extra[:nr]) > DENSE_ALLREDUCE_MAX):
            key, kcid = _shuffle_key(groups, pm)
            splan = ShufflePlan(pm, key, W)
        pw = ShufflePlan.width(pm, W) if groups else 0
        extra += ([1] + splan.preamble()) if splan is not None else [0] * (1 + pw)
        pbn = normalize_structure(pm, comm, extra)
        pre = pbn.preamble
        pbn.preamble = [r[:nr] for r in pre]
        rb = _dense_allreduce(groups, partial, pbn, ctx) if dense_plan and groups else None
        counts = [r[nr] for r in pre]
        if rb is not None:
            unique, out_dist = True, REPLICATED
            how = "dense all-reduce"
        elif not groups or sum(counts) <= SMALL_AGG_GATHER:
            sj = [j for j, k in enumerate(strs) if pbn.columns[k].is_plain_string]
            sb = [[r[nr + 1 + j] for j in sj] for r in pre]
            keys = list(pbn.columns)
            cols = _gather_columns([pbn.columns[k] for k in keys], counts, comm,
                                   None if any(x < 0 for x in sum(sb, [])) else sb)
            rb, out_dist = Batch(dict(zip(keys, cols)), sum(counts)), REPLICATED
            how = "gather"
        else:
            base = nr + 1 + len(strs)
            if splan is not None and all(r[base] for r in pre):
                if not splan.receive([r[base + 1:] for r in pre], comm.rank, pbn):
                    splan = None
            else:
                splan = None
            if key is None:
                key, kcid = _shuffle_key(groups, pbn)
            rb = shuffle(pbn, key, ctx, kcid, normalized=True, plan=splan)
            out_dist = rb.dist
            how = "shuffle" + (" (counts in preamble)" if splan is not None else "")
        log.debug("aggregate exchange: %d partial groups here, %d in all, %s", pb.num_rows, sum(counts), how)
    # ---- phase 2: merge (the dense all-reduce leaves one row per group:
    # its states only need finalising)
    # (groups that shipped row numbers all depend on the leading integer key:
    # the merge groups by it and checks the rest)
    res = finalize_unique(groups, plan, rb) if unique else \
        merge_partials(groups, plan, rb, ids, ctx, fd=restore is not None)
    if restore is not None:
        res = restore(res)
    return with_dist(res, out_dist)


def _partial_by_rows(groups, partial, b: Batch, ids, ctx):
    """Phase-1 partial aggregate whose exchange ships ROW NUMBERS instead of
    string group keys, where it can: GROUP BY keys that are plain strings of
    a REPLICATED input of a join still in index form (TPC-H Q10: c_name,
    c_address, c_phone, c_comment of the replicated customer table, grouped
    with c_custkey over orders x lineitem partitioned by order key). The
    local grouping runs by the leading integer key with the others checked
    to be functionally dependent on it (exec/aggregate.py _late_group_keys);
    each group then carries its row in the replicated input -- the same row
    number on every rank -- and the strings are taken from that input after
    the merge, on the owning rank only (~4M groups x ~130 string bytes at
    SF100 no longer cross the fabric). Every rank must take the same shape,
    so the dependency check's outcome is agreed by one tiny all-gather.
    Returns (partial batch, exchange group keys, restore(merged) or None)."""
    from ..exec.joins import LateBatch
    from ..exec.aggregate import aggregate
    rows = {}
    if isinstance(b, LateBatch) and len(groups) > 1 and b.num_rows >= 0:
        for i, (ci, e) in enumerate(groups):
            if not isinstance(e, ColRef) or e.cid not in b.owner:
                continue
            k = b.owner[e.cid]
            bb, idx = b.parts[k]
            src = bb.src if hasattr(bb, "take_rows") else bb      # (a lazy filtered scan: its source column)
            if idx is not None and dist_of(bb) == REPLICATED and src.columns[e.cid].is_plain_string:
                rows[i] = k
    if not rows or len(rows) == len(groups):
        return aggregate(groups, partial, b, ctx), groups, None
    row_ci = {k: L.ColInfo(ids(), "__row", T.INT64, False) for k in sorted(set(rows.values()))}
    replaced = {groups[i][0].cid for i in rows}
    pb = aggregate(groups, partial, b, ctx, row_parts={ci.cid: k for k, ci in row_ci.items()}, skip=replaced)
    have = all(ci.cid in pb.columns for ci in row_ci.values())
    ok = all(r[0] for r in ctx.comm.allgather_ints([int(have)]))
    log.debug("partial aggregate ships row numbers for %d string key(s): local %s, agreed %s",
              len(rows), have, ok)
    if not ok:
        if have:
            # another rank's grouping did not take the row-number shape: this
            # rank groups again with every key materialised
            pb = aggregate(groups, partial, b, ctx)
        return pb, groups, None
    pb = Batch({c: v for c, v in pb.columns.items() if c not in replaced}, pb.num_rows, pb.dist)
    ex_groups = [g for i, g in enumerate(groups) if i not in rows] + \
        [(ci, ColRef(ci.cid, ci.name, ci.dtype, False)) for ci in row_ci.values()]
    parts = {k: b.parts[k][0] for k in row_ci}

    def restore(res: Batch) -> Batch:
        # the strings stay in the replicated input until read (columnar.py
        # LazyColumn): a top-k above takes only its rows
        from ..columnar import LazyColumn
        cols = {c: v for c, v in res.columns.items() if c not in {ci.cid for ci in row_ci.values()}}
        for i, k in rows.items():
            ci, e = groups[i]
            r = res.columns[row_ci[k].cid].data
            cols[ci.cid] = LazyColumn(ci.dtype, parts[k], e.cid, r)
        return Batch(cols, res.num_rows, res.dist)
    return pb, ex_groups, restore


def _shuffle_key(groups, b: Batch):
    """Partition key of a shuffle by the group keys: the first key's, unless
    it is a low-cardinality type (dictionary string, boolean) and more keys
    follow -- then a mix of all of them (TPC-H Q16 groups by brand, type,
    size: 25 brands would leave ranks idle). Returns (key, placement cid or
    None for a mixed key)."""
    cols = [b.columns[ci.cid] for ci, _ in groups]
    c0 = cols[0]
    if len(cols) == 1 or not (c0.is_dict or c0.dtype.kind == "bool"):
        return partition_keys(c0), groups[0][0].cid
    key = None
    for c in cols:
        k = partition_keys(c).to(torch.int64)
        key = k if key is None else key * 1000003 + k
    return key.contiguous(), None


def _dense_candidate(groups, partial) -> bool:
    """Plan-level part of the dense all-reduce test (alike on every rank)."""
    for _, a in partial:
        if a.func not in ("sum", "count", "min", "max", "bool_and", "bool_or") or a.dtype.is_string:
            return False
    for ci, _ in groups:
        t = ci.dtype
        if not (t.is_string or t.kind == "bool" or t.kind == "date32" or (t.is_integer and not t.is_decimal)):
            return False
    return True


def _is_int_key(ci) -> bool:
    t = ci.dtype
    return not t.is_string and t.kind != "bool" and (t.kind == "date32" or t.is_integer)


def _int_key_ranges(groups, pb: Batch) -> List[int]:
    """[lo, hi] of every integer-typed group key over this rank's partial
    groups (an empty rank reports an empty range)."""
    from ..ops import hashing as H
    out = []
    for ci, _ in groups:
        if not _is_int_key(ci):
            continue
        c = pb.columns[ci.cid]
        rng = H.key_range(c.data.to(torch.int64) if c.data.dtype not in (torch.int32, torch.int64) else c.data,
                          c.valid) if pb.num_rows and c.data.dim() == 1 else None
        out += list(rng) if rng else [2**62, -2**62]
    return out


#: partial groups (all ranks) up to which the exchange all-gathers them and
#: merges on every rank (replicated result) instead of shuffling
SMALL_AGG_GATHER = 1 << 15


def _local_domain(groups, pb: Batch, ranges: List[int]) -> int:
    """Dense key domain over this rank's partial groups alone (a lower bound
    of the global one: shared dictionaries and merged ranges only grow)."""
    dom, ri = 1, 0
    for ci, _ in groups:
        c = pb.columns[ci.cid]
        if _is_int_key(ci):
            lo, hi = ranges[ri], ranges[ri + 1]
            ri += 2
            span = hi - lo + 1 if lo <= hi else 1
        elif c.dtype.is_string and not c.is_dict:
            return DENSE_ALLREDUCE_MAX + 1
        else:
            span = len(c.dictionary) if c.is_dict else 2
        dom *= max(span, 1) + (1 if c.valid is not None else 0)
    return dom


def wire_order(b: Batch) -> list:
    """The order an exchange packs ``b``'s columns in: by column id, the same
    on every rank -- a batch's dict order follows how its columns were built
    (a join side taken as the identity on one rank keeps its gathered columns
    first, exec/joins.py LateBatch), which ranks need not share."""
    try:
        return sorted(b.columns)
    except TypeError:
        return list(b.columns)


def _with_validity(b: Batch) -> Batch:
    """Every column with a validity mask (all-true where absent): the dense
    all-reduce's state matrix then has the same columns on every rank."""
    out = {}
    for k, c in b.columns.items():
        if c.valid is None:
            c = Column(c.dtype, c.data, torch.ones(len(c), dtype=torch.bool, device=c.data.device), c.offsets,
                       c.dictionary)
        out[k] = c
    return Batch(out, b.num_rows, b.dist)


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


def merge_partials(groups, plan, rb: Batch, ids, ctx, fd: bool = False) -> Batch:
    """Phase 2: merge the partial states in ``rb`` (rows = partial groups) into
    the final aggregates of ``plan`` (see ``partial_plan``)."""
    from ..exec.aggregate import _avg, aggregate
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
    fb = aggregate(fgroups, final, rb, ctx, fd=fd)
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


def finalize_unique(groups, plan, rb: Batch) -> Batch:
    """``merge_partials`` for partial states already merged to one row per
    group (the dense all-reduce): the final columns come straight from the
    states -- no second grouping pass."""
    from ..exec.aggregate import _avg
    out = {ci.cid: rb.columns[ci.cid] for ci, _ in groups}
    for func, ci, a, p1, p2 in plan:
        if func == "avg":
            s, c = rb.columns[p1.cid], rb.columns[p2.cid]
            cnt = c.data if c.valid is None else torch.where(c.valid, c.data, torch.zeros_like(c.data))
            out[ci.cid] = Column(a.dtype, _avg(s.data, cnt, a.arg.dtype, a.dtype), cnt > 0)
        elif func == "count":
            c = rb.columns[p1.cid]
            out[ci.cid] = Column(T.INT64, c.data if c.valid is None else
                                 torch.where(c.valid, c.data, torch.zeros_like(c.data)))
        else:
            c = rb.columns[p1.cid]
            out[ci.cid] = Column(a.dtype, c.data, c.valid)
    return Batch(out, rb.num_rows)


#: largest dense group-key domain whose partial states are all-reduced
DENSE_ALLREDUCE_MAX = 4096
_I64_MAX, _I64_MIN = 2**63 - 1, -2**63


def _dense_allreduce(groups, partial, pb: Batch, ctx) -> Optional[Batch]:
    """Two-phase aggregation over a small dense key domain (no GROUP BY, or
    group keys that are dictionary strings, booleans or integers whose
    domains multiply to at most DENSE_ALLREDUCE_MAX, e.g. TPC-H Q1's
    returnflag x linestatus, Q13's order counts): every rank scatters its
    partial states into dense per-key tables and ONE all-reduce per reduction
    op (SUM / MIN / MAX) merges them -- no shuffle, and the result is
    replicated on every rank (so a following ORDER BY needs no gather).
    ``pb`` comes from ``normalize_structure`` (identical structure on every
    rank; its preamble holds every rank's integer-key ranges), so every rank
    takes the same decision. Integer SUMs travel as three int64 parts (high
    word, low word's two 32-bit halves) that cannot overflow and recombine
    into exact 128-bit sums. The states are scattered as matrices (one
    index_add / scatter_reduce per op), so the launch count does not grow with
    the number of aggregates. Returns the merged partial-state batch or None
    when the shape does not apply."""
    from ..ops.agg import _wide_flags
    from ..ops.select import mask_to_indices
    comm = ctx.comm
    dev = ctx.device
    cols = [pb.columns[ci.cid] for ci, _ in partial]
    keys = [pb.columns[ci.cid] for ci, _ in groups]
    if any(k.dtype.is_string and not k.is_dict for k in keys):
        return None
    ranges = [list(r) for r in pb.preamble]
    sizes, offs, ri = [], [], 0
    for (ci, _), k in zip(groups, keys):
        nullable = k.valid is not None
        if _is_int_key(ci):
            lo = min(r[ri] for r in ranges)
            hi = max(r[ri + 1] for r in ranges)
            ri += 2
            span = hi - lo + 1 if lo <= hi else 1
            offs.append(lo if lo <= hi else 0)
        else:
            span = len(k.dictionary) if k.is_dict else 2
            offs.append(0)
        sizes.append(max(span, 1) + (1 if nullable else 0))
    domain = 1
    for z in sizes:
        domain *= z
        if domain > DENSE_ALLREDUCE_MAX:
            return None
    n = pb.num_rows
    idx = None
    for j, k in enumerate(keys):
        code = k.data.to(torch.int64) - offs[j] if offs[j] else k.data.to(torch.int64)
        if k.valid is not None:
            code = torch.where(k.valid, code, torch.full_like(code, sizes[j] - 1))
        idx = code if idx is None else idx * sizes[j] + code
    if idx is None:
        idx = torch.zeros(n, dtype=torch.int64, device=dev)
    i64 = torch.int64
    # ---- per aggregate: which matrix columns hold its state
    valid_cols = []        # (slot, valid mask) for columns that have a validity
    isums, fsums, mins, maxs = [], [], [], []    # (partial index, tensor)
    for j, ((ci, a), c) in enumerate(zip(partial, cols)):
        isf = c.data.dtype in (torch.float32, torch.float64)
        if c.valid is not None:
            valid_cols.append((j, c.valid))
        if a.func in ("sum", "count") and not isf:
            isums.append((j, c))
        elif a.func in ("sum", "count"):
            fsums.append((j, c.data.to(torch.float64)))
        elif a.func in ("min", "bool_and"):
            mins.append((j, c.data.to(torch.float64 if isf else i64)))
        else:
            maxs.append((j, c.data.to(torch.float64 if isf else i64)))
    # int64 matrix: [presence | valid counts | sum hi words | mid halves | low halves]
    icols = [torch.ones(n, dtype=i64, device=dev)] + [v.to(i64) for _, v in valid_cols]
    if isums:
        lo_w = torch.stack([c.data[:, 0] if c.is_wide else c.data.to(i64) for _, c in isums], 1)
        hi_w = lo_w >> 63
        for t, (_, c) in enumerate(isums):
            if c.is_wide:
                hi_w[:, t] = c.data[:, 1]
        parts = torch.cat([hi_w, (lo_w >> 32) & 0xFFFFFFFF, lo_w & 0xFFFFFFFF], 1)
        vmask = [c.valid for _, c in isums]
        if any(v is not None for v in vmask):
            vm = torch.stack([v if v is not None else torch.ones(n, dtype=torch.bool, device=dev) for v in vmask], 1)
            parts = parts * vm.repeat(1, 3).to(i64)
        imat = torch.cat([torch.stack(icols, 1), parts], 1)
    else:
        imat = torch.stack(icols, 1)
    reds = {}

    def scatter(mat, op, fill):
        out = torch.full((domain, mat.shape[1]), fill, dtype=mat.dtype, device=dev)
        if n:
            if op == "sum":
                out.index_add_(0, idx, mat)
            else:
                out.scatter_reduce_(0, idx.view(-1, 1).expand(-1, mat.shape[1]), mat, op, include_self=True)
        return comm.allreduce_tensor(out, {"amin": "min", "amax": "max"}.get(op, op))

    def masked(lst, fill):
        m = torch.stack([t for _, t in lst], 1)
        vm = [cols[j].valid for j, _ in lst]
        if any(v is not None for v in vm):
            ok = torch.stack([v if v is not None else torch.ones(n, dtype=torch.bool, device=dev) for v in vm], 1)
            m = torch.where(ok, m, torch.full_like(m, fill))
        return m
    reds["i"] = scatter(imat, "sum", 0)
    if fsums:
        reds["f"] = scatter(masked(fsums, 0.0), "sum", 0.0)
    for name, lst, op in (("mn", mins, "amin"), ("mx", maxs, "amax")):
        fl_ = [x for x in lst if x[1].dtype == torch.float64]
        it_ = [x for x in lst if x[1].dtype != torch.float64]
        if fl_:
            fill = float("inf") if op == "amin" else float("-inf")
            reds[name + "f"] = scatter(masked(fl_, fill), op, fill)
        if it_:
            fill = _I64_MAX if op == "amin" else _I64_MIN
            reds[name + "i"] = scatter(masked(it_, fill), op, fill)
    present = mask_to_indices(reds["i"][:, 0] > 0)
    m = present.numel()
    rows = {k: v.index_select(0, present) for k, v in reds.items()}
    out = {}
    rest = present.to(i64)
    for j in range(len(keys) - 1, -1, -1):
        code = rest % sizes[j]
        rest = rest // sizes[j]
        k = keys[j]
        valid = None
        if k.valid is not None:
            valid = code != sizes[j] - 1
            code = torch.where(valid, code, torch.zeros_like(code))
        ci = groups[j][0]
        if k.is_dict:
            out[ci.cid] = Column(k.dtype, code.to(torch.int32), valid, dictionary=k.dictionary)
        elif k.dtype.kind == "bool":
            out[ci.cid] = Column(k.dtype, code.to(torch.bool), valid)
        else:
            out[ci.cid] = Column(k.dtype, (code + offs[j]).to(k.data.dtype), valid)
    iv = rows["i"]
    vslot = {j: 1 + t for t, (j, _) in enumerate(valid_cols)}

    def has(j):
        return iv[:, vslot[j]] > 0 if j in vslot else None
    if isums:
        S = len(isums)
        base = 1 + len(valid_cols)
        hi, mid, low = iv[:, base:base + S], iv[:, base + S:base + 2 * S], iv[:, base + 2 * S:base + 3 * S]
        sign = -(2**63)
        lo = low + ((mid & 0xFFFFFFFF) << 32)                     # wraps as uint64
        carry = ((lo ^ sign) < (low ^ sign)).to(i64)              # unsigned overflow of that add
        hi = hi + (mid >> 32) + carry
        # column-major once (every state column a contiguous view), and ONE
        # device check (one readback) whether any merged sum needs 128 bits
        lo_t, hi_t = lo.t().contiguous(), hi.t().contiguous()
        wide = False
        if m and any(partial[j][1].func != "count" for j, _ in isums):
            if lo.is_cuda:
                wide = bool(to_host_ints(_wide_flags([(lo_t.reshape(-1), hi_t.reshape(-1))]))[0])
            else:
                wide = not bool((hi_t == (lo_t >> 63)).all())
        for t, (j, c) in enumerate(isums):
            ci = partial[j][0]
            if partial[j][1].func == "count":
                out[ci.cid] = Column(c.dtype, lo_t[t])
                continue
            data = torch.stack([lo_t[t], hi_t[t]], 1) if wide else lo_t[t]
            out[ci.cid] = Column(c.dtype, data, has(j))
    for key, lst in (("f", fsums), ("mnf", [x for x in mins if x[1].dtype == torch.float64]),
                     ("mxf", [x for x in maxs if x[1].dtype == torch.float64]),
                     ("mni", [x for x in mins if x[1].dtype != torch.float64]),
                     ("mxi", [x for x in maxs if x[1].dtype != torch.float64])):
        mat = rows[key].t().contiguous() if lst else None
        for t, (j, _) in enumerate(lst):
            c = cols[j]
            v = mat[t]
            data = v.to(c.data.dtype) if c.dtype.kind != "bool" else v != 0
            hv = has(j)
            if hv is not None:
                data = torch.where(hv, data, torch.zeros_like(data))
            out[partial[j][0].cid] = Column(c.dtype, data.contiguous(), hv)
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
