"""Synthetic TPC-H data generated directly on the execution device.

Shapes, key layouts and value distributions follow the TPC-H spec (sparse
order keys, 1-7 lines per order, partsupp supplier formula, retail-price
formula, date windows, return-flag / line-status rules, o_totalprice and
o_orderstatus derived from the lines). Randomness is a counter-based hash of
(stream, global row id), so:

* the data is identical on CPU and GPU (tests run the CPU path, the bench the
  GPU path);
* any rank can generate exactly its own hash partition — rank r of W keeps the
  rows whose partition key k has ``mix64(k) % W == r``, the same function the
  exchange operators use, so co-partitioned joins (lineitem/orders,
  part/partsupp) need no shuffle.

Numeric columns are torch ops on the device; text columns (comments, names,
addresses, phones, part names) are written by the HIP text kernel
(csrc/kernels/datagen.hip). The reference has no generator at all; its only
Parquet fixture is a 176-byte text placeholder (reference data/sample.parquet).
"""
from __future__ import annotations

import datetime
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import torch

from ... import types as T
from ...catalog import Field, MemoryTable
from ...columnar import Column
from ...ops import _lib
from ...ops.misc import partition_ids
from ...ops.select import offsets_from_lengths
from . import schema as S

M32 = 0xFFFFFFFF
EPOCH = datetime.date(1970, 1, 1)


def _days(s: str) -> int:
    return (datetime.date.fromisoformat(s) - EPOCH).days


START, END, CURRENT = _days(S.START_DATE), _days(S.END_DATE), _days(S.CURRENT_DATE)


def _h32(x: torch.Tensor) -> torch.Tensor:
    # 32-bit avalanche hash in int64 arithmetic; multipliers < 2^31 keep every
    # product < 2^63, so the result is exact on every device.
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M32
    x = x ^ (x >> 15)
    x = (x * 0x2C1B3C6D) & M32
    x = x ^ (x >> 16)
    return x


def _seed(stream: int, seed: int) -> int:
    v = (stream * 0x9E3779B9 + seed * 0x632BE5AB) & M32
    t = torch.tensor([v], dtype=torch.int64)
    return int(_h32(_h32(t) ^ 0x5BD1E995)[0])


def rnd(idx: torch.Tensor, stream: int, seed: int = 0) -> torch.Tensor:
    s = _seed(stream, seed)
    lo = idx & M32
    hi = (idx >> 32) & M32
    return _h32((_h32(lo ^ s) + hi * 0x27D4EB2F + s) & M32)


def uniform(idx: torch.Tensor, stream: int, lo: int, hi: int, seed: int = 0) -> torch.Tensor:
    return lo + rnd(idx, stream, seed) % (hi - lo + 1)


# ------------------------------------------------------------------------ text
_VOCAB_CACHE: Dict[tuple, tuple] = {}


def _vocab(words: List[str], device) -> tuple:
    key = (tuple(words), str(device))
    if key not in _VOCAB_CACHE:
        enc = [w.encode() for w in words]
        off = np.zeros(len(enc) + 1, np.int32)
        off[1:] = np.cumsum([len(e) for e in enc])
        chars = np.frombuffer(b"".join(enc), np.uint8).copy()
        _VOCAB_CACHE[key] = (torch.from_numpy(chars).to(device), torch.from_numpy(off).to(device), len(enc))
    return _VOCAB_CACHE[key]


KIND = {"words": 0, "distinct_words": 1, "alnum": 2, "prefix_int": 3, "prefix_randint": 4, "phone": 5}


def gen_text(kind: str, row_ids: torch.Tensor, seed: int, min_len: int, max_len: int, device,
             words: Optional[List[str]] = None, inject: str = "", inject_every: int = 0,
             aux: Optional[torch.Tensor] = None) -> Column:
    """Plain-string column with one generated value per global row id."""
    N = _lib.native()
    n = row_ids.numel()
    device = torch.device(device)
    row_ids = row_ids.to(torch.int64).contiguous()
    vc, vo, vn = _vocab(words or ["x"], device)
    inj = torch.tensor(list(inject.encode()) or [0], dtype=torch.uint8).to(device)
    aux_t = aux.to(torch.int32).contiguous() if aux is not None else None
    params = (KIND[kind], seed & 0xFFFFFFFFFFFFFFFF, 0, min_len, max_len, vc.data_ptr(), vo.data_ptr(), vn,
              inj.data_ptr(), len(inject.encode()), inject_every, 0, _lib.ptr(aux_t), row_ids.data_ptr())
    gpu = device.type == "cuda"
    s = _lib.stream(row_ids) if gpu else 0
    lens = torch.empty(n, dtype=torch.int64, device=device)
    _lib.KERNEL_CALLS["textgen"] += 1
    N.textgen_lengths(params, n, lens.data_ptr(), gpu, s)
    off, total = offsets_from_lengths(lens)
    chars = torch.empty(total, dtype=torch.uint8, device=device)
    N.textgen_write(params, n, off.data_ptr(), chars.data_ptr(), gpu, s)
    return Column(T.UTF8, chars, None, offsets=off)


def dict_col(codes: torch.Tensor, values: List[str], device) -> Column:
    d = Column.from_arrow(pa.array(values, pa.large_string()), device=device, dict_encode=False)
    return Column(T.UTF8, codes.to(torch.int32), None, dictionary=d)


def _i32(t):
    return Column(T.INT32, t.to(torch.int32))


def _dec(t):
    return Column(T.DECIMAL(15, 2), t.to(torch.int64))


def _date(t):
    return Column(T.DATE32, t.to(torch.int32))


def _owned(keys: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    if world <= 1:
        return torch.ones(keys.numel(), dtype=torch.bool, device=keys.device)
    return partition_ids(keys.to(torch.int64).contiguous(), world) == rank


# ---------------------------------------------------------------------- tables
def gen_region(device) -> MemoryTable:
    k = torch.arange(5, device=device)
    cols = {
        "r_regionkey": _i32(k),
        "r_name": dict_col(k, S.REGIONS, device),
        "r_comment": gen_text("words", k, 71, 4, 10, device, S.WORDS),
    }
    return MemoryTable(cols, 5, replicated=True)


def gen_nation(device) -> MemoryTable:
    k = torch.arange(25, device=device)
    cols = {
        "n_nationkey": _i32(k),
        "n_name": dict_col(k, [n for n, _ in S.NATIONS], device),
        "n_regionkey": _i32(torch.tensor([r for _, r in S.NATIONS], device=device)),
        "n_comment": gen_text("words", k, 72, 4, 12, device, S.WORDS),
    }
    return MemoryTable(cols, 25, replicated=True)


def gen_supplier(sf, device, rank=0, world=1) -> MemoryTable:
    n = max(int(10_000 * sf), 1)
    k = torch.arange(1, n + 1, device=device, dtype=torch.int64)
    k = k[_owned(k, rank, world)]
    nk = uniform(k, 40, 0, 24)
    cols = {
        "s_suppkey": _i32(k),
        "s_name": gen_text("prefix_int", k - 1, 0, 9, 9, device, inject="Supplier#"),
        "s_address": gen_text("alnum", k, 41, 10, 40, device),
        "s_nationkey": _i32(nk),
        "s_phone": gen_text("phone", k, 42, 0, 0, device, aux=nk),
        "s_acctbal": _dec(uniform(k, 43, -99999, 999999)),
        "s_comment": gen_text("words", k, 44, 5, 14, device, S.WORDS, inject="Customer Complaints", inject_every=2000),
    }
    return MemoryTable(cols, k.numel(), partitioned_by="s_suppkey" if world > 1 else None)


def _retail(pk: torch.Tensor) -> torch.Tensor:
    return 90000 + ((pk // 10) % 20001) + 100 * (pk % 1000)


def gen_part(sf, device, rank=0, world=1) -> MemoryTable:
    n = max(int(200_000 * sf), 1)
    k = torch.arange(1, n + 1, device=device, dtype=torch.int64)
    k = k[_owned(k, rank, world)]
    m = uniform(k, 30, 1, 5)
    nn = uniform(k, 31, 1, 5)
    types = [f"{a} {b} {c}" for a in S.TYPE_S1 for b in S.TYPE_S2 for c in S.TYPE_S3]
    conts = [f"{a} {b}" for a in S.CONT_S1 for b in S.CONT_S2]
    cols = {
        "p_partkey": _i32(k),
        "p_name": gen_text("distinct_words", k, 32, 5, 5, device, S.COLORS),
        "p_mfgr": dict_col(m - 1, [f"Manufacturer#{i}" for i in range(1, 6)], device),
        "p_brand": dict_col((m - 1) * 5 + (nn - 1), [f"Brand#{a}{b}" for a in range(1, 6) for b in range(1, 6)], device),
        "p_type": dict_col(uniform(k, 33, 0, 149), types, device),
        "p_size": _i32(uniform(k, 34, 1, 50)),
        "p_container": dict_col(uniform(k, 35, 0, 39), conts, device),
        "p_retailprice": _dec(_retail(k)),
        "p_comment": gen_text("words", k, 36, 1, 4, device, S.WORDS),
    }
    return MemoryTable(cols, k.numel(), partitioned_by="p_partkey" if world > 1 else None)


def _ps_supp(pk: torch.Tensor, j: torch.Tensor, nsupp: int) -> torch.Tensor:
    return (pk + j * (nsupp // 4 + (pk - 1) // nsupp)) % nsupp + 1


def gen_partsupp(sf, device, rank=0, world=1, lean=False) -> MemoryTable:
    npart = max(int(200_000 * sf), 1)
    ns = max(int(10_000 * sf), 1)
    pk = torch.arange(1, npart + 1, device=device, dtype=torch.int64)
    pk = pk[_owned(pk, rank, world)]
    pk4 = pk.repeat_interleave(4)
    j = torch.arange(4, device=device, dtype=torch.int64).repeat(pk.numel())
    gid = (pk4 - 1) * 4 + j
    cols = {
        "ps_partkey": _i32(pk4),
        "ps_suppkey": _i32(_ps_supp(pk4, j, ns)),
        "ps_availqty": _i32(uniform(gid, 50, 1, 9999)),
        "ps_supplycost": _dec(uniform(gid, 51, 100, 100000)),
    }
    if not lean:
        cols["ps_comment"] = gen_text("words", gid, 52, 8, 20, device, S.WORDS)
    return MemoryTable(cols, pk4.numel(), partitioned_by="ps_partkey" if world > 1 else None)


def gen_customer(sf, device, rank=0, world=1) -> MemoryTable:
    n = max(int(150_000 * sf), 1)
    k = torch.arange(1, n + 1, device=device, dtype=torch.int64)
    k = k[_owned(k, rank, world)]
    nk = uniform(k, 60, 0, 24)
    cols = {
        "c_custkey": _i32(k),
        "c_name": gen_text("prefix_int", k - 1, 0, 9, 9, device, inject="Customer#"),
        "c_address": gen_text("alnum", k, 61, 10, 40, device),
        "c_nationkey": _i32(nk),
        "c_phone": gen_text("phone", k, 62, 0, 0, device, aux=nk),
        "c_acctbal": _dec(uniform(k, 63, -99999, 999999)),
        "c_mktsegment": dict_col(uniform(k, 64, 0, 4), S.SEGMENTS, device),
        "c_comment": gen_text("words", k, 65, 4, 14, device, S.WORDS),
    }
    return MemoryTable(cols, k.numel(), partitioned_by="c_custkey" if world > 1 else None)


def gen_orders_lineitem(sf, device, rank=0, world=1, lean=False):
    no = max(int(1_500_000 * sf), 1)
    ncust = max(int(150_000 * sf), 1)
    npart = max(int(200_000 * sf), 1)
    ns = max(int(10_000 * sf), 1)
    i = torch.arange(no, device=device, dtype=torch.int64)
    okey = (i // 8) * 32 + (i % 8) + 1
    own = _owned(okey, rank, world)
    i, okey = i[own], okey[own]
    r = uniform(i, 1, 0, max(2 * ncust // 3 - 1, 0))
    custkey = 3 * (r // 2) + 1 + (r % 2)
    odate = START + uniform(i, 2, 0, (END - START) - 151)
    nlines = uniform(i, 4, 1, 7)
    # ---- lineitem
    no_loc = i.numel()
    oidx = torch.repeat_interleave(torch.arange(no_loc, device=device), nlines)
    starts = torch.cumsum(nlines, 0) - nlines
    L = oidx.numel()
    lineno = torch.arange(L, device=device) - starts.index_select(0, oidx) + 1
    gi = i.index_select(0, oidx) * 8 + lineno
    pk = uniform(gi, 10, 1, npart)
    sk = _ps_supp(pk, uniform(gi, 11, 0, 3), ns)
    qty = uniform(gi, 12, 1, 50)
    ext = qty * _retail(pk)
    disc = uniform(gi, 13, 0, 10)
    tax = uniform(gi, 14, 0, 8)
    od = odate.index_select(0, oidx)
    ship = od + uniform(gi, 15, 1, 121)
    commit = od + uniform(gi, 16, 30, 90)
    receipt = ship + uniform(gi, 17, 1, 30)
    # return flag dictionary: A, N, R
    rf = torch.where(receipt <= CURRENT, torch.where(uniform(gi, 18, 0, 1) == 0, 2, 0), 1)
    ls = (ship > CURRENT).to(torch.int64)  # 0 = F, 1 = O
    lcols = {
        "l_orderkey": _i32(okey.index_select(0, oidx)),
        "l_partkey": _i32(pk),
        "l_suppkey": _i32(sk),
        "l_linenumber": _i32(lineno),
        "l_quantity": _dec(qty * 100),
        "l_extendedprice": _dec(ext),
        "l_discount": _dec(disc),
        "l_tax": _dec(tax),
        "l_returnflag": dict_col(rf, ["A", "N", "R"], device),
        "l_linestatus": dict_col(ls, ["F", "O"], device),
        "l_shipdate": _date(ship),
        "l_commitdate": _date(commit),
        "l_receiptdate": _date(receipt),
        "l_shipinstruct": dict_col(uniform(gi, 19, 0, 3), S.INSTRUCTIONS, device),
        "l_shipmode": dict_col(uniform(gi, 20, 0, 6), S.MODES, device),
    }
    if not lean:
        lcols["l_comment"] = gen_text("words", gi, 21, 2, 6, device, S.WORDS)
    # ---- derived order columns
    charge = ext * (100 + tax) * (100 - disc)  # cents * 1e4
    tot = torch.zeros(no_loc, dtype=torch.int64, device=device).index_add_(0, oidx, charge)
    totalprice = (tot + 5000) // 10000
    nf = torch.zeros(no_loc, dtype=torch.int64, device=device).index_add_(0, oidx, 1 - ls)
    status = torch.where(nf == nlines, 0, torch.where(nf == 0, 1, 2))  # F, O, P
    ocols = {
        "o_orderkey": _i32(okey),
        "o_custkey": _i32(custkey),
        "o_orderstatus": dict_col(status, ["F", "O", "P"], device),
        "o_totalprice": _dec(totalprice),
        "o_orderdate": _date(odate),
        "o_orderpriority": dict_col(uniform(i, 3, 0, 4), S.PRIORITIES, device),
        "o_clerk": gen_text("prefix_randint", i, 5, 9, max(int(1000 * sf), 1), device, inject="Clerk#"),
        "o_shippriority": _i32(torch.zeros(no_loc, dtype=torch.int64, device=device)),
        "o_comment": gen_text("words", i, 6, 3, 12, device, S.WORDS),
    }
    part = "o_orderkey" if world > 1 else None
    orders = MemoryTable(ocols, no_loc, partitioned_by=part)
    lineitem = MemoryTable(lcols, L, partitioned_by="l_orderkey" if world > 1 else None)
    return orders, lineitem


#: multi-rank layout: the fact tables are hash-partitioned by order key
#: (co-located, so lineitem-orders joins and per-order aggregation are
#: rank-local) and every dimension table is replicated on every rank (at SF100
#: they are ~125M rows, ~8 GB decoded, against 288 GB of HBM per GPU), so a
#: fact-dimension join needs no exchange at all: only aggregate merges and
#: final results cross xGMI. ``replicate_dims=False`` hash-partitions every
#: table by its primary key instead (exercises the shuffle paths).
PARTITIONED = ("orders", "lineitem")
#: primary-key partitioning of every table (``replicate_dims=False``)
PARTITION_KEY = {"region": None, "nation": None, "supplier": "s_suppkey", "customer": "c_custkey",
                 "part": "p_partkey", "partsupp": "ps_partkey", "orders": "o_orderkey", "lineitem": "l_orderkey"}
REPLICATED = ("region", "nation", "supplier", "customer", "part", "partsupp")
#: the column every generated table is stored in ascending order of
CLUSTER_KEY = {"region": "r_regionkey", "nation": "n_nationkey", "supplier": "s_suppkey", "customer": "c_custkey",
               "part": "p_partkey", "partsupp": "ps_partkey", "orders": "o_orderkey", "lineitem": "l_orderkey"}


def generate(sf: float, device="cpu", rank: int = 0, world: int = 1, lean: bool = False,
             tables: Optional[List[str]] = None, replicate_dims: bool = True,
             spmd: Optional[bool] = None) -> Dict[str, MemoryTable]:
    """All 8 TPC-H tables (this rank's partition) as device-resident MemoryTables.
    ``spmd`` (default: world > 1) tags the tables with the multi-rank layout
    (also for a forced world of one, parallel/comm.py ``force_spmd``)."""
    device = torch.device(device)
    want = set(tables or S.TABLES)
    out: Dict[str, MemoryTable] = {}
    spmd = world > 1 if spmd is None else spmd
    if spmd and world == 1:
        out = generate(sf, device, 0, 1, lean, tables, spmd=False, replicate_dims=replicate_dims)
        for t, tab in out.items():
            if replicate_dims and t in REPLICATED:
                tab.replicated, tab.partitioned_by = True, None
            elif t != "region" and t != "nation":
                tab.partitioned_by = PARTITION_KEY[t]
        return out
    if world > 1 and replicate_dims:
        dims = [t for t in REPLICATED if t in want]
        if dims:
            out.update(generate(sf, device, 0, 1, lean, dims, spmd=False))
            for t in dims:
                out[t].replicated, out[t].partitioned_by = True, None
        want -= set(REPLICATED)
        if not want:
            return out
    if "region" in want:
        out["region"] = gen_region(device)
    if "nation" in want:
        out["nation"] = gen_nation(device)
    if "supplier" in want:
        out["supplier"] = gen_supplier(sf, device, rank, world)
    if "customer" in want:
        out["customer"] = gen_customer(sf, device, rank, world)
    if "part" in want:
        out["part"] = gen_part(sf, device, rank, world)
    if "partsupp" in want:
        out["partsupp"] = gen_partsupp(sf, device, rank, world, lean)
    if "orders" in want or "lineitem" in want:
        o, l = gen_orders_lineitem(sf, device, rank, world, lean)
        if "orders" in want:
            out["orders"] = o
        if "lineitem" in want:
            out["lineitem"] = l
    for name, tab in out.items():
        tab.cluster_key = CLUSTER_KEY[name]
    return out


def register(engine, sf: float, rank: int = 0, world: int = 1, lean: bool = False,
             replicate_dims: bool = True, spmd: Optional[bool] = None) -> Dict[str, MemoryTable]:
    tabs = generate(sf, engine.device, rank, world, lean, replicate_dims=replicate_dims, spmd=spmd)
    for name, t in tabs.items():
        engine.register_table(name, t)
    return tabs


def to_arrow(tables: Dict[str, MemoryTable]) -> Dict[str, pa.Table]:
    out = {}
    for name, t in tables.items():
        out[name] = pa.table({k: c.to_arrow() for k, c in t.columns.items()})
    return out
