"""SPMD execution across processes (gloo on CPU): every rank generates its hash
partition of TPC-H, runs all 22 queries with shuffles / broadcasts / two-phase
aggregation, and rank 0's results must equal the sqlite oracle on the full
data. This is the multi-rank path bench.py takes over RCCL on N GPUs."""
import json
import os
import socket
import tempfile

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, sf, queries, device="cpu", low_thresholds=False, replicate_dims=True,
            budget_gb=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    if budget_gb is not None:
        os.environ["IGLOO_DEVICE_BUDGET_GB"] = str(budget_gb)
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen
    from igloo_amd.models.tpch import queries as Q
    from igloo_amd.parallel.comm import Communicator
    if low_thresholds:
        # small data must still take the large-data paths (sorted joins, run ids, Bloom probes)
        from igloo_amd.exec import joins as O
        from igloo_amd.ops import hashing as H
        from igloo_amd.parallel import exchange as X
        from igloo_amd.parallel import slicing as SL
        X.SMALL_AGG_GATHER = 0              # aggregates shuffle their partial groups
        X.SMALL_GATHER_STR_BYTES = 16       # long strings overflow the one-collective top-k gather
        X.PIPELINE_MIN_BYTES = 0            # fixed-width shuffles run as pipelined chunks
        X.PIPELINE_CHUNK_BYTES = 2048
        O.SORTED_JOIN_MIN_ROWS = 1000
        H.SORTED_CHECK_ROWS = 1000
        H.BLOOM_MIN_RATIO = 2
        SL.SLICE_MIN_ROWS = 1000
        SL.SLICE_MIXED_MIN_ROWS = 1000      # Q20 / Q22 slice partsupp / customer
        if low_thresholds == "sorted" and device == "cpu":
            # the GPU-only sorted-search join with its unique-key pairs (the
            # identity side of a foreign-key join) on CPU ranks: key_unique()
            # decided from the data, as resident-column tags do on the GPU
            import torch
            O.SORTED_PATHS_ON_CPU = True
            H.key_unique = lambda k: k.dim() == 1 and torch.unique(k).numel() == k.numel()
    comm = Communicator.init(backend="gloo", device=device, timeout_s=120)
    e = ig.QueryEngine(device=device, comm=comm)
    for name, t in datagen.generate(sf, device, rank, world, replicate_dims=replicate_dims).items():
        e.register_table(name, t)
    res = {}
    for q in queries:
        try:
            from igloo_amd.models.tpch.oracle import normalize
            rows = [[normalize(v) for v in r.values()] for r in e.sql(Q.QUERIES[q]).table.to_pylist()]
            res[q] = {"rows": rows, "collectives": e.last_metrics.get("collectives"),
                      "bytes": e.last_metrics.get("exchange_bytes"),
                      "morsels": (e.last_metrics.get("morsels") or {}).get("morsels", 0)}
            if low_thresholds:
                # steady state (what a repeated query costs): join statistics
                # memoised, pipelined-exchange chunks counted as one exchange
                e.sql(Q.QUERIES[q])
                res[q]["exchanges_warm"] = e.last_metrics.get("exchanges")
        except Exception as ex:  # noqa: BLE001
            res[q] = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    comm.shutdown()


def run_distributed(world, con, device="cpu", low_thresholds=False, replicate_dims=True, budget_gb=None):
    """Run TPC-H 1-22 on ``world`` ranks (gloo) and compare rank 0 with sqlite."""
    from igloo_amd.models.tpch import oracle
    qs = list(range(1, 23))
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.json")
        mp.start_processes(_worker, args=(world, _free_port(), out, 0.01, qs, device, low_thresholds, replicate_dims,
                                          budget_gb),
                           nprocs=world,
                           join=True, start_method="spawn")
        res = json.load(open(out))
    run_distributed.last = res
    return check(res, qs, con)


@pytest.mark.parametrize("world,replicate_dims,low", [(2, True, False), (3, True, True), (2, False, False),
                                                      (3, False, False), (4, True, True), (4, False, True),
                                                      (4, False, "sorted"),
                                                      (8, True, False), (8, True, True), (8, False, False)])
def test_tpch_distributed_gloo(world, replicate_dims, low, tpch_cpu):
    """Both multi-rank layouts: replicated dimension tables with fact tables
    co-partitioned by order key (the bench layout), and every table
    hash-partitioned by its primary key (every shuffle / broadcast path).
    ``low``: small data takes the large-data paths (sorted joins, key-range
    slices of replicated tables for Q2 / Q11 / Q16)."""
    _, _, con = tpch_cpu
    bad = run_distributed(world, con, replicate_dims=replicate_dims, low_thresholds=low)
    assert not bad, "\n".join(bad)
    calls = {int(q): r["collectives"] for q, r in run_distributed.last.items()}
    print("collectives per query:", calls)
    # packed exchanges + dense all-reduce aggregation: Q1 (4 groups) merges its
    # partial states with one all-reduce per op, Q6 (global sum) likewise
    assert calls[1] <= 2 and calls[6] <= 1, calls
    assert sum(calls.values()) <= 22 * 10, calls
    if replicate_dims:
        # fact-dimension joins are rank-local: the headline queries exchange
        # only aggregate merges and results
        assert all(calls[q] <= 6 for q in (1, 3, 5, 9, 15, 17, 18, 21)), calls
    if replicate_dims and not low:
        # the bench layout: no query needs more than 5 collectives (global
        # aggregates one all-reduce, grouped ones a structure all-gather plus
        # one data collective, a top-k result one fixed-size all-gather)
        assert max(calls.values()) <= 5 and sum(calls.values()) <= 60, calls
    if replicate_dims and low:
        # the SF100 code paths (range slices, sorted joins, shuffled partial
        # groups, pipelined exchanges in tiny chunks): bounded too
        assert max(calls.values()) <= 12 and sum(calls.values()) <= 120, calls
        # ... and in the steady state at most 6 exchanges a query, Q20 7 (its
        # runtime key filter's gather, the grouped lineitem aggregate's
        # shuffle, the part-key broadcast, the semi-join marks)
        warm = {int(q): r["exchanges_warm"] for q, r in run_distributed.last.items()}
        print("steady-state exchanges per query:", warm)
        assert all(v <= (7 if q == 20 else 6) for q, v in warm.items()), warm


def check(res, qs, con):
    from igloo_amd.models.tpch import oracle
    bad = []
    for q in qs:
        r = res[str(q)]
        if "error" in r:
            bad.append(f"Q{q}: {r['error']}")
            continue
        exp = [tuple(str(x) if isinstance(x, str) else x for x in row) for row in oracle.run_sqlite(con, q)]
        got = [tuple(row) for row in r["rows"]]
        d = oracle.rows_match(got, exp)
        if d:
            bad.append(f"Q{q}: {d}")
    return bad


def _num(x):
    if isinstance(x, str):
        try:
            return float(x)
        except ValueError:
            return x
    return x


_OUTER_SQL = {
    "left": "SELECT t2.k AS rk, count(*) AS n, sum(t1.a) AS s FROM t1 LEFT JOIN t2 ON t1.k = t2.k "
            "GROUP BY t2.k ORDER BY rk NULLS FIRST",
    "right": "SELECT t1.k AS lk, count(*) AS n, sum(t2.b) AS s FROM t1 RIGHT JOIN t2 ON t1.k = t2.k "
             "GROUP BY t1.k ORDER BY lk NULLS FIRST",
    "full": "SELECT t1.k AS lk, count(*) AS n FROM t1 FULL JOIN t2 ON t1.k = t2.k "
            "GROUP BY t1.k ORDER BY lk NULLS FIRST",
    "full_r": "SELECT t2.k AS rk, count(*) AS n FROM t1 FULL JOIN t2 ON t1.k = t2.k "
              "GROUP BY t2.k ORDER BY rk NULLS FIRST",
}


def _outer_tables(rank, world):
    """t1 (k 0..99) and t2 (k 50..149, two rows per key), hash-partitioned by k
    with the engine's partition function (a world of one holds everything)."""
    import numpy as np
    import pyarrow as pa
    import torch
    from igloo_amd.ops.misc import partition_ids
    k1 = np.arange(100, dtype=np.int64)
    k2 = np.repeat(np.arange(50, 150, dtype=np.int64), 2)

    def mine(k):
        if world == 1:
            return np.ones(len(k), dtype=bool)
        return partition_ids(torch.from_numpy(k), world).numpy() == rank
    m1, m2 = mine(k1), mine(k2)
    t1 = pa.table({"k": k1[m1], "a": (k1 * 3)[m1]})
    t2 = pa.table({"k": k2[m2], "b": (k2 + 1)[m2]})
    return t1, t2


def _outer_worker(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import igloo_amd as ig
    from igloo_amd.catalog import MemoryTable
    from igloo_amd.parallel.comm import Communicator
    comm = Communicator.init(backend="gloo", device="cpu", timeout_s=120)
    e = ig.QueryEngine(device="cpu", comm=comm)
    t1, t2 = _outer_tables(rank, world)
    e.register_table("t1", MemoryTable.from_arrow(t1, partitioned_by="k"))
    e.register_table("t2", MemoryTable.from_arrow(t2, partitioned_by="k"))
    res = {name: e.query(sql).to_pylist() for name, sql in _OUTER_SQL.items()}
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    comm.shutdown()


def test_outer_join_null_group_placement():
    """GROUP BY the NULL-padded side's key of a co-partitioned outer join:
    NULL-padded rows live on every rank, so the key must not be taken as the
    output's placement (one NULL group, not one per rank)."""
    import igloo_amd as ig
    from igloo_amd.catalog import MemoryTable
    e = ig.QueryEngine(device="cpu")
    t1, t2 = _outer_tables(0, 1)
    e.register_table("t1", MemoryTable.from_arrow(t1))
    e.register_table("t2", MemoryTable.from_arrow(t2))
    want = {name: e.query(sql).to_pylist() for name, sql in _OUTER_SQL.items()}
    assert sum(r["rk"] is None for r in want["left"]) == 1
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.json")
        mp.start_processes(_outer_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
        got = json.load(open(out))
    for name in _OUTER_SQL:
        assert got[name] == want[name], name


def _wide_worker(rank, world, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from decimal import Decimal
    import pyarrow as pa
    import igloo_amd as ig
    from igloo_amd.catalog import MemoryTable
    from igloo_amd.parallel.comm import Communicator
    comm = Communicator.init(backend="gloo", device="cpu", timeout_s=120)
    n = 4000
    big = 9 * 10**16
    rows = range(rank, n, world)          # this rank's slice
    t = pa.table({"g": pa.array([i % 7 for i in rows], pa.int64()),
                  "v": pa.array([Decimal(big + i).scaleb(-2) * (1 if i % 3 else -1) for i in rows],
                                pa.decimal128(18, 2))})
    e = ig.QueryEngine(device="cpu", comm=comm)
    e.register_table("t", MemoryTable.from_arrow(t))
    r = e.query("SELECT g, sum(v) AS s, count(*) AS n FROM t GROUP BY g ORDER BY g").to_pylist()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump([{k: str(v) for k, v in x.items()} for x in r], f)
    comm.shutdown()


def test_distributed_aggregate_merges_128bit_partial_sums():
    """Per-rank partial SUMs past 64 bits (wide decimals, e.g. SF100 charge
    sums) merge exactly across ranks."""
    from decimal import Decimal
    big = 9 * 10**16
    want = {}
    for i in range(4000):
        v = Decimal(big + i).scaleb(-2) * (1 if i % 3 else -1)
        s, c = want.get(i % 7, (Decimal(0), 0))
        want[i % 7] = (s + v, c + 1)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.json")
        mp.start_processes(_wide_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
        got = json.load(open(out))
    assert [int(r["g"]) for r in got] == list(range(7))
    for r in got:
        s, c = want[int(r["g"])]
        assert Decimal(r["s"]) == s and int(r["n"]) == c, r


def _surface_worker(rank, world, port, out_path):
    """The SQL-surface suite (tests/test_sql_surface.py: windows, set
    operations, recursive CTEs, grouping sets) over tables whose rows are
    spread round-robin over the ranks."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import pyarrow as pa
    import igloo_amd as ig
    import test_sql_surface as TS
    from igloo_amd.catalog import MemoryTable
    from igloo_amd.parallel.comm import Communicator
    comm = Communicator.init(backend="gloo", device="cpu", timeout_s=120)
    e = ig.QueryEngine(device="cpu", comm=comm)
    full = TS._engine("cpu")
    for name in ("t", "a", "b", "e"):
        tab = full.catalog.get_table(name)
        arrow = pa.table({f.name: tab.columns[f.name].to_arrow() for f in tab.schema()})
        mine = arrow.take(pa.array(list(range(rank, arrow.num_rows, world)), pa.int64()))
        e.register_table(name, MemoryTable.from_arrow(mine))
    res = {}
    for i, (q, _) in enumerate(TS.CASES):
        try:
            res[i] = [list(r.values()) for r in e.query(q).to_pylist()]
        except Exception as ex:  # noqa: BLE001
            res[i] = {"error": f"{type(ex).__name__}: {ex}"}
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f, default=str)
    comm.shutdown()


@pytest.mark.parametrize("world", [2, 3])
def test_sql_surface_distributed(world):
    """Window functions (shuffled by a shared PARTITION BY key, else
    gathered), INTERSECT / EXCEPT [ALL], recursive CTEs and GROUPING SETS on
    several gloo ranks match sqlite."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import test_sql_surface as TS
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res.json")
        mp.start_processes(_surface_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                           start_method="spawn")
        got = json.load(open(out))
    bad = []
    for i, (q, oracle) in enumerate(TS.CASES):
        r = got[str(i)]
        if isinstance(r, dict):
            bad.append(f"{q}: {r['error']}")
            continue
        if TS._rows(tuple(x) for x in r) != TS._expected(q, oracle):
            bad.append(q)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("world", [2, 3])
def test_tpch_distributed_bounded_memory(world, tpch_cpu):
    """Bounded-memory execution under SPMD: a per-rank device
    budget far below the data makes filtered scans stream and aggregates run
    as morsel pipelines whose rank-agreed morsel counts keep every rank's
    collectives in step; all 22 queries still match sqlite."""
    _, _, con = tpch_cpu
    bad = run_distributed(world, con, replicate_dims=False, budget_gb=0.0004)
    assert not bad, "\n".join(bad)
    streamed = [int(q) for q, r in run_distributed.last.items() if r.get("morsels")]
    assert len(streamed) >= 10, streamed
