"""Cache tier + CDC wired into execution, and Parquet statistics pruning.

BASELINE config 5 shape: an Iceberg fact table joined with a Postgres
dimension table (fake wire-protocol server), both served from the engine's
cache tier (reference crates/cache/src/lib.rs:12-56; README.md:42 "automatic
cache invalidation via CDC")."""
import os

import pyarrow as pa
import pyarrow.parquet as pq

import igloo_amd as ig
from igloo_amd.connectors import iceberg
from igloo_amd.connectors.postgres import PostgresTable
from igloo_amd.models.tpch import parquet_gen
from tests.fakedb import FakePostgres


def _dim():
    return pa.table({"c_id": pa.array([1, 2, 3], pa.int64()), "c_name": pa.array(["ann", "bob", "cat"])})


def _facts(scale=1):
    return pa.table({"o_cid": pa.array([1, 1, 2, 3, 3, 3], pa.int64()),
                     "o_amt": pa.array([x * scale for x in (5, 6, 7, 8, 9, 10)], pa.int64())})


SQL = ("SELECT c_name, sum(o_amt) AS total FROM orders JOIN customers ON o_cid = c_id "
       "GROUP BY c_name ORDER BY c_name")


def test_iceberg_join_postgres_cache_hit_eviction_and_snapshot_invalidation(tmp_path):
    srv = FakePostgres({"customers": _dim(), "versions": pa.table({"v": pa.array([1], pa.int64())})}, auth="md5")
    try:
        path = str(tmp_path / "orders_ice")
        iceberg.write_table(path, _facts(), snapshot_id=1)
        e = ig.QueryEngine(device="cpu")
        orders = e.register_iceberg("orders", path)
        cust = e.register_table("customers", PostgresTable(srv.dsn, "customers",
                                                           version_sql="SELECT max(v) FROM versions"))
        want = [{"c_name": "ann", "total": 11}, {"c_name": "bob", "total": 7}, {"c_name": "cat", "total": 27}]
        assert e.query(SQL).to_pylist() == want
        assert orders.misses == 2 and orders.hits == 0 and cust.misses == 2
        copies = sum(q.startswith("SELECT \"") for q in srv.queries)
        assert e.query(SQL).to_pylist() == want          # second run: cache hits, no COPY
        assert orders.hits == 2 and cust.hits == 2
        assert sum(q.startswith("SELECT \"") for q in srv.queries) == copies
        assert e.cache.stats["hits"] >= 4
        # snapshot bump: a new Iceberg commit replaces the data files
        iceberg.write_table(path, _facts(scale=10), snapshot_id=2)
        orders.cdc._last_poll.clear()                    # skip the 1 s poll interval
        got = e.query(SQL).to_pylist()
        assert got[0] == {"c_name": "ann", "total": 110}, got
        assert any(ev.table == "orders" and ev.version == 2 for ev in e.cdc.events)
    finally:
        srv.close()


def test_cache_demotes_to_host_under_tiny_hbm_budget(tmp_path):
    pq.write_table(_facts(), str(tmp_path / "o.parquet"))
    e = ig.QueryEngine(device="cpu", cache_hbm_gb=40 / 2**30)   # 40 bytes: one int64 column of 6 rows fits
    src = e.register_parquet("orders", str(tmp_path / "o.parquet"))
    assert e.query("SELECT sum(o_amt) AS s FROM orders WHERE o_cid > 1").to_pylist() == [{"s": 34}]
    assert e.cache.stats["evictions"] >= 1 and e.cache.hbm_used <= 40
    assert e.cache.host_used > 0
    # demoted entries are promoted back on the next scan, answers unchanged
    assert e.query("SELECT sum(o_amt) AS s FROM orders WHERE o_cid > 1").to_pylist() == [{"s": 34}]
    assert src.hits >= 2


def test_parquet_file_rewrite_invalidates(tmp_path):
    d = tmp_path / "ds"
    d.mkdir()
    pq.write_table(_facts(), str(d / "a.parquet"))
    e = ig.QueryEngine(device="cpu")
    src = e.register_parquet("orders", str(d))
    assert e.query("SELECT count(*) AS n FROM orders").to_pylist() == [{"n": 6}]
    # a second file appears anywhere in the dataset -> new version -> re-read
    pq.write_table(_facts(), str(d / "b.parquet"))
    e.cdc._last_poll.clear()
    assert e.query("SELECT count(*) AS n FROM orders").to_pylist() == [{"n": 12}]
    assert len(src.files) == 2


def test_row_group_statistics_pruning(tmp_path):
    n = 10_000
    t = pa.table({"k": pa.array(range(n), pa.int64()),
                  "d": pa.array([i % 97 for i in range(n)], pa.int32()),
                  "p": pa.array([i * 3 for i in range(n)], pa.decimal128(15, 2)),
                  "s": pa.array([f"s{i // 1000}" for i in range(n)])})
    pq.write_table(t, str(tmp_path / "t.parquet"), row_group_size=1000)
    e = ig.QueryEngine(device="cpu")
    src = e.register_parquet("t", str(tmp_path / "t.parquet"), cache=False)
    r = e.query("SELECT count(*) AS n, sum(d) AS sd FROM t WHERE k >= 2500 AND k < 4000").to_pylist()
    assert r == [{"n": 1500, "sd": sum(i % 97 for i in range(2500, 4000))}]
    st = src.last_gpu_stats
    assert st["row_groups"] == 10 and st["row_groups_read"] == 2 and st["row_groups_pruned"] == 8
    r = e.query("SELECT count(*) AS n FROM t WHERE k IN (5, 9999)").to_pylist()
    assert r == [{"n": 2}] and src.last_gpu_stats["row_groups_read"] == 2
    r = e.query("SELECT count(*) AS n FROM t WHERE p > 29000.00").to_pylist()   # decimal stats (p = 3k)
    assert r == [{"n": sum(1 for i in range(n) if i * 3 > 29000)}]
    assert src.last_gpu_stats["row_groups_read"] == 1
    r = e.query("SELECT count(*) AS n FROM t WHERE s = 's7'").to_pylist()
    assert r == [{"n": 1000}] and src.last_gpu_stats["row_groups_read"] == 1
    # a predicate the statistics cannot refute reads everything
    e.query("SELECT count(*) AS n FROM t WHERE d = 3")
    assert src.last_gpu_stats["row_groups_pruned"] == 0


def test_tpch_parquet_dataset_roundtrip(tmp_path):
    """The bench's dataset layout: written in parallel, read back through the
    cache tier with the same answers as the generated tables."""
    from igloo_amd.models.tpch import datagen, queries
    man = parquet_gen.write_dataset(0.01, str(tmp_path), device="cpu", rows_per_file=20_000, row_group=8192,
                                    threads=4)
    assert not man["reused"] and man["files"] > 8
    assert parquet_gen.write_dataset(0.01, str(tmp_path), device="cpu", rows_per_file=20_000, row_group=8192,
                                     threads=4)["reused"]
    ep = ig.QueryEngine(device="cpu")
    parquet_gen.register_dataset(ep, str(tmp_path), 0.01)
    eg = ig.QueryEngine(device="cpu")
    datagen.register(eg, 0.01)
    for q in (1, 3, 6, 13, 16):
        a = ep.query(queries.QUERIES[q])
        b = eg.query(queries.QUERIES[q])
        assert a.to_pylist() == b.to_pylist(), q
    li = os.path.join(parquet_gen.dataset_dir(str(tmp_path), 0.01), "lineitem")
    assert sorted(os.listdir(li))[0] == "part-00000.parquet"


def test_row_group_pruning_on_the_cached_path(tmp_path):
    """Statistics pruning also applies to scans served from the cache tier:
    the resident column is complete (the fill reads every row group) and a
    filtered scan hands out only the row ranges of the row groups the
    statistics cannot rule out."""
    n = 10_000
    t = pa.table({"k": pa.array(range(n), pa.int64()),
                  "d": pa.array([i % 97 for i in range(n)], pa.int32()),
                  "s": pa.array([f"s{i // 1000}" for i in range(n)])})
    pq.write_table(t, str(tmp_path / "t.parquet"), row_group_size=1000)
    e = ig.QueryEngine(device="cpu")
    src = e.register_parquet("t", str(tmp_path / "t.parquet"))      # cached (the default)
    assert type(src).__name__ == "CachedTable" and src.prunes
    for _ in range(2):   # miss (fill), then hit
        r = e.query("SELECT count(*) AS n, sum(d) AS sd FROM t WHERE k >= 2500 AND k < 4000").to_pylist()
        assert r == [{"n": 1500, "sd": sum(i % 97 for i in range(2500, 4000))}]
        assert src.last_prune_stats == {"row_groups": 10, "row_groups_read": 2, "row_groups_pruned": 8}
    assert src.hits >= 2
    # two separate ranges (an index gather), strings included
    r = e.query("SELECT count(*) AS n, min(s) AS lo, max(s) AS hi FROM t WHERE k IN (5, 9999)").to_pylist()
    assert r == [{"n": 2, "lo": "s0", "hi": "s9"}] and src.last_prune_stats["row_groups_read"] == 2
    r = e.query("SELECT count(*) AS n FROM t WHERE s = 's7'").to_pylist()
    assert r == [{"n": 1000}] and src.last_prune_stats["row_groups_read"] == 1
    e.query("SELECT count(*) AS n FROM t WHERE d = 3")
    assert src.last_prune_stats.get("row_groups_pruned", 0) == 0
