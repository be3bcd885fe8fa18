"""Query graphs (exec/graphs.py): a repeated query over unchanged data is
captured into one HIP graph once its host readbacks replay completely; every
later execution is a graph launch plus one device check. Results must stay
identical to the eager executions; a replayed value that no longer matches the
device, or a changed generated-kernel set, drops the graph and the query runs
eagerly again with the right answer."""
import pytest

pytestmark = pytest.mark.gpu

QS = [1, 3, 4, 5, 6, 9, 10, 12, 13, 14, 16, 18, 19, 21, 22]


@pytest.fixture(scope="module")
def gpu_engine():
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, 0.1)
    return e


def _run(e, sql, n):
    from igloo_amd.utils.digest import digest
    out = []
    for _ in range(n):
        out.append((digest(e.sql(sql).table), e.last_metrics["speculation"]))
    return out


def test_tpch_queries_run_as_graphs(gpu_engine):
    from igloo_amd.exec import graphs
    from igloo_amd.models.tpch import queries
    from igloo_amd.ops import jit
    jit.wait_all(timeout=120)
    graphed = []
    for q in QS:
        runs = _run(gpu_engine, queries.QUERIES[q], 7)
        assert len({d for d, _ in runs}) == 1, (q, runs)
        if runs[-1][1] == "graph":
            graphed.append(q)
    print("graphed:", graphed, graphs.STATS)
    assert graphs.STATS["failed"] == 0 and graphs.STATS["mismatch"] == 0, graphs.STATS
    assert len(graphed) >= len(QS) * 2 // 3, (graphed, graphs.STATS)


def _graph_state(e, sql):
    for st in e._spec.values():
        g = st.get("graph")
        if g is not None:
            yield st, g


def test_graph_mismatch_reexecutes(gpu_engine):
    e = gpu_engine
    sql = ("SELECT l_returnflag, count(*) AS n, sum(l_quantity) AS q FROM lineitem "
           "WHERE l_shipdate <= date '1998-09-01' GROUP BY l_returnflag ORDER BY l_returnflag")
    runs = _run(e, sql, 6)
    assert runs[-1][1] == "graph", runs
    want = runs[-1][0]
    # corrupt what the graph compares its replayed values against: the next
    # execution must notice, drop the graph and recompute eagerly
    for st, g in list(_graph_state(e, sql)):
        if g.expected.numel():
            g.expected.add_(1)
    again = _run(e, sql, 1)
    assert again[0][0] == want
    assert again[0][1] != "graph"
    assert _run(e, sql, 1)[0][0] == want


def test_graph_recaptured_after_jit_generation_change(gpu_engine, monkeypatch):
    from igloo_amd.ops import jit
    e = gpu_engine
    sql = "SELECT o_orderpriority, count(*) AS n FROM orders GROUP BY o_orderpriority ORDER BY o_orderpriority"
    runs = _run(e, sql, 6)
    assert runs[-1][1] == "graph", runs
    real = jit.generation
    monkeypatch.setattr(jit, "generation", lambda: (real() or 0) + 1000)
    after = _run(e, sql, 5)
    assert {d for d, _ in after} == {runs[-1][0]}
    assert after[0][1] != "graph"


def _until_graph(e, sql, n=8):
    from igloo_amd.utils.digest import digest
    seen = []
    for _ in range(n):
        d = digest(e.sql(sql).table)
        seen.append((d, e.last_metrics["speculation"]))
        if seen[-1][1] == "graph":
            break
    return seen


def test_graph_replay_sees_parquet_rewrite(tmp_path):
    """CDC under graphs: a query that has become a graph must notice a
    rewritten source file (the replay itself never reaches the scan)."""
    import os
    import pyarrow as pa
    import pyarrow.parquet as pq
    import igloo_amd as ig
    from igloo_amd.ops import jit
    d = tmp_path / "t"
    d.mkdir()
    n = 20_000

    def write(mult):
        pq.write_table(pa.table({"k": pa.array(range(n), pa.int64()),
                                 "v": pa.array([i * mult for i in range(n)], pa.int64())}), str(d / "a.parquet"))
    write(1)
    e = ig.QueryEngine(device="cuda:0")
    e.register_parquet("t", str(d))
    sql = "SELECT count(*) AS n, sum(v) AS s FROM t WHERE k < 5000"
    jit.wait_all(timeout=120)
    runs = _until_graph(e, sql)
    assert runs[-1][1] == "graph", runs
    assert e.query(sql).to_pylist() == [{"n": 5000, "s": sum(range(5000))}]
    write(3)
    st = os.stat(d / "a.parquet")
    os.utime(d / "a.parquet", ns=(st.st_atime_ns, st.st_mtime_ns + 5_000_000_000))
    e.cdc._last_poll.clear()          # skip the 1 s poll interval
    assert e.query(sql).to_pylist() == [{"n": 5000, "s": 3 * sum(range(5000))}]
    assert e.last_metrics["speculation"] != "graph"
    assert e.graph_stats["dropped_stale"] >= 1
    runs = _until_graph(e, sql)
    assert runs[-1][1] == "graph", runs
    assert e.query(sql).to_pylist() == [{"n": 5000, "s": 3 * sum(range(5000))}]


def test_graph_pools_bounded_by_hbm_budget():
    """Graph pools count against the engine's HBM budget: past it the least
    recently replayed graphs are dropped, answers unchanged."""
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops import jit
    from igloo_amd.utils.digest import digest
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, 0.02)
    jit.wait_all(timeout=120)
    want = {q: digest(ig.QueryEngine(device="cuda:0", catalog=e.catalog).sql(queries.QUERIES[q]).table)
            for q in (1, 3, 6)}
    e.hbm_budget = 1      # every graph beyond the newest one is over budget
    for q in (1, 3, 6, 1):
        runs = _until_graph(e, queries.QUERIES[q])
        assert {x for x, _ in runs} == {want[q]}, q
        assert runs[-1][1] == "graph", (q, runs)
        assert len(e._graphs) == 1 and e.graph_bytes == e._graphs[next(iter(e._graphs))]["graph"].nbytes
    assert e.graph_stats["evicted"] >= 3, e.graph_stats
    e.hbm_budget = None
