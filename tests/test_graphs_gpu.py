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
