"""TPC-H on the GPU (gfx950 kernels) vs the CPU engine and the sqlite oracle."""
import pytest

from igloo_amd.models.tpch import oracle, queries

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tpch_gpu(gpu_device):
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen
    e = ig.QueryEngine(device=gpu_device)
    tabs = datagen.register(e, 0.01)
    return e, tabs


def test_gpu_datagen_matches_cpu(tpch_gpu, tpch_cpu):
    _, gt = tpch_gpu
    _, ct, _ = tpch_cpu
    for name in ct:
        for col in ct[name].columns:
            a = ct[name].columns[col].to_arrow()
            b = gt[name].columns[col].to_arrow()
            assert a.equals(b), f"{name}.{col} differs between CPU and GPU generation"


@pytest.mark.parametrize("q", list(range(1, 23)))
def test_tpch_gpu_query(tpch_gpu, tpch_cpu, q):
    e, _ = tpch_gpu
    _, _, con = tpch_cpu
    got = [tuple(r.values()) for r in e.sql(queries.QUERIES[q]).table.to_pylist()]
    exp = oracle.run_sqlite(con, q)
    diff = oracle.rows_match(got, exp)
    assert not diff, f"Q{q}: {diff}"


def test_native_kernels_were_used(tpch_gpu):
    from igloo_amd.ops._lib import KERNEL_CALLS
    for k in ("select", "join_build", "join_probe", "groupby", "agg_update", "gather_multi"):
        assert KERNEL_CALLS[k] > 0, f"{k} never launched: {dict(KERNEL_CALLS)}"


def test_tpch_distributed_gpu_ranks(tpch_cpu):
    """Two SPMD ranks sharing the one GPU (gloo, collectives staged through the
    host): exercises every GPU-only operator path (fused scans, sorted joins,
    run-id group-by, HLL NDV merges, runtime filters) under hash partitioning,
    shuffles and two-phase aggregation — the code the 8-GPU RCCL run takes."""
    import test_distributed_cpu as D
    _, _, con = tpch_cpu
    bad = D.run_distributed(2, con, device="cuda:0", low_thresholds=True)
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("world,replicate_dims", [(4, True), (4, False), (8, True), (8, False)])
def test_tpch_distributed_gpu_ranks_driver_worlds(world, replicate_dims, tpch_cpu):
    """All 22 queries at the driver's scaling world sizes (4 and 8 ranks), every
    rank's operators on the one GPU (collectives staged through gloo), both
    layouts: replicated dimensions with co-partitioned facts (the bench layout)
    and every table hash-partitioned (every shuffle / broadcast branch). Low
    thresholds make SF0.01 take the SF100 code paths (sorted joins, range
    slices, shuffled partial groups, pipelined chunked exchanges)."""
    import test_distributed_cpu as D
    _, _, con = tpch_cpu
    bad = D.run_distributed(world, con, device="cuda:0", low_thresholds=True, replicate_dims=replicate_dims)
    assert not bad, "\n".join(bad)
    calls = {int(q): r["collectives"] for q, r in D.run_distributed.last.items()}
    assert sum(calls.values()) > 0, calls
