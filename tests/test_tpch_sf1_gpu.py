"""TPC-H at SF1 on the GPU with DEFAULT thresholds (no monkeypatching), so the
large-data paths the SF100 bench takes are the ones checked: sorted-key
range joins, run-id group-by over clustered keys, dense range / secondary
indexes, Bloom-filtered probes, narrow fused scans, radix sort / top-k.

Oracle: the CPU engine on the identical generated data (the generator is
bit-identical on CPU and GPU). Results are compared through bench.digest
(row count, exact decimal / integer sums, hashed multisets). The same
queries also run over Parquet files written from that data and decoded on
the GPU (cache tier), the bench's data path.

Reference parity: the reference's only end-to-end test asserts exact rows
of a Parquet query (crates/engine/tests/integration_test.rs:62-76)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
SF = 1.0


@pytest.fixture(scope="module")
def engines(tmp_path_factory):
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, parquet_gen
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    gpu = ig.QueryEngine(device="cuda:0")
    datagen.register(gpu, SF)
    cpu = ig.QueryEngine(device="cpu")
    datagen.register(cpu, SF)
    root = str(tmp_path_factory.mktemp("tpch_pq"))
    parquet_gen.write_dataset(SF, root, device="cuda:0", threads=8)
    torch.cuda.empty_cache()
    pq = ig.QueryEngine(device="cuda:0")
    parquet_gen.register_dataset(pq, root, SF)
    return gpu, cpu, pq


@pytest.mark.parametrize("q", range(1, 23))
def test_sf1_gpu_equals_cpu(engines, q):
    from igloo_amd.utils.digest import digest
    from igloo_amd.models.tpch import queries
    from igloo_amd.ops import _lib
    gpu, cpu, pq = engines
    _lib.KERNEL_CALLS.clear()
    want = digest(cpu.sql(queries.QUERIES[q]).table)
    got = digest(gpu.sql(queries.QUERIES[q]).table)
    assert got == want, f"Q{q} HBM-generated tables"
    assert sum(_lib.KERNEL_CALLS.values()) > 0   # the native kernels ran
    got_pq = digest(pq.sql(queries.QUERIES[q]).table)
    assert got_pq == want, f"Q{q} Parquet-sourced tables"
    print(f"Q{q} ok", flush=True)
