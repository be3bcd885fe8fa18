"""Test configuration: `gpu` marker + native build once per session."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# generated kernels compile on first use (not in the background) so every GPU
# test exercises the code path warm queries take (igloo_amd/ops/jit.py)
os.environ.setdefault("IGLOO_JIT", "sync")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the gfx950 kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    from igloo_amd import _build
    _build.build()
    yield


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return "cuda:0"


@pytest.fixture(scope="session")
def tpch_cpu():
    """SF0.01 TPC-H on CPU + sqlite oracle connection."""
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, oracle
    e = ig.QueryEngine(device="cpu")
    tabs = datagen.register(e, 0.01)
    con = oracle.load_sqlite(datagen.to_arrow(tabs))
    return e, tabs, con
