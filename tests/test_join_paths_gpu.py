"""Every physical join strategy vs the CPU engine on the same data.

The GPU picks among hash build/probe (with or without the Bloom pre-filter),
reverse builds for semi/anti/left joins against a much larger side, and the
binary-search path when the big side's key column is sorted. Thresholds are
lowered so small inputs exercise each path; results must equal the CPU
reference exactly (order-insensitive)."""
import numpy as np
import pyarrow as pa
import pytest

import igloo_amd as ig
from igloo_amd.exec import operators as O
from igloo_amd.ops import hashing as H

pytestmark = pytest.mark.gpu


def _tables(seed=5, n_big=200_000, n_small=3_000, sorted_big=True):
    r = np.random.default_rng(seed)
    k = r.integers(0, n_big // 4, n_big)
    if sorted_big:
        k = np.sort(k)
    big = pa.table({"bk": pa.array(k, pa.int64()), "bs": pa.array(r.integers(0, 7, n_big), pa.int64()),
                    "bv": pa.array(r.integers(-100, 100, n_big), pa.int64())})
    sk = r.integers(-10, n_big // 4 + 10, n_small)
    sv = pa.array(r.integers(0, 7, n_small), pa.int64())
    small = pa.table({"sk": pa.array(sk, pa.int64()), "ss": sv,
                      "sn": pa.array([None if i % 17 == 0 else int(x) for i, x in enumerate(sk)], pa.int64())})
    return big, small


QUERIES = [
    "SELECT sk, bv FROM small JOIN big ON sk = bk",
    "SELECT sk, bv FROM small JOIN big ON sk = bk AND bs <> ss",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk)",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs <> ss)",
    "SELECT sk FROM small WHERE NOT EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs <> ss)",
    "SELECT sk FROM small WHERE EXISTS (SELECT 1 FROM big WHERE bk = sk AND bs < ss)",
    "SELECT sk FROM small WHERE NOT EXISTS (SELECT 1 FROM big WHERE bk = sk AND ss >= bs)",
    "SELECT sn, count(bv) AS c FROM small LEFT JOIN big ON sn = bk GROUP BY sn",
    "SELECT sk, count(*) AS c FROM small JOIN big ON sk = bk GROUP BY sk",
]


def _norm(t):
    return sorted((tuple((k, v) for k, v in sorted(r.items())) for r in t.to_pylist()), key=repr)


@pytest.mark.parametrize("sorted_big,perm", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_join_paths_match_cpu(gpu_device, monkeypatch, sorted_big, perm, qi):
    """perm: the unsorted resident big side is joined through its secondary
    (sorted permutation) index instead of a hash probe."""
    monkeypatch.setattr(O, "PERM_INDEX", perm)
    monkeypatch.setattr(O, "PERM_INDEX_MAX_FRAC", 1)
    monkeypatch.setattr(O, "SORTED_JOIN_MIN_ROWS", 1000)
    monkeypatch.setattr(H, "SORTED_CHECK_ROWS", 1000)
    monkeypatch.setattr(H, "BLOOM_MIN_RATIO", 2)
    big, small = _tables(sorted_big=sorted_big)
    res = {}
    for dev in ("cpu", gpu_device):
        e = ig.QueryEngine(device=dev)
        e.register_table("big", big)
        e.register_table("small", small)
        res[dev] = _norm(e.query(QUERIES[qi]))
    assert res["cpu"] == res[gpu_device]
