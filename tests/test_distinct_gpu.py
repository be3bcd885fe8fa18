"""COUNT / SUM / AVG (DISTINCT) on the device (ops/hashing.py
first_rows_mask keeps the first row of every (group, value) pair) against the
CPU engine, with NULL values, a global aggregate and a direct-mapped and a
hashed pair domain."""
import numpy as np
import pyarrow as pa
import pytest

import igloo_amd as ig

pytestmark = pytest.mark.gpu


def _norm(t):
    return sorted((tuple(sorted(r.items())) for r in t.to_pylist()), key=repr)


@pytest.mark.parametrize("span", [50, 5_000_000])
def test_distinct_aggregates_match_cpu(gpu_device, span):
    r = np.random.default_rng(11)
    n = 200_000
    v = r.integers(0, span, n)
    t = pa.table({"g": pa.array(r.integers(0, 300, n), pa.int64()),
                  "v": pa.array([None if i % 23 == 0 else int(x) for i, x in enumerate(v)], pa.int64())})
    qs = ["SELECT g, count(DISTINCT v) AS c, sum(DISTINCT v) AS s FROM t GROUP BY g",
          "SELECT count(DISTINCT v) AS c, avg(DISTINCT v) AS a FROM t",
          "SELECT g % 7 AS h, count(DISTINCT v) AS c FROM t WHERE v > 10 GROUP BY g % 7"]
    for q in qs:
        res = {}
        for dev in ("cpu", gpu_device):
            e = ig.QueryEngine(device=dev)
            e.register_table("t", t)
            res[dev] = _norm(e.query(q))
        assert res["cpu"] == res[gpu_device], q
