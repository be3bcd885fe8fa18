"""TPC-H substitution parameters (models/tpch/params.py): every generated
query stream runs on the engine and matches the independent sqlite oracle
(SF0.01, CPU) — the ad-hoc workload bench.py ``--vary-params`` times."""
import random

import pytest

from igloo_amd.models.tpch import oracle, params
from igloo_amd.models.tpch.queries import QUERIES


def test_validation_text_when_no_rng():
    assert all(params.query(q) == QUERIES[q] for q in QUERIES)


def test_every_query_substitutes_and_is_deterministic():
    a, b = params.stream(range(1, 23), 11), params.stream(range(1, 23), 11)
    assert a == b
    c = params.stream(range(1, 23), 12)
    assert sum(a[q] != QUERIES[q] for q in a) >= 20
    assert a != c


@pytest.mark.parametrize("seed", [1, 2])
def test_param_streams_match_sqlite(seed, tpch_cpu):
    e, _, con = tpch_cpu
    bad = []
    for q, sql in params.stream(range(1, 23), seed, 0.01).items():
        got = [tuple(oracle.normalize(v) for v in r.values()) for r in e.sql(sql).table.to_pylist()]
        exp = [tuple(str(x) if isinstance(x, str) else x for x in row) for row in con.execute(oracle.to_sqlite(sql))]
        d = oracle.rows_match(got, exp)
        if d:
            bad.append(f"Q{q}: {d}")
    assert not bad, "\n".join(bad)
