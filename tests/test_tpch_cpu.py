"""All 22 TPC-H queries on the CPU path vs the sqlite oracle (SF 0.01)."""
import pytest

from igloo_amd.models.tpch import oracle, queries


@pytest.mark.parametrize("q", list(range(1, 23)))
def test_tpch_query_matches_sqlite(tpch_cpu, q):
    e, _, con = tpch_cpu
    got = [tuple(r.values()) for r in e.sql(queries.QUERIES[q]).table.to_pylist()]
    exp = oracle.run_sqlite(con, q)
    diff = oracle.rows_match(got, exp)
    assert not diff, f"Q{q}: {diff}"
