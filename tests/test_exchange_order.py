"""Exchanges pack columns in one order on every rank (parallel/exchange.py
wire_order), whatever order a rank's batch dict was built in: a join side
taken as the identity on one rank keeps its cached columns first
(exec/joins.py LateBatch.materialize) -- TPC-H Q9 on 4 partitioned ranks lost
rows when the orders differed."""
import torch

from igloo_amd import types as T
from igloo_amd.columnar import Batch, Column
from igloo_amd.exec.joins import LateBatch
from igloo_amd.parallel.exchange import wire_order


def _col(v):
    return Column(T.INT64, torch.tensor(v, dtype=torch.int64))


def test_wire_order_is_by_column_id():
    a = Batch({5: _col([1]), 2: _col([2]), 9: _col([3])}, 1)
    b = Batch({9: _col([3]), 5: _col([1]), 2: _col([2])}, 1)
    assert wire_order(a) == wire_order(b) == [2, 5, 9]


def test_materialize_keeps_base_order_with_cached_columns():
    base = Batch({1: _col([10, 11, 12]), 2: _col([20, 21, 22]), 3: _col([30, 31, 32])}, 3)
    idx = torch.tensor([2, 0], dtype=torch.int64)
    fresh = LateBatch([(base, idx)], 2)
    cached = LateBatch([(base, idx)], 2)
    cached.gather(3)                     # gathered earlier (a join key) on this rank only
    m1, m2 = fresh.materialize(), cached.materialize()
    assert list(m1.columns) == list(m2.columns) == [1, 2, 3]
    for c in (1, 2, 3):
        assert torch.equal(m1.columns[c].data, m2.columns[c].data)
