"""Key-range slices of replicated tables (parallel/slicing.py): every row
lands on exactly one rank, including int32 keys at the top of their range."""
import pytest
import torch

from igloo_amd import types as T
from igloo_amd.columnar import Column
from igloo_amd.parallel import slicing as SL


@pytest.mark.parametrize("keys", [
    [2**31 - 4, 2**31 - 3, 2**31 - 2, 2**31 - 1, 2**31 - 1],   # chunk 1, MAX repeated
    [2**31 - 2, 2**31 - 1, 2**31 - 1],                          # fewer keys than ranks
    [5, 5, 5],
    list(range(0, 1000, 7)),
    [-(2**31), -(2**31) + 1, 0, 2**31 - 1],
])
@pytest.mark.parametrize("world", [1, 3, 4, 8])
def test_range_slices_partition_rows(keys, world):
    kt = torch.tensor(keys, dtype=torch.int32)
    n = kt.numel()
    kmin, kmax = int(kt[0]), int(kt[-1])
    chunk = SL.range_chunk(kmin, kmax, world)
    owned = []
    for r in range(world):
        a, b = SL._range_cut_rows(kt, n, kmin, kmax, chunk, r)
        assert 0 <= a <= b <= n
        owned += list(range(a, b))
        # a rank's rows hold exactly its keys
        for i in range(a, b):
            assert kmin + r * chunk <= keys[i] < kmin + (r + 1) * chunk
    assert sorted(owned) == list(range(n)), (world, owned)


def test_slice_columns_int32_near_max():
    kt = torch.tensor([2**31 - 4, 2**31 - 3, 2**31 - 2, 2**31 - 1, 2**31 - 1], dtype=torch.int32)
    pay = torch.arange(5, dtype=torch.int64)
    got = []
    for r in range(4):
        cols = {"k": Column(T.INT32, kt.clone()), "v": Column(T.INT64, pay.clone())}
        out, rows, tag = SL.slice_columns(cols, 5, "k", 4, r)
        assert tag is not None
        got += out["v"].data.tolist()
    assert sorted(got) == [0, 1, 2, 3, 4]
