"""Host reference paths of the small ops helpers the device paths mirror
(ops/select.py, ops/hashing.py): counts, offsets with a device-side total,
composite-key packing and the first-row-of-group mask."""
import torch

from igloo_amd.ops import hashing as H
from igloo_amd.ops.select import count_true, exclusive_scan, mask_to_indices, offsets_from_lengths


def test_count_true_and_indices():
    g = torch.Generator().manual_seed(1)
    m = torch.rand(10_001, generator=g) < 0.3
    assert count_true(m) == int(m.sum())
    idx = mask_to_indices(m)
    assert torch.equal(idx.long(), torch.nonzero(m).flatten())
    assert getattr(idx, "_igloo_incr", False)


def test_offsets_from_lengths_host_and_device_total():
    lens = torch.tensor([3, 0, 5, 1], dtype=torch.int64)
    off, tot = offsets_from_lengths(lens)
    assert off.tolist() == [0, 3, 3, 8, 9] and tot == 9
    off2, tot2 = offsets_from_lengths(lens, host_total=False)
    assert off2.tolist() == off.tolist() and int(tot2[0]) == 9
    ex, t = exclusive_scan(lens)
    assert ex.tolist() == [0, 3, 3, 8] and t == 9


def test_pack_keys_equality_preserving():
    g = torch.Generator().manual_seed(2)
    cols = [torch.randint(-5, 40, (5000,), generator=g), torch.randint(0, 3, (5000,), generator=g).to(torch.int32),
            torch.randint(10**6, 10**6 + 50, (5000,), generator=g)]
    packed = H.pack_keys(cols)
    tup = list(zip(*[c.tolist() for c in cols]))
    by_tuple = {}
    for t, p in zip(tup, packed.tolist()):
        assert by_tuple.setdefault(t, p) == p          # equal tuples -> equal keys
    assert len(set(by_tuple.values())) == len(by_tuple)  # distinct tuples -> distinct keys
    left = [c[:2000] for c in cols]
    right = [c[2000:] for c in cols]
    pl, pr = H.pack_keys_pair(left, right)
    assert torch.equal(torch.cat([pl, pr]), packed)


def test_first_rows_mask_host():
    k = torch.tensor([5, 3, 5, 7, 3, 3, 9], dtype=torch.int64)
    m = H.first_rows_mask(k)
    assert m.tolist() == [True, True, False, True, False, False, True]
