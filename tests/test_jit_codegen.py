"""Generated scan kernels (exec/fused_jit.py) compile for gfx950 with hiprtc
on the host (no GPU needed): Q1 / Q6 / Q19 shapes, masks, min/max, checked
and split sums, narrow and 8-byte columns."""
import pytest
import torch

from igloo_amd.exec import fused_jit as FJ
from igloo_amd.ops import _lib

pytestmark = pytest.mark.skipif(not _lib.have_native(), reason="native extension not built")


def _compile(src, name):
    code = _lib.native().jit_compile(src, name, "gfx950")
    assert len(code) > 1000
    return code


def cols(*widths):
    dt = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    return FJ._Shape([torch.zeros(8, dtype=dt[w]) for w in widths])


def test_mask_kernel_compiles():
    sh = cols(4, 1, 2, 8)
    terms = [(0, 0, 8766, 9130, 0), (1, 0, 5, 7, 0), (2, 1, -10, 23, 0), (3, 2, 0, 0, 0b1011),
             (0, 3, 0, 100, 3)]
    src = FJ.mask_source(sh, terms, has_mask=True)
    assert "igloo_jit_scan_mask" in src
    _compile(src, "igloo_jit_scan_mask")
    # the tiled variant: one select tile per workgroup step, its count stored with the mask
    tiled = FJ.mask_source(sh, terms, has_mask=True, tiled=True)
    assert "i64* __restrict__ tc" in tiled and f"{FJ.SELECT_TILE}" in tiled
    _compile(tiled, "igloo_jit_scan_mask")


def test_q6_shape_single_group():
    sh = cols(2, 1, 1, 4)      # shipdate, discount, quantity, extendedprice
    terms = [(0, 0, 8766, 9130, 0), (1, 0, 5, 7, 0), (2, 0, -(2**63), 2399, 0)]
    aggs = [(0, 0, ((3, 0, 1), (1, 0, 1)))]
    src = FJ.agg_source(sh, terms, False, [], 1, aggs, [False], 64)
    assert "add128" in src and "WG_ADD" not in src.split("void igloo_jit_scan_agg")[1]
    _compile(src, "igloo_jit_scan_agg")


def test_q1_shape_groups_split_and_chains():
    sh = cols(2, 1, 1, 2, 4, 1, 1)   # shipdate, returnflag, linestatus, qty, price, disc, tax
    terms = [(0, 0, -(2**63), 10471, 0)]
    keys = [(1, 0, 2), (2, 0, 1)]
    aggs = [(0, 0, ((3, 0, 1),)), (0, 0, ((4, 0, 1),)), (0, 0, ((4, 0, 1), (5, 100, -1))),
            (0, 1, ((4, 0, 1), (5, 100, -1), (6, 100, 1))), (0, 0, ((5, 0, 1),)), (2, 0, ((4, 0, 1),)),
            (3, 0, ((3, 0, 1),))]
    split = [False, False, False, True, False, False, False]
    src = FJ.agg_source(sh, terms, False, keys, 6, aggs, split, 64)
    assert "WG_ADD" in src and "WG_MIN" in src and "WG_MAX" in src
    _compile(src, "igloo_jit_scan_agg")


def test_or_groups_and_checked_overflow():
    sh = cols(8, 8, 4)
    terms = [(2, 2 | 1 << 8, 0, 0, 0b110), (0, 0 | 1 << 8, 1, 11, 0), (2, 2 | 2 << 8, 0, 0, 0b1),
             (1, 0 | 2 << 8, 10, 20, 0)]
    aggs = [(0, 1, ((0, 0, 1), (1, 0, 1))), (0, 1, ((0, 0, 1), (1, 0, 1), (2, 3, 2)))]
    src = FJ.agg_source(sh, terms, True, [], 1, aggs, [True, True], 64)
    assert "__builtin_mul_overflow" in src and "||" in src
    _compile(src, "igloo_jit_scan_agg")


def test_q1_shape_mfma_compiles():
    sh = cols(2, 1, 1, 2, 4, 1, 1)
    terms = [(0, 0, -(2**63), 10471, 0)]
    keys = [(1, 0, 2), (2, 0, 1)]
    aggs = [(0, 0, ((3, 0, 1),)), (0, 0, ((4, 0, 1),)), (0, 0, ((4, 0, 1), (5, 100, -1))),
            (0, 1, ((4, 0, 1), (5, 100, -1), (6, 100, 1))), (0, 0, ((5, 0, 1),))]
    src, lds = FJ.mfma_agg_source(sh, terms, False, keys, 6, aggs)
    assert "__builtin_amdgcn_mfma_i32_16x16x64_i8" in src and lds <= 160 * 1024
    _compile(src, "igloo_jit_scan_agg_mfma")
