"""Sparse ascending gathers (late materialisation after a selective join:
TPC-H Q9 takes 32M of 600M lineitem rows, density 5.4 %): K int32 columns
gathered one by one (gather_multi, one column per descriptor) against one
gather of a row-packed copy (K x 4 bytes per row, 16-byte loads).
   python scripts/bench_gather_packed.py [--rows 600e6] [--density 0.054] [--cols 4]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from igloo_amd.ops._lib import native, ptr  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=600e6)
    ap.add_argument("--density", type=float, default=0.054)
    ap.add_argument("--cols", type=int, default=4)
    a = ap.parse_args()
    N = native()
    n = int(a.rows)
    g = torch.Generator(device="cuda").manual_seed(0)
    cols = [torch.randint(0, 1 << 30, (n,), device="cuda", dtype=torch.int32, generator=g) for _ in range(a.cols)]
    keep = torch.rand(n, device="cuda", generator=g) < a.density
    idx = torch.nonzero(keep).flatten().to(torch.int32)
    m = idx.numel()
    s = torch.cuda.current_stream().cuda_stream
    outs = [torch.empty(m, dtype=torch.int32, device="cuda") for _ in cols]

    def separate():
        N.gather_multi(ptr(idx), False, m, [(ptr(c), ptr(o), 4, 0, 0, n) for c, o in zip(cols, outs)], s)

    w = 4 * a.cols
    wp = 16 if w <= 16 else 32
    packed = torch.zeros(n, wp // 4, dtype=torch.int32, device="cuda")
    for k, c in enumerate(cols):
        packed[:, k] = c
    pout = torch.empty(m, wp // 4, dtype=torch.int32, device="cuda")

    def packed_gather():
        N.gather_multi(ptr(idx), False, m, [(ptr(packed), ptr(pout), 16, 0, 0, n)] if wp == 16 else
                       [(ptr(packed), ptr(pout), 16, 0, 0, n)], s)

    t1 = timed(separate)
    t2 = timed(packed_gather)
    assert torch.equal(pout[:, 0], outs[0]) and torch.equal(pout[:, a.cols - 1], outs[-1])
    print(f"rows={n} density={a.density} gathered={m} cols={a.cols}: separate {t1:.3f} ms, "
          f"packed {wp} B rows {t2:.3f} ms ({t1 / t2:.2f}x)", flush=True)
    del cols, outs, packed, pout

    # the engine's case (ops/packed_gather.py): int64 columns whose values fit
    # int32 / int8 / int16 / int32 (Q9's l_extendedprice, l_discount,
    # l_quantity, l_suppkey), one 16-byte packed row widened back to int64
    from igloo_amd.ops.pack import layout, pack_rows
    lim = [(1 << 30), 100, 20000, (1 << 30)][:a.cols]
    wide = [torch.randint(-v, v, (n,), device="cuda", dtype=torch.int64, generator=g) for v in lim]
    narrowed = [w.to(torch.int32 if v > 30000 else torch.int16 if v > 120 else torch.int8) for w, v in zip(wide, lim)]
    lay = layout(narrowed)
    pk, _ = pack_rows(narrowed, None, n, lay)
    del narrowed
    wouts = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in wide]
    pouts = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in wide]
    fields = [(ptr(pouts[i]), off, w, 8, 1) for i, w, off in lay[1]]

    def wide_separate():
        N.gather_multi(ptr(idx), False, m, [(ptr(c), ptr(o), 8, 0, 0, n) for c, o in zip(wide, wouts)], s)

    def wide_packed():
        N.gather_packed(ptr(idx), False, m, ptr(pk), n, lay[0], fields, s)

    t3 = timed(wide_separate)
    t4 = timed(wide_packed)
    for o, p in zip(wouts, pouts):
        assert torch.equal(o, p)
    print(f"int64 columns x{a.cols}: separate {t3:.3f} ms, gather_packed {lay[0]} B rows {t4:.3f} ms "
          f"({t3 / t4:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
