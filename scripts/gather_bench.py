"""Gather kernel patterns on one MI355X: the index shapes the engine's late
materialisation produces, timed with HIP events, as effective bandwidth
(useful bytes: index + gathered values read, values written).

    python scripts/gather_bench.py [--src-rows 600000000] [--out gpurun_out/gather_bench.txt]

Cases: sorted indices (filter compaction) at several densities, random
indices into sources smaller / larger than the 256 MB MALL, 1 and 4 columns
per launch; each also with ``variant`` kernels when the native module has
them (``gather_multi`` vs ``gather_sorted_src``)."""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src-rows", type=int, default=600_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/gather_bench.txt")
    ap.add_argument("--so", default=None, help="load this build of the native extension instead (A/B)")
    a = ap.parse_args()
    import torch
    if a.so:
        import importlib.util
        spec = importlib.util.spec_from_file_location("igloo_amd._native", a.so)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        sys.modules["igloo_amd._native"] = m
        from igloo_amd.ops import _lib
        _lib._native = m
    from igloo_amd.columnar import Column
    from igloo_amd import types as T
    from igloo_amd.ops.gather import take_many
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    lines = []

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e))
        return best

    def case(name, src_rows, idx, ncols):
        cols = [Column(T.INT32, torch.randint(0, 1 << 30, (src_rows,), dtype=torch.int32, device=dev, generator=g))
                for _ in range(ncols)]
        ms = timed(lambda: take_many(cols, idx))
        n = idx.numel()
        useful = n * idx.element_size() + ncols * n * 4 * 2
        lines.append(f"{name:46s} n={n/1e6:7.1f}M src={src_rows/1e6:6.0f}M cols={ncols}  {ms:7.3f} ms  "
                     f"{useful / ms / 1e6:7.0f} GB/s useful  {ms / ncols:6.3f} ms/col")
        print(lines[-1], flush=True)
        del cols

    S = a.src_rows
    for dens in (0.5, 0.1, 0.01):
        mask = torch.rand(S, device=dev, generator=g) < dens
        idx = mask.nonzero().squeeze(1).to(torch.int32)
        del mask
        for nc in (1, 4):
            case(f"sorted (filter) density {dens}", S, idx, nc)
        del idx
        torch.cuda.empty_cache()
    for src, n in ((15_000_000, 60_000_000), (150_000_000, 60_000_000), (S, 60_000_000), (S, 300_000_000)):
        idx = torch.randint(0, src, (n,), dtype=torch.int32, device=dev, generator=g)
        for nc in (1, 4):
            case("random", src, idx, nc)
        # clustered: sorted runs of 8 consecutive rows at random starts (join output of a sorted probe)
        idx2 = (torch.randint(0, src - 8, (n // 8, 1), dtype=torch.int32, device=dev, generator=g)
                + torch.arange(8, dtype=torch.int32, device=dev)).reshape(-1)
        case("random runs of 8", src, idx2, 1)
        sidx = torch.sort(idx).values
        case("random, sorted", src, sidx, 1)
        del idx, idx2, sidx
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
