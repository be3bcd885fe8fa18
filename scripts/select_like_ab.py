"""A/B timing of the compaction (select.hip tile_write) and segment-LIKE
(strings.hip like_seg) kernels between two builds of the native extension.

    python scripts/select_like_ab.py --so _ab/native_old.so --tag old
    python scripts/select_like_ab.py --tag new        (the in-tree build)

Times mask_to_indices over 600M / 60M-row masks at several selectivities and
LIKE '%special%requests%' over SF10 o_comment (15M strings), CUDA events,
median of 15 runs."""
import argparse
import importlib.util
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default=None)
    ap.add_argument("--tag", default="new")
    a = ap.parse_args()
    import torch
    if a.so:
        spec = importlib.util.spec_from_file_location("igloo_amd._native", a.so)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        sys.modules["igloo_amd._native"] = m
    import igloo_amd as ig
    from igloo_amd.ops import _lib
    from igloo_amd.ops import strings as S
    from igloo_amd.ops.select import mask_to_indices
    if a.so:
        _lib._native = sys.modules["igloo_amd._native"]
    dev = "cuda:0"

    def timed(fn, reps=15):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[len(ts) // 2]
    g = torch.Generator(device=dev).manual_seed(1)
    for n in (600_000_000, 60_000_000):
        u = torch.rand(n, device=dev, generator=g)
        for sel in (0.5, 0.1, 0.01):
            mask = u < sel
            ref = torch.nonzero(mask).flatten().to(torch.int32)
            got = mask_to_indices(mask)
            assert torch.equal(got, ref), "compaction mismatch"
            ms = timed(lambda: mask_to_indices(mask, total=ref.numel()))
            print(f"[{a.tag}] select n={n} sel={sel}: {ms:.3f} ms", flush=True)
        del u
    from igloo_amd.ops.select import exclusive_scan
    for n in (100_000_000, 10_000_000):
        c = torch.randint(0, 4, (n,), device=dev, dtype=torch.int32, generator=g)
        ex, tot = exclusive_scan(c)
        assert tot == int(c.sum()) and int(ex[-1]) == tot - int(c[-1]), "scan mismatch"
        ms = timed(lambda: exclusive_scan(c, host_total=False))
        print(f"[{a.tag}] scan n={n}: {ms:.3f} ms", flush=True)
    torch.cuda.empty_cache()
    from igloo_amd.models.tpch import datagen
    e = ig.QueryEngine(device=dev)
    datagen.register(e, 10)
    col = e.sql_device("SELECT o_comment FROM orders").columns["o_comment"]
    for pat in ("%special%requests%", "%pending%"):
        r = S.like(col, pat)
        ms = timed(lambda: S.like(col, pat))
        print(f"[{a.tag}] like {pat} n={len(col)} hits={int(r.sum())}: {ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
