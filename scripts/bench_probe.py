"""Probe kernels (csrc/kernels/hashtable.hip probe_hits + probe_write, via
ops/hashing.py JoinTable.probe_select) at the shape of TPC-H Q21's biggest
probe: 600M lineitem supplier keys, half of them masked out (the in-place
probe under the filter mask), against the 40K suppliers of one nation (a
direct table with an exact bitmap). Times each workgroup cap of the two
launches (median of --reps).

    python scripts/bench_probe.py [--rows 600000000] [--caps 0,8192,4096,2048,1024]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=600_000_000)
    ap.add_argument("--build", type=int, default=40_000)
    ap.add_argument("--span", type=int, default=1_000_000)
    ap.add_argument("--caps", default="0,16384,8192,4096,2048,1024")
    ap.add_argument("--bits", default="2,1,0",
                    help="2: LDS-folded bitmap probe, 1: vector bitmap probe, 0: scalar probe (hashtable.hip)")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import numpy as np
    import torch
    from igloo_amd.ops import hashing as H
    from igloo_amd.ops._lib import native
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(3)
    probe = torch.randint(1, a.span + 1, (a.rows,), dtype=torch.int32, device=dev, generator=g)
    valid = torch.rand(a.rows, device=dev, generator=g) < 0.5
    build = torch.from_numpy(np.random.default_rng(1).choice(np.arange(1, a.span + 1), a.build,
                                                             replace=False).astype(np.int32)).to(dev)
    table = H.JoinTable(build, None, defer_unique=False)
    ref = None
    out = {}
    for cap, bits in [(int(c), int(b)) for b in a.bits.split(",") for c in a.caps.split(",")]:
        native().set_probe_grid_cap(cap)
        native().set_probe_bits(bits)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            pidx, bidx = table.probe_select(probe, valid)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        if ref is None:
            ref = (pidx.clone(), bidx.clone())
        same = torch.equal(pidx, ref[0]) and torch.equal(bidx, ref[1])
        k = f"cap={cap or 65536} bits={bits}"
        out[k] = {"ms": round(float(np.median(ts)), 3), "hits": int(pidx.numel()), "same": bool(same)}
        print(k, out[k], flush=True)
    native().set_probe_grid_cap(0)
    native().set_probe_bits(2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
