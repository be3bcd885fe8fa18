"""Time the fused sorted GROUP BY + HAVING kernels on a Q18-shaped input
(SF100 lineitem: 600M sorted int32 l_orderkey, runs of 1..7 rows, int32
quantities; HAVING sum(q) > 300 with COUNT(*) alongside): the streaming
kernel against the general one (IGLOO_DEBUG=having_general), in GB/s of keys +
values read.   python scripts/bench_having.py [--rows 600000000]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from igloo_amd.ops import agg as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=600_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(1)
    runs = torch.randint(1, 8, (a.rows // 4,), device="cuda", generator=g)
    keys = torch.repeat_interleave(torch.arange(runs.numel(), device="cuda", dtype=torch.int32), runs)[:a.rows]
    keys = keys.contiguous()
    n = keys.numel()
    vals = torch.randint(100, 5001, (n,), device="cuda", dtype=torch.int32, generator=g)
    del runs
    specs = [("count", None, None), ("sum_int", vals, None)]
    gb = n * 8 / 1e9
    for env in ("1", "0"):
        # the C++ side reads IGLOO_DEBUG per call: having_general = the run-folding kernel
        os.environ["IGLOO_DEBUG"] = "" if env == "1" else "having_general"
        got = A.sorted_having(keys, specs, 1, ">", 30000)
        m = got[0].numel() if got is not None else -1
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            A.sorted_having(keys, specs, 1, ">", 30000)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / a.reps
        print(f"streaming={env}: rows={n} passing={m} {ms:.3f} ms/call (host sync included) "
              f"{gb / ms * 1e3:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
