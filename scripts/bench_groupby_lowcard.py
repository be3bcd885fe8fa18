"""GROUP BY build on few distinct 64-bit hashed keys (Q22's country codes):
group_ids over n rows with g distinct values, per-kernel time.
   python scripts/bench_groupby_lowcard.py [--n 636906] [--g 7]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

from igloo_amd.ops import hashing as H  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=636906)
    ap.add_argument("--g", type=int, default=7)
    a = ap.parse_args()
    gen = torch.Generator(device="cuda").manual_seed(0)
    vals = torch.randint(-2**62, 2**62, (a.g,), device="cuda", generator=gen)
    keys = vals[torch.randint(0, a.g, (a.n,), device="cuda", generator=gen)]
    keys._igloo_hashed = True
    H.group_ids(keys)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        gid, g, rep = H.group_ids(keys)
    torch.cuda.synchronize()
    print(f"n={a.n} g={a.g}: group_ids {(time.perf_counter() - t) / 10 * 1e3:.3f} ms, groups {g}", flush=True)


if __name__ == "__main__":
    main()
