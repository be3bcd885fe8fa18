"""Host-sync latency on the GPU box: ``tensor.item()`` vs an async copy into
pinned memory polled by the host (what a data-dependent size costs).

usage: python scripts/sync_bench.py
"""
import time

import numpy as np
import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    s = torch.zeros(1, dtype=torch.int64, device=dev)
    pinned = torch.empty(1, dtype=torch.int64, pin_memory=True)
    view = pinned.numpy()
    for _ in range(50):
        x.add_(1)
        s.copy_(x[:1])
        s.item()
    torch.cuda.synchronize()
    n = 500
    t0 = time.perf_counter()
    for i in range(n):
        x.add_(1)
        torch.sum(x[:1024], 0, keepdim=True, out=s)
        s.item()
    ta = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for i in range(n):
        x.add_(1)
        torch.sum(x[:1024], 0, keepdim=True, out=s)
        view[0] = -1
        pinned.copy_(s, non_blocking=True)
        while view[0] == -1:
            pass
    tb = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for i in range(n):
        x.add_(1)
        torch.sum(x[:1024], 0, keepdim=True, out=s)
    torch.cuda.synchronize()
    tc = (time.perf_counter() - t0) / n
    print(f"item(): {ta * 1e6:.1f} us/iter   pinned copy + poll: {tb * 1e6:.1f} us/iter   "
          f"no sync (launch only): {tc * 1e6:.1f} us/iter")


if __name__ == "__main__":
    main()
