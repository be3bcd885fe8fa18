"""Attribute PyTorch ATen GPU kernels of the warm TPC-H suite to the igloo
call sites that launch them (torch.profiler with Python stacks).

usage: python scripts/aten_sites.py --sf 10 [--queries 1-22] [--top 40]"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["IGLOO_GRAPHS"] = "0"     # eager execution: a graph replay issues no ATen op to attribute


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops import jit
    from bench import parse_queries
    qs = parse_queries(a.queries)
    e = ig.QueryEngine(device="cuda:0")
    datagen.register(e, a.sf)
    for _ in range(2):
        for q in qs:
            e.sql(queries.QUERIES[q])
        jit.wait_all(120)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for q in qs:
            e.sql(queries.QUERIES[q])
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0.0, 0])
    for ev in prof.events():
        dev_us = getattr(ev, "device_time_total", 0) or getattr(ev, "cuda_time_total", 0)
        if not dev_us or not ev.name.startswith("aten::"):
            continue
        if any(ch.name.startswith("aten::") for ch in ev.cpu_children):
            continue     # count the innermost aten op only
        site = "?"
        frames = [fr for fr in (ev.stack or []) if "igloo_amd" in fr and "ops/_lib.py" not in fr]
        if frames:
            site = " <- ".join(fr.split("igloo_amd/")[-1] for fr in frames[:2])
        k = (ev.name, site)
        agg[k][0] += dev_us / 1e3
        agg[k][1] += 1
    tot = sum(v[0] for v in agg.values())
    print(f"aten device time {tot:.2f} ms over the suite")
    for (name, site), (ms, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{ms:8.3f} ms {n:5d}  {name:28s} {site}")


if __name__ == "__main__":
    main()
