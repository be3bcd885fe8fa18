"""Independent check of the GPU results at scale: the 22
TPC-H queries at SF10 on the GPU engine (HBM tables, gfx950 kernels) and on
the CPU engine (torch CPU operators: no HIP kernel, no graph, no readback
replay) over the same generated data; every result digest must agree.

    python scripts/oracle_gpu_vs_cpu.py --sf 10 [--json out.json]

The GPU tables are generated on the device and copied to the host for the CPU
engine (GPU and CPU generation are identical: tests/test_tpch_gpu.py
test_gpu_datagen_matches_cpu). Prints one line per query as it goes."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.catalog import MemoryTable
    from igloo_amd.models.tpch import datagen, params
    from igloo_amd.utils.digest import digest
    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    t0 = time.perf_counter()
    g = ig.QueryEngine(device="cuda:0")
    c = ig.QueryEngine(device="cpu")
    tabs = datagen.generate(a.sf, "cuda:0")
    for name, t in tabs.items():
        g.register_table(name, t)
        cols = {k: v.to("cpu") for k, v in t.columns.items()}
        c.register_table(name, MemoryTable(cols, t.num_rows(), fields=list(t.schema())))
    torch.cuda.synchronize()
    print(f"[oracle] sf={a.sf} generated + copied in {time.perf_counter() - t0:.1f}s", flush=True)
    out = {"sf": a.sf, "queries": {}}
    for q in qs:
        sql = params.validation(q, a.sf)
        tg = time.perf_counter()
        rg = g.sql(sql).table
        tg = time.perf_counter() - tg
        tc = time.perf_counter()
        rc = c.sql(sql).table
        tc = time.perf_counter() - tc
        dg, dc = digest(rg), digest(rc)
        ok = dg == dc
        out["queries"][q] = {"rows": rg.num_rows, "match": ok, "gpu_s": round(tg, 3), "cpu_s": round(tc, 2)}
        print(f"[oracle] Q{q:02d} rows={rg.num_rows:>8} gpu {tg:7.3f}s cpu {tc:8.2f}s "
              f"{'MATCH' if ok else 'MISMATCH'}", flush=True)
    n_ok = sum(1 for v in out["queries"].values() if v["match"])
    print(f"[oracle] {n_ok}/{len(qs)} GPU results equal the CPU engine's at SF{a.sf:g}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
