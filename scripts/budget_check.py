"""Run the 22 TPC-H queries on the GPU with the device memory capped (the
caching allocator's per-process fraction) and the engine's device budget set,
and check every result digest against the CPU engine on the same data.

usage: python scripts/budget_check.py [--sf 1] [--cap-gb 1] [--budget-gb 0.25]
Exit status 0 when all match and peak reserved memory stayed under the cap."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--cap-gb", type=float, default=1.0)
    ap.add_argument("--budget-gb", type=float, default=0.25)
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.utils.digest import digest
    from igloo_amd.catalog import MemoryTable
    from igloo_amd.models.tpch import datagen, queries
    cpu = ig.QueryEngine(device="cpu")
    tabs = datagen.generate(a.sf, "cpu")
    for name, t in tabs.items():
        cpu.register_table(name, t)
    want = {q: digest(cpu.sql(queries.QUERIES[q]).table) for q in range(1, 23)}
    cap = int(a.cap_gb * 2**30)
    total = torch.cuda.get_device_properties(0).total_memory
    torch.cuda.set_per_process_memory_fraction(cap / total, 0)
    torch.cuda.reset_peak_memory_stats(0)
    g = ig.QueryEngine(device="cuda:0", cache_hbm_gb=a.budget_gb / 4, cache_host_gb=64,
                       config={"device_budget_gb": a.budget_gb})
    for name, t in tabs.items():
        # host-resident tables: every scan moves a transient copy to the device
        g.register_table(name, MemoryTable(t.columns, t.num_rows(), replicated=t.replicated, resident=False))
    bad, spilled = [], 0
    for q in range(1, 23):
        got = digest(g.sql(queries.QUERIES[q]).table)
        sp = g.last_metrics["spill"]
        spilled += sp["joins"]
        peak = torch.cuda.max_memory_reserved(0)
        print(f"Q{q}: {'ok' if got == want[q] else 'MISMATCH'} spill={sp} peak_reserved={peak / 2**20:.0f} MiB",
              flush=True)
        if got != want[q]:
            bad.append(q)
    peak = torch.cuda.max_memory_reserved(0)
    print(f"peak reserved {peak / 2**20:.0f} MiB (cap {cap / 2**20:.0f} MiB), partitioned joins {spilled}, "
          f"mismatches {bad}", flush=True)
    sys.exit(0 if not bad and peak <= cap and spilled > 0 else 1)


if __name__ == "__main__":
    main()
