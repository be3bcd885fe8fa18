"""Which eager-COUNT path TPC-H Q13 takes on the GPU (diagnostic).

    python scripts/eager_count_probe.py --sf 10"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--parquet", default=None, help="write + register the Parquet dataset here (the bench's source)")
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.exec import aggregate as AG
    from igloo_amd.models.tpch import datagen, queries
    seen = []
    real_masked, real_full = AG.HashAggExec._eager_count_masked, AG._full_key_hist

    def masked(self, lg, lb, lkey, rkey, ctx):
        out = real_masked(self, lg, lb, lkey, rkey, ctx)
        seen.append(("masked", out is not None))
        return out

    def full(rcol, kmin, span):
        h = real_full(rcol, kmin, span)
        seen.append(("full_hist", h is not None, rcol.valid is not None,
                     bool(getattr(rcol.data, "_igloo_resident", False)), str(rcol.data.dtype)))
        return h
    AG.HashAggExec._eager_count_masked = masked
    AG._full_key_hist = full
    e = ig.QueryEngine(device="cuda:0")
    if a.parquet:
        from igloo_amd.models.tpch import parquet_gen
        parquet_gen.write_dataset(a.sf, a.parquet, device="cuda:0", rank=0, world=1)
        torch.cuda.empty_cache()
        parquet_gen.register_dataset(e, a.parquet, a.sf, 0, 1)
    else:
        datagen.register(e, a.sf)
    q = queries.QUERIES[13]
    for i in range(3):
        seen.clear()
        torch.cuda.synchronize()
        t = time.perf_counter()
        e.sql(q)
        torch.cuda.synchronize()
        print(f"run {i}: {(time.perf_counter() - t) * 1e3:.2f} ms spec={e.last_metrics.get('speculation')} {seen}",
              flush=True)
    nodes = [ln for ln in e.sql("EXPLAIN ANALYZE " + q).table.column("plan").to_pylist()[0].splitlines()]
    print("\n".join(nodes[:40]))


if __name__ == "__main__":
    main()
