"""Micro-benchmark of the GPU Parquet decode path (snappy + page decode):
writes TPC-H lineitem (SF given) as one snappy Parquet file and decodes every
column on the GPU a few times. Run under rocprofv3 --kernel-trace --stats for
per-kernel times.

usage: python scripts/snappy_bench.py [--sf 1] [--reps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from igloo_amd import types as T  # noqa: E402
from igloo_amd.connectors.gpu_parquet import GpuParquetReader  # noqa: E402
from igloo_amd.models.tpch import parquet_gen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/igloo_snappy_bench")
    a = ap.parse_args()
    man = parquet_gen.write_dataset(a.sf, a.dir, device="cuda:0", rows_per_file=1 << 40)
    path = os.path.join(parquet_gen.dataset_dir(a.dir, a.sf), "lineitem", "part-00000.parquet")
    import pyarrow.parquet as pq
    sch = pq.read_schema(path)
    cols = [(f.name, T.from_arrow_type(f.type)) for f in sch]
    r = GpuParquetReader([path])
    groups = [(0, g) for g in range(len(r.metas[0].row_groups))]
    size = os.path.getsize(path)
    for i in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out, rej = r.read(cols, groups, "cuda:0")
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {i}: {dt:.3f}s  {size / dt / 1e9:.2f} GB/s file  stats={r.last_stats} rejected={rej}", flush=True)
        del out


if __name__ == "__main__":
    main()
