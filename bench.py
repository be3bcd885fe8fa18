"""Headline benchmark: TPC-H SF100 total query time (22 queries) + scan rows/s.

BASELINE.json metric: "TPC-H SF100 total query time (s) + rows/sec scan,
1/2/4/8 MI355X". One step = one run of the full 22-query suite. Data is
synthetic TPC-H-shaped, generated directly in HBM by each rank for its own
hash partition (the HBM cache tier; generation time is reported separately
and is not part of the timed region). Every query in the timed region runs to
completion with its result materialised on the host.

Single GPU:  python bench.py --gpus 1 --steps 3 --warmup 1
N GPUs:      python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                 --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "TPC-H SF100 total query time (s) + rows/sec scan, 1/2/4/8 MI355X"


def parse_queries(s: str):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--sf", type=float, default=100.0)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--lean", action="store_true", help="skip comment columns no query reads")
    ap.add_argument("--per-query", action="store_true", help="print per-query times to stderr")
    ap.add_argument("--cpu", action="store_true", help="run on CPU (debug)")
    a = ap.parse_args()

    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # IGLOO_BENCH_SHARE_GPU=1: every rank on cuda:0 with host-staged gloo
    # collectives — a rehearsal of the multi-rank path on a one-GPU box
    shared = os.environ.get("IGLOO_BENCH_SHARE_GPU") == "1"
    device = "cpu" if a.cpu else ("cuda:0" if shared else f"cuda:{local}")
    if not a.cpu:
        torch.cuda.set_device(torch.device(device))
    comm = None
    if world > 1:
        from igloo_amd.parallel.comm import Communicator
        comm = Communicator.init(backend="gloo" if (a.cpu or shared) else "nccl", device=device)

    def barrier():
        if comm is not None:
            comm.barrier()
        if not a.cpu:
            torch.cuda.synchronize()

    qs = parse_queries(a.queries)
    eng = ig.QueryEngine(device=device, comm=comm)
    t0 = time.perf_counter()
    tabs = datagen.generate(a.sf, device, rank, world, lean=a.lean)
    for name, t in tabs.items():
        eng.register_table(name, t)
    barrier()
    gen_s = time.perf_counter() - t0
    local_rows = {k: v.num_rows() for k, v in tabs.items()}
    rows = dict(local_rows)
    if comm is not None:
        for k in rows:
            rows[k] = local_rows[k] if tabs[k].replicated else comm.allreduce_int(local_rows[k])
    scanned = sum(rows[t] for q in qs for t in queries.SCANNED[q])
    if rank == 0:
        print(f"[bench] sf={a.sf} world={world} gen={gen_s:.1f}s rows={rows}", file=sys.stderr, flush=True)

    def suite(record=None):
        for q in qs:
            tq = time.perf_counter()
            eng.sql(queries.QUERIES[q])
            if record is not None:
                barrier()
                record[q] = record.get(q, 0.0) + (time.perf_counter() - tq)

    for w in range(a.warmup):
        tw = time.perf_counter()
        suite()
        barrier()
        if rank == 0:
            print(f"[bench] warmup {w}: {time.perf_counter() - tw:.3f}s", file=sys.stderr, flush=True)
    per_q = {} if a.per_query else None
    barrier()
    if os.environ.get("IGLOO_PROF_GAP"):
        time.sleep(1.0)   # idle gap that scripts/kernel_summary.py uses to isolate the timed steps in a trace
    t1 = time.perf_counter()
    for s in range(a.steps):
        suite(per_q)
        if rank == 0:
            print(f"[bench] step {s}: {time.perf_counter() - t1:.3f}s cumulative", file=sys.stderr, flush=True)
    barrier()
    elapsed = time.perf_counter() - t1
    if comm is not None:
        elapsed = comm.allreduce_max_float(elapsed)
    step_s = elapsed / max(a.steps, 1)
    if rank == 0:
        if per_q:
            for q in qs:
                print(f"[bench] Q{q:02d} {per_q[q] / a.steps * 1e3:9.2f} ms", file=sys.stderr)
        out = {
            "metric": METRIC,
            "value": round(step_s, 4),
            "unit": "s (22-query suite, lower is better)",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(step_s * 1e3, 2),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "exact decimal(15,2) int64 fixed-point / int32 keys",
            "data": "synthetic TPC-H-shaped (spec distributions), generated in HBM; cold-from-Parquet time not included",
            "config": {"model": f"TPC-H SF{a.sf:g} queries {a.queries}", "global_batch": sum(rows.values()),
                       "seq_len": None, "parallelism": f"dp{world}" if world > 1 else "single-gpu",
                       "sf": a.sf, "queries": qs},
            "scan_rows_per_s": round(scanned / step_s, 1),
            "datagen_s": round(gen_s, 2),
        }
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.shutdown()


if __name__ == "__main__":
    main()
