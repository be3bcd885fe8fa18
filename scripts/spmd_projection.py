"""Projected 8-GPU time per TPC-H query from a world-of-one SPMD run.

Every operator of every query runs under EXPLAIN ANALYZE on the SPMD path
(a world of one: every exchange and collective really runs, RCCL). Each
operator's exclusive time is charged by the placement of its output:

* replicated output (work every rank repeats): counted in full at 8 GPUs;
* partitioned output: divided by 8 (each rank holds 1/8 of the rows);

plus the collectives: per call a latency of ``--lat-us`` (8-rank RCCL small
collective) and the bytes each rank sends at ``--gbps`` of aggregate xGMI
egress (an all-to-all uses all 7 links). EXPLAIN ANALYZE synchronises around
every operator, so its totals exceed the graph-replay times; the projection is
also reported scaled by the measured graph-mode time of the query
(``--graph-ms`` file from bench.py --per-query, optional).

    python scripts/spmd_projection.py --sf 100 --json gpurun_out/projection.json
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def walk(n):
    yield n
    for c in n.children:
        yield from walk(c)


def _graph_ms(path):
    out = {}
    if path and os.path.exists(path):
        for line in open(path):
            m = re.match(r"\[bench\] Q(\d+)\s+([\d.]+) ms", line)
            if m:
                out[int(m.group(1))] = float(m.group(2))
    return out


def rescore(a):
    """Graph-scaled projection from a saved run (the EXPLAIN ANALYZE split into
    replicated / partitioned work and collectives) and a bench.py log."""
    d = json.load(open(a.rescore))
    g = _graph_ms(a.graph_log)
    tot = {"g1": 0.0, "t8_scaled": 0.0}
    for r in d["queries"]:
        g1 = g.get(r["q"])
        r["graph_world1_ms"] = g1
        r["t8_scaled_to_graph_ms"] = round(r["t8_ms"] * g1 / r["t1_analyze_ms"], 3) if g1 else None
        if g1:
            tot["g1"] += g1
            tot["t8_scaled"] += r["t8_scaled_to_graph_ms"]
        print(f"Q{r['q']:02d}  world-1 graph {g1 or 0:7.2f} ms  replicated share "
              f"{r['replicated_ms'] / max(r['t1_analyze_ms'], 1e-9):5.1%}  collectives {r['collectives']:2d}  "
              f"-> T8 {r['t8_scaled_to_graph_ms'] or 0:6.2f} ms")
    print(f"suite: world-1 graph {tot['g1']:.2f} ms -> projected {d['world']} GPUs {tot['t8_scaled']:.2f} ms "
          f"({tot['g1'] / max(tot['t8_scaled'], 1e-9):.2f}x)")
    d["suite_graph_world1_ms"] = round(tot["g1"], 3)
    d["suite_t8_scaled_ms"] = round(tot["t8_scaled"], 3)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(d, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--lat-us", type=float, default=30.0)
    ap.add_argument("--gbps", type=float, default=500.0, help="per-rank aggregate xGMI egress used by exchanges")
    ap.add_argument("--graph-log", default=None, help="bench.py --per-query log of the SPMD world-1 graph run")
    ap.add_argument("--json", default=None)
    ap.add_argument("--rescore", default=None, help="a --json output: recompute the graph-scaled column only")
    a = ap.parse_args()
    if a.rescore:
        return rescore(a)
    os.environ.update(RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29800 + os.getpid() % 100))
    import torch
    import igloo_amd as ig
    from igloo_amd.exec.planner import create_physical_plan
    from igloo_amd.models.tpch import datagen, queries as Q
    from igloo_amd.parallel.comm import Communicator
    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    comm = Communicator.init(backend="nccl" if dev != "cpu" else "gloo", device=dev, force_spmd=True)
    e = ig.QueryEngine(device=dev, comm=comm)
    for n, t in datagen.generate(a.sf, dev, 0, 1, spmd=True).items():
        e.register_table(n, t)
    graph_ms = {}
    if a.graph_log and os.path.exists(a.graph_log):
        for line in open(a.graph_log):
            m = re.match(r"\[bench\] Q(\d+)\s+([\d.]+) ms", line)
            if m:
                graph_ms[int(m.group(1))] = float(m.group(2))
    W = a.world
    rows, tot = [], {"t1": 0.0, "rep": 0.0, "part": 0.0, "coll": 0.0, "t8": 0.0, "t8_scaled": 0.0, "g1": 0.0}
    for q in qs:
        sql = Q.QUERIES[q]
        for _ in range(2):
            e.sql(sql)                  # derived structures built, kernels compiled
        best = None
        for _ in range(2):
            plan, _names = e.logical_plan(sql)
            node = create_physical_plan(plan)
            ctx = e.make_context(analyze=True)
            ctx.slices = e._slices_for(plan)
            c0 = (comm.calls, comm.bytes_sent)
            node.execute(ctx)
            out = node
            from igloo_amd.parallel.exchange import gather_all
            if dev != "cpu":
                torch.cuda.synchronize()
            calls, nbytes = comm.calls - c0[0], comm.bytes_sent - c0[1]
            rep = part = 0.0

            def inputs_replicated(n) -> bool:
                """The operator's work is repeated on every rank: all its inputs
                are replicated (a leaf: its own output; an input fused into the
                operator and never executed on its own: its source)."""
                if not n.children:
                    m = ctx.metrics.get(id(n))
                    if m is not None and m.get("dist") is not None:
                        return m["dist"] == ("replicated",)
                    src = getattr(getattr(n, "logical", None), "source", None)
                    return bool(getattr(src, "replicated", False)) and id(src) not in ctx.slices
                flags = []
                for c in n.children:
                    m = ctx.metrics.get(id(c))
                    flags.append(m["dist"] == ("replicated",) if m is not None else inputs_replicated(c))
                return all(flags)

            def excl_ms(n) -> float:
                m = ctx.metrics[id(n)]
                kids = 0.0
                stack = list(n.children)
                while stack:          # nearest measured descendants
                    c = stack.pop()
                    if id(c) in ctx.metrics:
                        kids += ctx.metrics[id(c)]["ms"]
                    else:
                        stack.extend(c.children)
                return max(m["ms"] - kids, 0.0)
            for n in walk(node):
                if id(n) not in ctx.metrics:
                    continue
                if inputs_replicated(n):
                    rep += excl_ms(n)
                else:
                    part += excl_ms(n)
            t1 = rep + part
            if best is None or t1 < best[0]:
                best = (t1, rep, part, calls, nbytes)
        t1, rep, part, calls, nbytes = best
        coll = calls * a.lat_us / 1e3 + nbytes * (W - 1) / W / W / (a.gbps * 1e6)
        t8 = rep + part / W + coll
        g1 = graph_ms.get(q)
        scaled = t8 * (g1 / t1) if g1 else None
        rows.append({"q": q, "t1_analyze_ms": round(t1, 3), "replicated_ms": round(rep, 3),
                     "partitioned_ms": round(part, 3), "collectives": calls, "exchange_bytes_world1": nbytes,
                     "collective_ms_8": round(coll, 3), "t8_ms": round(t8, 3),
                     "graph_world1_ms": g1, "t8_scaled_to_graph_ms": round(scaled, 3) if scaled else None})
        for k, v in (("t1", t1), ("rep", rep), ("part", part), ("coll", coll), ("t8", t8)):
            tot[k] += v
        if scaled:
            tot["t8_scaled"] += scaled
            tot["g1"] += g1
        print(f"Q{q:02d}  analyze {t1:8.2f} ms  replicated {rep:7.2f}  partitioned {part:8.2f}  "
              f"collectives {calls:3d} ({nbytes / 1e6:8.1f} MB)  -> T8 {t8:7.2f} ms"
              + (f"  | graph w1 {g1:6.2f} -> T8 {scaled:6.2f} ms" if scaled else ""), flush=True)
    print("suite: " + ", ".join(f"{k} {v:.2f} ms" for k, v in tot.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"sf": a.sf, "world": W, "lat_us": a.lat_us, "gbps": a.gbps, "queries": rows, "suite": tot}, f,
                      indent=1)
    e.close()
    comm.shutdown()


if __name__ == "__main__":
    main()
