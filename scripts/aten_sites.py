"""Which call sites launch ATen kernels (fills, casts / copies, where, cat,
...) and for how long, per TPC-H query (warm, graphs off).

Every ATen op dispatched while the suite runs passes through a
TorchDispatchMode that brackets it with HIP events and attributes it to its
three innermost igloo_amd frames (torch.profiler's Python stacks come back
empty on this image, so the profiler cannot name the sites); ops that launch
nothing (empty, views, metadata, scalar reads) are skipped. Our own kernels go
through the extension, not the dispatcher, and are not seen here
(scripts/kernel_summary.py covers them). Times include the launch.

usage: python scripts/aten_sites.py [--sf 10] [--queries 1-22] [--top 45]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["IGLOO_GRAPHS"] = "0"     # eager execution: a graph replay issues no ATen op to attribute

_SKIP = ("empty", "view", "alias", "as_strided", "detach", "_local_scalar_dense", "resize_", "set_",
         "lift_fresh", "unsqueeze", "squeeze", "expand", "t.", "transpose", "permute", "select.", "slice.",
         "_unsafe_view", "reshape", "unbind", "split")


def site():
    st = [f for f in traceback.extract_stack()[:-3]
          if "igloo_amd" in f.filename and "ops/_lib.py" not in f.filename]
    return " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}({f.name})" for f in st[-3:][::-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode
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

    events = []          # (ev0, ev1, op, site, query)

    class Mode(TorchDispatchMode):
        q = 0

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = f"{func.overloadpacket.__name__}.{func._overloadname}"
            if name.startswith(_SKIP):
                return func(*args, **(kwargs or {}))
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            out = func(*args, **(kwargs or {}))
            ev1.record()
            events.append((ev0, ev1, name, site(), self.q))
            return out

    mode = Mode()
    with mode:
        for q in qs:
            mode.q = q
            e.sql(queries.QUERIES[q])
    torch.cuda.synchronize()
    by_site = collections.defaultdict(lambda: [0, 0.0, set()])    # (op, site) -> calls, ms, queries
    by_op = collections.defaultdict(lambda: [0, 0.0])
    total = 0.0
    for ev0, ev1, name, s, q in events:
        ms = ev0.elapsed_time(ev1)
        total += ms
        r = by_site[(name, s)]
        r[0] += 1
        r[1] += ms
        r[2].add(q)
        o = by_op[name]
        o[0] += 1
        o[1] += ms
    lines = [f"ATen ops over the suite (eager, event-timed incl. launch): {len(events)} calls, {total:.3f} ms",
             "", "== by op"]
    for name, (c, ms) in sorted(by_op.items(), key=lambda kv: -kv[1][1])[:20]:
        lines.append(f"  {ms:8.3f} ms {c:5d} calls  {name}")
    lines += ["", "== by site"]
    for (name, s), (c, ms, qq) in sorted(by_site.items(), key=lambda kv: -kv[1][1])[:a.top]:
        ql = ",".join(str(x) for x in sorted(qq))
        lines.append(f"  {ms:8.3f} ms {c:5d} calls  {name:24s} Q[{ql}]  {s}")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
