"""Which call sites gather how many bytes, per TPC-H query (warm, graphs off).

Wraps ops/gather.py (take_many, gather_tensor, the plain-string gather) and
attributes every gather to its three innermost igloo_amd frames, with rows and
bytes written; the summary lists per query the sites by bytes. With
``--timed`` every fixed-width gather is also bracketed by HIP events and
classified by index pattern (ascending or not) and source size (fits the 4 MB
L2, the 256 MB MALL, or neither): kernel milliseconds per class.

usage: python scripts/gather_sites.py [--sf 10] [--queries 9,10] [--timed] [--out gpurun_out/gather_sites.txt]
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["IGLOO_GRAPHS"] = "0"


def site():
    st = [f for f in traceback.extract_stack()[:-2] if "igloo_amd" in f.filename and "ops/gather.py" not in f.filename]
    return " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}({f.name})" for f in st[-3:][::-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10.0)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--out", default="gpurun_out/gather_sites.txt")
    ap.add_argument("--device", default="cuda:0")
    ap.add_argument("--timed", action="store_true")
    a = ap.parse_args()
    import torch
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, queries
    from igloo_amd.ops import gather as G
    from bench import parse_queries

    qs = parse_queries(a.queries)
    e = ig.QueryEngine(device=a.device)
    sync = torch.cuda.synchronize if a.device.startswith("cuda") else (lambda: None)
    datagen.register(e, a.sf)
    for q in qs:
        e.sql(queries.QUERIES[q])
    sync()

    rec = collections.defaultdict(lambda: [0, 0, 0])     # site -> [calls, rows, bytes]
    o_many, o_tensor, o_str = G.take_many, G.gather_tensor, G._take_plain_strings
    events = []        # (start, end, class, rows, bytes, site)

    def klass(srcs, idx):
        n = idx.numel()
        asc = n < 2 or bool((idx[1:] >= idx[:-1]).all().item())
        sb = max((t.numel() * t.element_size() for t in srcs), default=0)
        size = "L2" if sb <= 4 << 20 else "MALL" if sb <= 256 << 20 else "HBM"
        rows = max((t.shape[0] for t in srcs), default=1)
        dens = n / max(rows, 1)
        return f"{'ascending' if asc else 'random':9s} src {size:4s} density {'>=0.1' if dens >= 0.1 else '<0.1':5s}"

    def timed(fn, srcs, idx, kind):
        if not a.timed or not idx.is_cuda or idx.numel() == 0:
            return fn(), None
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        out = fn()
        ev1.record()
        return out, (ev0, ev1, klass(srcs, idx))

    def take_many(cols, idx, neg=False):
        out, ev = timed(lambda: o_many(cols, idx, neg), [c.data for c in cols if not c.is_plain_string], idx, "m")
        key = ("take_many", site())
        r = rec[key]
        r[0] += 1
        r[1] += idx.numel()
        b = sum(c.data.numel() * c.data.element_size() for c in out if not c.is_plain_string)
        r[2] += b
        if ev:
            events.append(ev + (idx.numel(), b, key))
        return out

    def gather_tensor(t, idx):
        out, ev = timed(lambda: o_tensor(t, idx), [t], idx, "t")
        key = ("gather_tensor", site())
        r = rec[key]
        r[0] += 1
        r[1] += idx.numel()
        r[2] += out.numel() * out.element_size()
        if ev:
            events.append(ev + (idx.numel(), out.numel() * out.element_size(), key))
        return out

    def take_str(col, idx, neg):
        out = o_str(col, idx, neg)
        r = rec[("strings", site())]
        r[0] += 1
        r[1] += idx.numel()
        r[2] += out.data.numel() + out.offsets.numel() * 8
        return out

    G.take_many, G.gather_tensor, G._take_plain_strings = take_many, gather_tensor, take_str
    # modules that imported the names directly
    import igloo_amd.exec.aggregate as AG
    import igloo_amd.exec.joins as JN
    import igloo_amd.exec.scan as SC
    import igloo_amd.exec.sorting as SR
    import igloo_amd.ops.strings as ST
    import igloo_amd.parallel.exchange as EX
    for mod in (SC, JN, AG, SR, ST, EX):
        for name, fn in (("take_many", take_many), ("gather_tensor", gather_tensor)):
            if hasattr(mod, name):
                setattr(mod, name, fn)
    lines = []
    by_class = collections.defaultdict(lambda: [0, 0.0, 0, 0])    # class -> calls, ms, rows, bytes
    for q in qs:
        rec.clear()
        del events[:]
        e.sql(queries.QUERIES[q])
        sync()
        qms = 0.0
        site_ms = collections.Counter()
        for ev0, ev1, k, rows, b, key in events:
            ms = ev0.elapsed_time(ev1)
            qms += ms
            site_ms[key] += ms
            c = by_class[k]
            c[0] += 1
            c[1] += ms
            c[2] += rows
            c[3] += b
        tot = sum(v[2] for v in rec.values())
        lines.append(f"== Q{q}: {tot / 1e9:.3f} GB gathered" + (f", {qms:.3f} ms in gather launches" if a.timed else ""))
        for (kind, s), (c, rows, b) in sorted(rec.items(), key=lambda kv: -kv[1][2])[:8]:
            ms = f"{site_ms[(kind, s)]:7.3f} ms " if a.timed else ""
            lines.append(f"  {ms}{b / 1e9:8.3f} GB {rows / 1e6:9.2f} Mrows {c:4d} calls  {kind:13s} {s}")
    if a.timed:
        lines.append("\n== by index pattern / source size (fixed-width gathers, event-timed)")
        for k, (c, ms, rows, b) in sorted(by_class.items(), key=lambda kv: -kv[1][1]):
            lines.append(f"  {k}  {c:4d} calls {ms:8.3f} ms {rows / 1e6:9.1f} Mrows {b / 1e9:7.3f} GB written "
                         f"{b / max(ms, 1e-9) / 1e6:7.0f} GB/s")
    txt = "\n".join(lines)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
