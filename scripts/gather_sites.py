"""Which call sites gather how many bytes, per TPC-H query (warm, graphs off).

Wraps ops/gather.py (take_many, gather_tensor, the plain-string gather) and
attributes every gather to its three innermost igloo_amd frames, with rows and
bytes written; the summary lists per query the sites by bytes.

usage: python scripts/gather_sites.py [--sf 10] [--queries 9,10] [--out gpurun_out/gather_sites.txt]
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

    def take_many(cols, idx, neg=False):
        out = o_many(cols, idx, neg)
        r = rec[("take_many", site())]
        r[0] += 1
        r[1] += idx.numel()
        r[2] += sum(c.data.numel() * c.data.element_size() for c in out if not c.is_plain_string)
        return out

    def gather_tensor(t, idx):
        out = o_tensor(t, idx)
        r = rec[("gather_tensor", site())]
        r[0] += 1
        r[1] += idx.numel()
        r[2] += out.numel() * out.element_size()
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
    for q in qs:
        rec.clear()
        e.sql(queries.QUERIES[q])
        sync()
        tot = sum(v[2] for v in rec.values())
        lines.append(f"== Q{q}: {tot / 1e9:.3f} GB gathered")
        for (kind, s), (c, rows, b) in sorted(rec.items(), key=lambda kv: -kv[1][2])[:8]:
            lines.append(f"  {b / 1e9:8.3f} GB {rows / 1e6:9.2f} Mrows {c:4d} calls  {kind:13s} {s}")
    txt = "\n".join(lines)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
