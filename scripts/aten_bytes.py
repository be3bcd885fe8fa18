"""ATen ops issued by the engine on the GPU, attributed to igloo call sites by
a TorchDispatchMode (every aten op passes through it with its Python stack):
per (op, innermost two engine frames) the call count and the bytes of the
tensors it writes -- the ATen work left on the hot path, ranked.

    python scripts/aten_bytes.py --sf 10 [--queries 1-22] [--top 40]

Queries run eagerly (IGLOO_GRAPHS=0) after a warm-up, so every op is issued."""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["IGLOO_GRAPHS"] = "0"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=10)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--top", type=int, default=40)
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
    rec = collections.defaultdict(lambda: [0, 0])
    skip = {"aten::empty", "aten::empty_strided", "aten::view", "aten::_unsafe_view", "aten::as_strided",
            "aten::slice", "aten::select", "aten::reshape", "aten::t", "aten::transpose", "aten::expand",
            "aten::alias", "aten::detach", "aten::unsqueeze", "aten::squeeze", "aten::permute", "aten::split",
            "aten::_local_scalar_dense", "aten::set_", "aten::record_stream"}

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = "aten::" + func.__name__.split(".")[0]
            if name in skip:
                return out
            outs = out if isinstance(out, (tuple, list)) else [out]
            nbytes = sum(t.numel() * t.element_size() for t in outs if isinstance(t, torch.Tensor) and t.is_cuda)
            if not nbytes:
                return out
            fr = [f for f in traceback.extract_stack()[:-1] if "igloo_amd" in f.filename and "_lib.py" not in f.filename]
            site = " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}" for f in fr[-2:][::-1]) or "?"
            r = rec[(name, site)]
            r[0] += 1
            r[1] += nbytes
            return out
    with Mode():
        for q in qs:
            e.sql(queries.QUERIES[q])
    torch.cuda.synchronize()
    tot = sum(v[1] for v in rec.values())
    print(f"ATen ops writing {tot / 1e9:.3f} GB over the suite ({sum(v[0] for v in rec.values())} calls)")
    for (name, site), (n, b) in sorted(rec.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{b / 1e6:10.1f} MB {n:5d}  {name:26s} {site}")


if __name__ == "__main__":
    main()
