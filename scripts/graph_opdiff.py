"""Debug a query graph without replaying it: log every ATen op (name, output
shapes, igloo call site) of one eager replay and of the capture of the same
query, dump the captured graph (DOT), and print where the two op sequences
first differ. Nothing captured is ever launched."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import igloo_amd as ig  # noqa: E402
from igloo_amd.exec import graphs  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402
from igloo_amd.ops import jit  # noqa: E402


def site():
    fr = [f for f in traceback.extract_stack() if "igloo_amd" in f.filename]
    return " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}" for f in fr[-3:][::-1])


class OpLog(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        outs = out if isinstance(out, (tuple, list)) else [out]
        shapes = [tuple(o.shape) for o in outs if isinstance(o, torch.Tensor)]
        self.ops.append((str(func), shapes, site()))
        return out


q = int(os.environ.get("Q", "16"))
sf = float(os.environ.get("SF", "0.01"))
e = ig.QueryEngine(device="cuda:0")
datagen.register(e, sf)
sql = queries.QUERIES[q]
for i in range(4):
    if i == 1:
        jit.wait_all(timeout=120)
    e.sql(sql)
    print(f"run {i}: {e.last_metrics['speculation']}", flush=True)
st = next(v for v in e._spec.values() if v.get("log") is not None)
eager = OpLog()
with eager:
    e.sql(sql)
print("eager run:", e.last_metrics["speculation"], len(eager.ops), "ops", flush=True)
st = next(v for v in e._spec.values() if v.get("log") is not None)
cap = OpLog()
orig_execute = e._execute_plan


def logged(plan, ctx=None):
    with cap:
        return orig_execute(plan, ctx)


e._execute_plan = logged
os.environ["IGLOO_GRAPH_DUMP"] = "gpurun_out/graph_dump"
plan = next(p for k, (p, _n) in e._plans.items() if k[0] == sql)
g = graphs.capture(e, plan, st["log"], e.make_context)
print("captured:", g is not None, graphs.STATS, graphs.LAST_ERROR[-1:] if graphs.LAST_ERROR else "", flush=True)
print("capture ops:", len(cap.ops), flush=True)
n = min(len(eager.ops), len(cap.ops))
first = next((i for i in range(n) if eager.ops[i][:2] != cap.ops[i][:2]), None)
print("first difference at op", first, flush=True)
lo = max(0, (first or n) - 5)
for i in range(lo, min(n, (first or n) + 15)):
    print(f"{i:5d} E {eager.ops[i][0]:<40} {str(eager.ops[i][1]):<28} {eager.ops[i][2]}")
    print(f"{i:5d} C {cap.ops[i][0]:<40} {str(cap.ops[i][1]):<28} {cap.ops[i][2]}")
big = [(i, o) for i, o in enumerate(cap.ops) if any(s and s[0] > 100_000 for s in o[1])]
print("capture ops with >100k rows:", big[:20], flush=True)
# the captured graph is dropped without being launched
del g
