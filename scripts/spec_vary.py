"""Find speculation sites whose values vary between executions: run a query
many times with real readbacks recorded (IGLOO_GRAPHS=0) and print every call
site whose recorded values differ between runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import igloo_amd as ig  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402
from igloo_amd.ops import _lib  # noqa: E402

import traceback  # noqa: E402

STACKS = []
_orig = _lib.to_host_ints


def _traced(t):
    if getattr(_lib._spec, "cur", None) is not None and t.is_cuda:
        STACKS.append(" <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}({f.name})"
                                  for f in traceback.extract_stack()[-9:-1][::-1] if "igloo_amd" in f.filename))
    return _orig(t)


for _m in list(sys.modules.values()):
    if _m is not None and getattr(_m, "__name__", "").startswith("igloo_amd") and getattr(_m, "to_host_ints", None) is _orig:
        _m.to_host_ints = _traced
sf = float(os.environ.get("SF", "0.01"))
e = ig.QueryEngine(device="cuda:0")
datagen.register(e, sf)
for q in [int(x) for x in os.environ.get("QS", "16").split(",")]:
    plan = None
    logs = []
    e.sql(queries.QUERIES[q])
    plan, _ = e.logical_plan(queries.QUERIES[q])
    for i in range(int(os.environ.get("N", "12"))):
        STACKS.clear()
        sp = _lib.Speculation("record")
        _lib.set_speculation(sp)
        try:
            e._execute_plan(plan)
        finally:
            _lib.set_speculation(None)
        logs.append(sp.log)
        stacks = list(STACKS)
    lens = {len(l) for l in logs}
    print(f"Q{q}: {len(logs)} runs, sequence lengths {sorted(lens)}", flush=True)
    if len(lens) == 1:
        for j in range(len(logs[0])):
            vals = {tuple(l[j][1]) for l in logs}
            if len(vals) > 1:
                code, line = logs[0][j][0][0]
                print(f"  site {j}: {code.co_filename.split('igloo_amd/')[-1]}:{line} ({code.co_name}) values {sorted(vals)[:6]}",
                      flush=True)
                if len(stacks) == len(logs[0]):
                    print("     stack:", stacks[j], flush=True)
