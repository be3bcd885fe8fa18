"""Run a few TPC-H queries until they are captured as query graphs and print
what the capture did (exec/graphs.py STATS / LAST_ERROR)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igloo_amd as ig  # noqa: E402
from igloo_amd.exec import graphs  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402
from igloo_amd.ops import jit  # noqa: E402

sf = float(os.environ.get("SF", "0.01"))
qs = [int(q) for q in os.environ.get("QS", "6,1,3").split(",")]
SYNC = os.environ.get("SYNCDEBUG") == "1"
_seen = set()


def _showwarning(message, category, filename, lineno, file=None, line=None):
    import traceback
    frames = [f for f in traceback.extract_stack() if "igloo_amd" in f.filename]
    key = tuple((f.filename, f.lineno) for f in frames[-3:])
    if key not in _seen:
        _seen.add(key)
        print(f"[sync] {message}".strip()[:120], flush=True)
        for f in frames[-4:]:
            print(f"    {f.filename.split('repo/')[-1]}:{f.lineno} {f.name}", flush=True)


if SYNC:
    import warnings
    warnings.simplefilter("always")
    warnings.showwarning = _showwarning
e = ig.QueryEngine(device="cuda:0")
datagen.register(e, sf)
for q in qs:
    for i in range(6):
        if i == 2:
            jit.wait_all(timeout=120)
        if SYNC:
            torch.cuda.set_sync_debug_mode(1 if i >= 3 else 0)
        t = time.perf_counter()
        r = e.sql(queries.QUERIES[q])
        if SYNC:
            torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize()
        print(f"Q{q} run {i}: {e.last_metrics['speculation']} {1e3 * (time.perf_counter() - t):.2f} ms rows={r.table.num_rows}",
              flush=True)
    print(graphs.STATS, flush=True)
    if e.last_metrics["speculation"] != "graph":
        for st in e._spec.values():
            for site, vals in (st.get("log") or []):
                if vals is None:
                    code, line = site[0]
                    print(f"  volatile readback: {code.co_filename.split('repo/')[-1]}:{line} ({code.co_name})", flush=True)
    for m in graphs.LAST_ERROR:
        print(m, flush=True)
    graphs.LAST_ERROR.clear()
