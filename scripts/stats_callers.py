"""Which call sites run column_stats (a full pass over a key column) on
intermediates during warm TPC-H queries, and over how many rows."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import igloo_amd as ig  # noqa: E402
from igloo_amd.models.tpch import datagen, queries  # noqa: E402
from igloo_amd.ops import hashing as H  # noqa: E402

sf = float(os.environ.get("SF", "10"))
e = ig.QueryEngine(device="cuda:0")
datagen.register(e, sf)
for q in range(1, 23):
    e.sql(queries.QUERIES[q])
orig = H.column_stats
calls = collections.Counter()
rows = collections.Counter()


def traced(keys, valid=None):
    if getattr(keys, "_igloo_stats", None) is None or valid is not None:
        st = [f for f in traceback.extract_stack()[:-1] if "igloo_amd" in f.filename][-3:]
        k = " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}({f.name})" for f in st[::-1])
        calls[k] += 1
        rows[k] += keys.numel()
    return orig(keys, valid)


H.column_stats = traced
for mod in list(sys.modules.values()):
    if mod is not None and getattr(mod, "__name__", "").startswith("igloo_amd") and getattr(mod, "column_stats", None) is orig:
        mod.column_stats = traced
for q in range(1, 23):
    e.sql(queries.QUERIES[q])
for k, c in sorted(calls.items(), key=lambda kv: -rows[kv[0]])[:25]:
    print(f"{rows[k] / 1e6:10.1f} Mrows {c:4d} calls  {k}")
