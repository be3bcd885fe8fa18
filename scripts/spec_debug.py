"""Per-query speculation modes over 5 runs (IGLOO_SPEC_DEBUG=1 prints mismatching readbacks)."""
import sys; sys.path.insert(0, '.')
import igloo_amd as ig
from igloo_amd.models.tpch import datagen, queries
from igloo_amd.utils.digest import digest
e = ig.QueryEngine(device="cuda:0"); datagen.register(e, 1.0)
for q in range(1, 23):
    modes = []; ds = set()
    for _ in range(5):
        ds.add(digest(e.sql(queries.QUERIES[q]).table)); modes.append(e.last_metrics["speculation"])
    print(q, modes, len(ds), flush=True)
