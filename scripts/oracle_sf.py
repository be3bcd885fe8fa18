"""Independent answer oracle at scale: the CPU engine against sqlite3 over
the same generated TPC-H data, all 22 queries (an oracle beyond
SF0.01). The SF1 GPU tests compare GPU results with the CPU engine
(tests/test_tpch_sf1_gpu.py), so this run anchors them to an implementation
that shares no code with the engine (sqlite's own parser, planner and
executor).

    python scripts/oracle_sf.py --sf 1 [--queries 1-22] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--queries", default="1-22")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import igloo_amd as ig
    from igloo_amd.models.tpch import datagen, oracle, queries
    qs = []
    for part in a.queries.split(","):
        lo, _, hi = part.partition("-")
        qs += list(range(int(lo), int(hi or lo) + 1))
    t0 = time.perf_counter()
    e = ig.QueryEngine(device="cpu")
    tabs = datagen.register(e, a.sf)
    t1 = time.perf_counter()
    con = oracle.load_sqlite(datagen.to_arrow(tabs))
    t2 = time.perf_counter()
    print(f"[oracle] sf={a.sf} datagen {t1 - t0:.1f}s sqlite load {t2 - t1:.1f}s", flush=True)
    out = {"sf": a.sf, "queries": {}}
    bad = []
    for q in qs:
        ta = time.perf_counter()
        got = [tuple(oracle.normalize(v) for v in r.values()) for r in e.sql(queries.QUERIES[q]).table.to_pylist()]
        tb = time.perf_counter()
        exp = [tuple(str(x) if isinstance(x, str) else x for x in row) for row in oracle.run_sqlite(con, q)]
        tc = time.perf_counter()
        d = oracle.rows_match(got, exp)
        out["queries"][q] = {"rows": len(got), "engine_s": round(tb - ta, 3), "sqlite_s": round(tc - tb, 3),
                             "match": not d, "diff": d}
        if d:
            bad.append(q)
        print(f"[oracle] Q{q:02d} rows={len(got)} engine {tb - ta:.2f}s sqlite {tc - tb:.2f}s "
              f"{'OK' if not d else 'MISMATCH ' + d}", flush=True)
    out["mismatched"] = bad
    print(json.dumps({"sf": a.sf, "queries": len(qs), "mismatched": bad}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
