"""CPU proxy baseline: the same synthetic TPC-H data queried on
the host with pyarrow's multithreaded compute kernels (Acero group-by), since
DataFusion itself is not installable offline. Covers the scan-heavy Q1 and Q6
(whose plans are a filter + aggregate, i.e. what any columnar CPU engine
runs); times exclude data generation.

usage: python scripts/cpu_proxy.py --sf 10 [--repeat 3]
"""
import argparse
import datetime
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pyarrow as pa  # noqa: E402
import pyarrow.compute as pc  # noqa: E402


def lineitem_arrow(sf: float) -> pa.Table:
    from igloo_amd.models.tpch import datagen
    tabs = datagen.generate(sf, "cpu", 0, 1, tables=["lineitem"])
    li = tabs["lineitem"]
    cols = ["l_quantity", "l_extendedprice", "l_discount", "l_tax", "l_returnflag", "l_linestatus", "l_shipdate"]
    return pa.table({c: li.columns[c].to_arrow() for c in cols})


def q1(t: pa.Table):
    cutoff = datetime.date(1998, 12, 1) - datetime.timedelta(days=90)
    f = t.filter(pc.less_equal(t["l_shipdate"], pa.scalar(cutoff, pa.date32())))
    one = pa.scalar(1, pa.decimal128(15, 2))
    disc_price = pc.multiply(f["l_extendedprice"], pc.subtract(one, f["l_discount"])).cast(pa.decimal128(20, 4))
    charge = pc.multiply(disc_price, pc.add(one, f["l_tax"]))
    g = pa.table({"rf": f["l_returnflag"], "ls": f["l_linestatus"], "qty": f["l_quantity"],
                  "price": f["l_extendedprice"], "disc": f["l_discount"], "dp": disc_price, "ch": charge})
    return g.group_by(["rf", "ls"]).aggregate([("qty", "sum"), ("price", "sum"), ("dp", "sum"), ("ch", "sum"),
                                                ("qty", "mean"), ("price", "mean"), ("disc", "mean"),
                                                ("qty", "count")])


def q6(t: pa.Table):
    d0, d1 = pa.scalar(datetime.date(1994, 1, 1), pa.date32()), pa.scalar(datetime.date(1995, 1, 1), pa.date32())
    lo, hi = pa.scalar(5, pa.decimal128(15, 2)), pa.scalar(7, pa.decimal128(15, 2))
    m = pc.and_(pc.and_(pc.greater_equal(t["l_shipdate"], d0), pc.less(t["l_shipdate"], d1)),
                pc.and_(pc.and_(pc.greater_equal(t["l_discount"], pc.divide(lo, 100)),
                                pc.less_equal(t["l_discount"], pc.divide(hi, 100))),
                        pc.less(t["l_quantity"], pa.scalar(24, pa.decimal128(15, 2)))))
    f = t.filter(m)
    return pc.sum(pc.multiply(f["l_extendedprice"], f["l_discount"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    t0 = time.time()
    t = lineitem_arrow(a.sf)
    gen = time.time() - t0
    out = {"sf": a.sf, "rows": t.num_rows, "datagen_s": round(gen, 2), "threads": pa.cpu_count()}
    for name, fn in (("Q01", q1), ("Q06", q6)):
        fn(t)
        best = 1e9
        for _ in range(a.repeat):
            s = time.perf_counter()
            fn(t)
            best = min(best, time.perf_counter() - s)
        out[name + "_ms"] = round(best * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
