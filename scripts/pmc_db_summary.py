"""Per-kernel counter sums from rocprofv3 --pmc SQLite output (rocpd
run_results.db, its ``counters_collection`` view): one line per (kernel,
counter) with dispatches, summed value and summed duration, filtered by a
kernel-name substring.

    python scripts/pmc_db_summary.py gpurun_out/<dir>/run_results.db [--match probe_]"""
import argparse
import sqlite3


def _short(name: str) -> str:
    """Kernel name without its argument list (anonymous-namespace parentheses kept)."""
    name = name.replace("(anonymous namespace)", "{anon}")
    return name.split("(")[0].replace("{anon}", "(anon)")[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    for path in a.db:
        db = sqlite3.connect(path)
        q = ("select kernel_name, counter_name, count(distinct dispatch_id), sum(value), "
             "sum(duration) / count(distinct counter_name) from counters_collection "
             "where kernel_name like ? group by kernel_name, counter_name order by kernel_name, counter_name")
        print(f"# {path}")
        for k, c, n, v, d in db.execute(q, (f"%{a.match}%",)):
            print(f"{_short(k):60s} {c:16s} dispatches={n:4d} sum={v:16.0f} per_dispatch={v / n:14.0f}")


if __name__ == "__main__":
    main()
