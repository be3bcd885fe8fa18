"""Per-kernel time of the last N executions of a query in a rocprofv3 kernel
trace (csv): the region starts at the N-th-last launch of a marker kernel
that runs once per execution.   python scripts/trace_tail.py TRACE.csv MARKER N [TOP]"""
import csv
import sys
from collections import defaultdict


def main():
    path, marker, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if marker in r["Kernel_Name"]]
    t0 = marks[-n]
    tot, cnt = defaultdict(float), defaultdict(int)
    busy = 0.0
    for r in rows:
        if int(r["Start_Timestamp"]) < t0:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"].replace("igloo::kern::(anonymous namespace)::", "")[:100]
        tot[name] += d
        cnt[name] += 1
        busy += d
    end = max(int(r["End_Timestamp"]) for r in rows)
    print(f"region {(end - t0) / 1e6 / n:.3f} ms per execution, kernels busy {busy / n:.3f} ms per execution")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:top]:
        print(f"{v / n:9.3f} ms {cnt[k] / n:6.1f}x  {k}")


if __name__ == "__main__":
    main()
