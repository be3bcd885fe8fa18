"""Share of timed GPU busy time spent in PyTorch ATen kernels (at::native::*)
vs hand-written / generated kernels, from a rocprofv3 kernel trace of a
bench.py run with IGLOO_PROF_GAP=1 (timed steps only).

usage: python scripts/aten_share.py <run_kernel_trace.csv> [--steps N] [--top 25]"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(a.trace)))
    cut = 0
    for (s0, _, _), (s1, _, _) in zip(rows, rows[1:]):
        if s1 - s0 > 500e6:
            cut = s1
    rows = [r for r in rows if r[0] >= cut]
    cls = defaultdict(float)
    per = defaultdict(lambda: [0.0, 0])
    for s, e, n in rows:
        d = (e - s) / 1e6 / a.steps
        k = "aten" if n.startswith("at::") or "at::native" in n else (
            "copy" if "rocclr" in n else ("generated" if n.startswith("igloo_jit") else "hand-written"))
        cls[k] += d
        if k == "aten":
            nm = re.sub(r"<.*", "", n.replace("at::native::", ""))
            fn = re.search(r"at::native::(\w+Functor\w*|\w+Ops)", n)
            nm += ":" + fn.group(1) if fn else ""
            per[nm][0] += d
            per[nm][1] += 1
    busy = sum(cls.values())
    print(f"busy {busy:.2f} ms/step: " + ", ".join(f"{k} {v:.2f} ms ({100 * v / busy:.1f}%)" for k, v in
                                                  sorted(cls.items(), key=lambda kv: -kv[1])))
    for nm, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {t:7.3f} ms {c // a.steps:5d} calls  {nm}")


if __name__ == "__main__":
    main()
