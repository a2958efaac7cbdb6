"""Per-kernel-family time per step (split by hardware queue) of two rocprofv3 kernel traces of
bench.py, and their difference: python bench/trace_diff.py <traceA.csv> <traceB.csv> [--skip 6 --n 8]"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*\)$", "", n).replace("void ", "").replace("pmd::", "")[:60]


def load(path, skip, n):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "synth_images" in r["Kernel_Name"]]
    lo, hi = marks[skip], marks[skip + n]
    fam = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for r in rows[lo:hi]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / n
        fam[short(r["Kernel_Name"])][r["Queue_Id"]] += d
        cnt[short(r["Kernel_Name"])] += 1
    wall = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e6 / n
    return fam, cnt, wall


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--skip", type=int, default=6)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--top", type=int, default=25)
    x = ap.parse_args()
    a, ca, wa = load(x.a, x.skip, x.n)
    b, cb, wb = load(x.b, x.skip, x.n)
    print(f"wall ms/step: A {wa:.3f}  B {wb:.3f}  (B - A {wb - wa:+.3f})")
    rows = []
    for k in set(a) | set(b):
        ta, tb = sum(a[k].values()), sum(b[k].values())
        rows.append((tb - ta, k, ta, tb, ca[k] / x.n, cb[k] / x.n,
                     {q: round(v, 3) for q, v in a[k].items()}, {q: round(v, 3) for q, v in b[k].items()}))
    for r in sorted(rows, key=lambda r: -abs(r[0]))[:x.top]:
        print("%+.3f  %-60s A %.3f B %.3f  calls %.0f/%.0f  A%s B%s" % r)


if __name__ == "__main__":
    main()
