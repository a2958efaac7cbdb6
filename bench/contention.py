"""Contention attribution of the two-stream step (kernel traces of bench.py): for every main-stream
kernel instance, its duration next to the side stream minus its duration in a single-stream run of
the same step (PMD_WGRAD_STREAM=0, same order), attributed to the side-stream kernel families it
overlapped (by overlap time).  python bench/contention.py <two-stream trace> <single-stream trace> [--step 8]
(a trace: a rocprofv3 kernel_trace.csv, or a directory holding one; bash bench/contention.sh runs both)."""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def nm(r):
    return re.sub(r"\(.*\)$", "", r["Kernel_Name"]).replace("void ", "").replace("pmd::", "")[:58]


def step_rows(path, step):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with its optimizer kernel (the next step's batch may be generated on the side
    # stream during this step's forward, so the data kernel is no step boundary)
    marks = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
    return rows[marks[step] + 1:marks[step + 1] + 1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("two")
    ap.add_argument("one")
    ap.add_argument("--step", type=int, default=8)
    x = ap.parse_args()
    A = step_rows(x.two, x.step)
    B = step_rows(x.one, x.step)
    mq = A[-1]["Queue_Id"]          # the optimizer kernel runs on the main stream
    main_a = [r for r in A if r["Queue_Id"] == mq]
    side_a = [r for r in A if r["Queue_Id"] != mq]
    # drop from the single-stream run the kernels that only the side stream runs in the two-stream
    # one (a family that runs on both -- e.g. the forward convs next to the side-stream
    # projection shortcut -- stays, and difflib aligns what matches)
    side_only = {nm(r) for r in side_a} - {nm(r) for r in main_a}
    main_b = [r for r in B if nm(r) not in side_only]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    import difflib
    sm = difflib.SequenceMatcher(None, [nm(r) for r in main_a], [nm(r) for r in main_b], autojunk=False)
    pairs = []
    for blk in sm.get_matching_blocks():
        pairs += [(main_a[blk.a + i], main_b[blk.b + i]) for i in range(blk.size)]
    print(f"main kernels: two-stream {len(main_a)}, single-stream {len(main_b)}, aligned {len(pairs)}")
    blame = defaultdict(float)
    by_main = defaultdict(float)
    tot = 0.0
    for a, b in pairs:
        ex = dur(a) - dur(b)
        tot += ex
        by_main[nm(a)] += ex
        s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        ov = defaultdict(float)
        for o in side_a:
            lo, hi = max(s, int(o["Start_Timestamp"])), min(e, int(o["End_Timestamp"]))
            if hi > lo:
                ov[nm(o)] += (hi - lo)
        t = sum(ov.values())
        if t <= 0:
            blame["(no side kernel)"] += ex
        else:
            for k, v in ov.items():
                blame[k] += ex * v / t
    wall_a = (int(A[-1]["End_Timestamp"]) - int(A[0]["Start_Timestamp"])) / 1e3
    wall_b = (int(B[-1]["End_Timestamp"]) - int(B[0]["Start_Timestamp"])) / 1e3
    print(f"step wall us: two-stream {wall_a:.0f}, single-stream {wall_b:.0f}; main-kernel excess {tot:.0f} us")
    print("\nexcess of main-stream kernels, by the side-stream kernel they overlapped (us/step):")
    for k, v in sorted(blame.items(), key=lambda kv: -kv[1]):
        print(f"  {v:8.1f}  {k}")
    print("\nexcess by main-stream kernel family (us/step):")
    for k, v in sorted(by_main.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {v:8.1f}  {k}")
    fam_side = defaultdict(float)
    for o in side_a:
        fam_side[nm(o)] += dur(o)
    print("\nside-stream kernel time (us/step):")
    for k, v in sorted(fam_side.items(), key=lambda kv: -kv[1]):
        print(f"  {v:8.1f}  {k}")


if __name__ == "__main__":
    main()
