"""Per-stream timeline of the END of one training step's backward from a rocprofv3
(rocpd SQLite) kernel trace: which kernels run on which queue in the last
``--ms`` milliseconds before the optimizer kernel, and how long the main queue
sits idle waiting for the weight-gradient stream (the step's serial tail).

    python bench/prof_tail.py gpurun_out/prof/run_results.db [--step -2] [--ms 3]
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("void ", "").replace("pmd::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--ms", type=float, default=3.0)
    ap.add_argument("--marker", default="synth_images_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    qcol = next((k for k in ("stream_id", "queue_id") if k in cols), None)
    sel = f"name, start, end, {qcol if qcol else '0'}"
    ks = c.execute(f"select {sel} from kernels order by start").fetchall()
    marks = [i for i, k in enumerate(ks) if a.marker in k[0]] + [len(ks)]
    s = a.step if a.step >= 0 else len(marks) - 1 + a.step
    seg = ks[marks[s]:marks[s + 1]]
    sgd = next(k for k in seg if "sgd_kernel" in k[0])
    t_end = sgd[1]
    t0 = t_end - a.ms * 1e6
    print(f"# step {s}: last {a.ms} ms before sgd_kernel (queue column: {qcol})")
    print(f"{'queue':>6} {'start_us':>9} {'dur_us':>8}  kernel")
    busy = {}
    for name, st, en, q in seg:
        if en < t0 or st > t_end:
            continue
        busy.setdefault(q, []).append((max(st, t0), min(en, t_end)))
        print(f"{q:>6} {(st - t_end) / 1e3:9.1f} {(en - st) / 1e3:8.1f}  {short(name)}")
    for q, iv in sorted(busy.items()):
        iv.sort()
        tot, last = 0, t0
        for st, en in iv:
            st = max(st, last)
            if en > st:
                tot += en - st
                last = en
        print(f"# queue {q}: busy {tot / 1e3:.1f} of {a.ms * 1e3:.0f} us")


if __name__ == "__main__":
    main()
