"""Compact per-kernel summary of a rocprofv3 (rocpd SQLite) kernel trace.

    python bench/prof_summary.py gpurun_out/prof/run_results.db [--steps N] > profiles/x.txt

Template arguments are kept (they name the tile config), argument lists are
dropped.  With --steps the per-step time of each kernel is also shown.
"""
import argparse
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("void ", "").replace("pmd::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="training steps in the trace")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--skip", type=int, default=0,
                    help="ignore everything before the (skip+1)-th --marker dispatch (warm-up / "
                         "autotuning steps); then --steps defaults to the markers counted after it")
    ap.add_argument("--marker", default="synth_images_kernel", help="one dispatch per training step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = {}
    if a.skip:
        ks = c.execute("select name, start, end from kernels order by start").fetchall()
        marks = [i for i, (n, _, _) in enumerate(ks) if a.marker in n]
        if len(marks) <= a.skip:
            raise SystemExit(f"only {len(marks)} '{a.marker}' dispatches in the trace")
        ks = ks[marks[a.skip]:]
        if not a.steps:
            a.steps = len(marks) - a.skip
        span = (ks[-1][2] - ks[0][1]) / 1e6
        busy = sum(e - s for _, s, e in ks) / 1e6
        print(f"# window: {a.steps} steps, wall {span:.2f} ms ({span / a.steps:.2f} ms/step), "
              f"kernels busy {busy:.2f} ms ({100 * busy / span:.1f}% of wall)")
        for n, s_, e_ in ks:
            e = agg.setdefault(short(n), [0, 0.0])
            e[0] += 1
            e[1] += (e_ - s_) / 1e3
    else:
        rows = c.execute("select name, total_calls, total_duration, average from top_kernels").fetchall()
        for n, calls, tot, _ in rows:
            k = short(n)
            e = agg.setdefault(k, [0, 0.0])
            e[0] += calls
            e[1] += tot
    total = sum(v[1] for v in agg.values())
    print(f"# total kernel time {total / 1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches"
          + (f"; {total / 1e3 / a.steps:.2f} ms per step ({a.steps} steps)" if a.steps else ""))
    hdr = f"{'kernel':70s} {'calls':>7s} {'total ms':>9s} {'avg us':>8s} {'%':>6s}"
    if a.steps:
        hdr += f" {'ms/step':>8s}"
    print(hdr)
    for k, (calls, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        line = f"{k[:70]:70s} {calls:7d} {tot / 1e3:9.2f} {tot / calls:8.1f} {100 * tot / total:6.2f}"
        if a.steps:
            line += f" {tot / 1e3 / a.steps:8.3f}"
        print(line)


if __name__ == "__main__":
    main()
