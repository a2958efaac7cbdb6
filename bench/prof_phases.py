"""Forward / backward / optimizer phases of the training steps in a rocprofv3
(rocpd SQLite) kernel trace: per phase the wall span, the summed kernel time,
the time at least one kernel was running (union) and the time two or more
overlapped -- i.e. how much of each phase the chip is idle between dispatches
and how much the two-stream schedule actually overlaps.

    python bench/prof_phases.py gpurun_out/prof/run_results.db [--skip 5]

Phases (one step = synth_images_kernel .. next synth_images_kernel):
  forward  = step start .. xent_fwd_kernel end
  backward = xent_fwd end .. start of sgd_kernel
  update   = sgd_kernel .. step end
"""
import argparse
import sqlite3


def union_and_overlap(iv):
    """iv: list of (start, end) -> (union length, length covered by >= 2)."""
    ev = []
    for s, e in iv:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    depth, last, uni, ov = 0, None, 0, 0
    for t, d in ev:
        if last is not None:
            if depth >= 1:
                uni += t - last
            if depth >= 2:
                ov += t - last
        depth += d
        last = t
    return uni, ov


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=5, help="steps to ignore (warmup / tuning)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = c.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, k in enumerate(ks) if "synth_images_kernel" in k[0]]
    steps = []
    for si in range(a.skip, len(marks)):
        lo = marks[si]
        hi = marks[si + 1] if si + 1 < len(marks) else len(ks)
        seg = ks[lo:hi]
        xi = max(i for i, k in enumerate(seg) if "xent_fwd_kernel" in k[0])
        sg = [i for i, k in enumerate(seg) if "sgd_kernel" in k[0]]
        if not sg:
            continue
        t0, tx, ts = seg[0][1], seg[xi][2], seg[sg[0]][1]
        tend = ks[hi][1] if hi < len(ks) else max(k[2] for k in seg)
        ph = {}
        for name, lo_t, hi_t in (("forward", t0, tx), ("backward", tx, ts), ("update", ts, tend)):
            iv = [(max(s, lo_t), min(e, hi_t)) for _, s, e in seg if e > lo_t and s < hi_t]
            uni, ov = union_and_overlap(iv)
            ph[name] = (hi_t - lo_t, sum(e - s for s, e in iv), uni, ov)
        steps.append(ph)
    if not steps:
        print("no complete steps")
        return
    n = len(steps)
    print(f"# {n} steps (after skipping {a.skip}); ms per step, averaged")
    print(f"{'phase':10s} {'span':>8s} {'kernel sum':>11s} {'busy(union)':>12s} {'idle':>7s} {'overlap>=2':>11s}")
    tot = [0.0] * 4
    for name in ("forward", "backward", "update"):
        v = [sum(s[name][i] for s in steps) / n / 1e6 for i in range(4)]
        tot = [x + y for x, y in zip(tot, v)]
        print(f"{name:10s} {v[0]:8.3f} {v[1]:11.3f} {v[2]:12.3f} {v[0] - v[2]:7.3f} {v[3]:11.3f}")
    print(f"{'step':10s} {tot[0]:8.3f} {tot[1]:11.3f} {tot[2]:12.3f} {tot[0] - tot[2]:7.3f} {tot[3]:11.3f}")


if __name__ == "__main__":
    main()
