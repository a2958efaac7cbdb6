"""Bytes budget of one ResNet-50 step: per kernel family, the HBM bytes
it moves (rocprofv3 --pmc, bench/pmc_step.sh, last step of the run), its time in the
serialised counter run, its time per step in the real TWO-STREAM step (rocprofv3
--kernel-trace of bench.py, mean over the timed steps, split by HIP stream: main = critical
path, side = weight gradients / collectives), and the time those bytes take at 6 TB/s.

    python bench/bytes_budget.py <pmc root> <kernel_trace.csv> [--warmup 5 --steps 10] > profiles/bytes_budget_r05.txt
"""
import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import last_step, load_pass, short  # noqa: E402

BW = 6.0e12   # bytes/s reachable (MI355X_MICROARCH: ~6-6.3 TB/s streaming)


def family(name):
    return short(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_root")
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    gb = defaultdict(lambda: [0.0, 0.0, 0.0, 0])    # rd, wr, serial ms, calls
    for p, cs in (("A", ()), ("B", ("FETCH_SIZE",)), ("C", ("WRITE_SIZE",))):
        per, dur = load_pass(os.path.join(a.pmc_root, "pass" + p))
        for i in last_step(per):
            k = family(per[i]["name"])
            if p == "A":
                gb[k][2] += dur.get(i, 0.0)
                gb[k][3] += 1
            if "FETCH_SIZE" in cs:
                gb[k][0] += 2.0 * per[i].get("FETCH_SIZE", 0.0) * 1024
            if "WRITE_SIZE" in cs:
                gb[k][1] += per[i].get("WRITE_SIZE", 0.0) * 1024
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    # steps end with the optimizer kernel (the next batch may be generated on the side stream
    # during a step's forward, so the data kernel is no step boundary)
    marks = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
    lo, hi = marks[a.warmup - 1] + 1, marks[a.warmup + a.steps - 1] + 1
    t0, t1 = int(rows[lo]["Start_Timestamp"]), int(rows[hi - 1]["End_Timestamp"])
    streams = defaultdict(float)
    two = defaultdict(lambda: defaultdict(float))
    for r in rows[lo:hi]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / a.steps
        s = r.get("Stream_Id") or r.get("Queue_Id")
        two[family(r["Kernel_Name"])][s] += d
        streams[s] += d
    main_s = max(streams, key=streams.get)          # the stream with the most kernel time
    step_ms = (t1 - t0) / 1e6 / a.steps
    print(f"# bytes budget of one ResNet-50 bs256 step, MI355X{(' -- ' + a.title) if a.title else ''}")
    print(f"# GB: rocprofv3 --pmc of the last step (2 x FETCH_SIZE + WRITE_SIZE); serial ms: that counter run")
    print(f"# main/side ms: per timed step of the two-stream kernel trace (stream {main_s} = main); "
          f"@6TB/s: GB / 6 TB/s")
    print(f"# two-stream step: {step_ms:.3f} ms wall; main-stream kernel time {streams[main_s]:.3f} ms; "
          "other streams " + ", ".join(f"{s}: {v:.3f}" for s, v in streams.items() if s != main_s))
    tot = [0.0] * 5
    print(f"{'kernel family':58s} {'calls':>5s} {'rdGB':>6s} {'wrGB':>6s} {'GB':>6s} {'@6TB/s':>7s} {'serial':>7s} "
          f"{'main':>7s} {'side':>7s}")
    keys = sorted(set(gb) | set(two), key=lambda k: -(gb[k][0] + gb[k][1]))
    for k in keys:
        rd, wr, ms, n = gb[k]
        m = two[k].get(main_s, 0.0)
        sd = sum(v for s, v in two[k].items() if s != main_s)
        g = (rd + wr) / 1e9
        if g < 0.005 and m + sd < 0.005:
            continue
        print(f"{k:58s} {n:5d} {rd / 1e9:6.2f} {wr / 1e9:6.2f} {g:6.2f} {1e3 * (rd + wr) / BW:7.3f} {ms:7.3f} "
              f"{m:7.3f} {sd:7.3f}")
        for j, v in enumerate((rd / 1e9, wr / 1e9, ms, m, sd)):
            tot[j] += v
    print(f"{'TOTAL':58s} {'':5s} {tot[0]:6.2f} {tot[1]:6.2f} {tot[0] + tot[1]:6.2f} "
          f"{1e3 * (tot[0] + tot[1]) * 1e9 / BW:7.3f} {tot[2]:7.3f} {tot[3]:7.3f} {tot[4]:7.3f}")


if __name__ == "__main__":
    main()
