"""Main-stream idle gaps of the bench.py step, split by cause, from a rocprofv3 --kernel-trace
--hip-trace run: for each gap before a main-stream kernel, was its launch API call issued by
the host only AFTER the previous kernel ended (host-bound: the Python/launch path is the
bottleneck), or was it queued in time (device-side: a cross-stream event wait / barrier packet
or dispatch latency)?   python bench/host_lag.py <dir with run_kernel_trace.csv, run_hip_api_trace.csv>"""
import csv
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    K = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
    api = {}
    for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))):
        api[r["Correlation_Id"]] = r
    marks = [i for i, r in enumerate(K) if "synth_images" in r["Kernel_Name"]]
    nm = lambda r: re.sub(r"\(.*\)$", "", r["Kernel_Name"]).replace("void ", "").replace("pmd::", "")[:48]
    tot = defaultdict(float)
    n = 0
    worst = []
    for s in range(len(marks) - 1)[-6:]:
        R = K[marks[s]:marks[s + 1]]
        mq = R[0]["Queue_Id"]
        m = [r for r in R if r["Queue_Id"] == mq]
        for a, b in zip(m, m[1:]):
            gap = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
            if gap <= 0:
                continue
            c = api.get(b["Correlation_Id"])
            if c is None:
                tot["no api record"] += gap
                continue
            issued = int(c["End_Timestamp"])           # the launch call has returned: packet is in the queue
            late = issued - int(a["End_Timestamp"])
            if late > 0:
                tot["host late"] += min(gap, late)
                tot["device after host"] += max(0, gap - late)
            else:
                tot["device (queued in time)"] += gap
            worst.append((gap / 1e3, late / 1e3, nm(a), nm(b)))
        n += 1
    print(f"main-stream idle per step over the last {n} steps (us):")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"  {v / 1e3 / n:8.1f}  {k}")
    print("\nlargest gaps (us): gap, host lateness (>0: launch returned after the previous kernel ended)")
    for w in sorted(worst, reverse=True)[:20]:
        print("  %6.1f  %7.1f  after %-48s before %s" % w)


if __name__ == "__main__":
    main()
