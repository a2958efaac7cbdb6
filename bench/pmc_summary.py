"""Per-kernel gfx950 counter summary of bench/pmc_step.sh (last training step).

    python bench/pmc_summary.py gpurun_out/pmc [--all] [--title TEXT] > profiles/pmc_r50_step_r01.txt

(--all: every dispatch of the run instead of the last training step)

Columns (summed over the step's dispatches of each kernel):
  ms          kernel time (kernel trace of the pass-A run)
  MFMA%       MFMA pipe utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles);
              GRBM_GUI_ACTIVE is summed over the 8 XCDs, so kernel cycles = GRBM_GUI_ACTIVE / 8
              (calibrated: a 16x16x32 bf16 MFMA adds 16 busy cycles; 100% = 2.5 PFLOP/s dense)
  TF          achieved bf16 MFMA TFLOP/s = SQ_INSTS_MFMA x 16384 / time (16x16x32 / 32x32x16 forms)
  VALU/MFMA   SQ_INSTS_VALU / SQ_INSTS_MFMA
  LDSconf%    SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS  (conflict cycles per LDS instruction, %)
  rdGB wrGB   HBM bytes: 2 x FETCH_SIZE (gfx950 FETCH_SIZE counts half of wide streaming reads,
              MI355X_MICROARCH.md) and WRITE_SIZE
  TB/s        (rd + wr) / ms
  L2hit%      TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*\)$", "", n).replace("void ", "").replace("pmd::", "")
    return n[:58]


def load_pass(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(dict)   # dispatch id -> {counter: value, name}
    for f in cc:
        for r in csv.DictReader(open(f)):
            did = int(r["Dispatch_Id"])
            per[did]["name"] = r["Kernel_Name"]
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for f in kt:
        for r in csv.DictReader(open(f)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return per, dur


def last_step(per, marker="sgd_kernel"):
    """Dispatches of the run's last step: after the next-to-last optimizer kernel, through the
    last (a step ends with its optimizer kernel; with the data prefetch, a batch is generated
    during the previous step, so the data kernel is no step boundary)."""
    ids = sorted(per)
    marks = [i for i in ids if marker in per[i]["name"]]
    if not marks:
        return ids
    start = marks[-2] + 1 if len(marks) >= 2 else ids[0]
    return [i for i in ids if start <= i <= marks[-1]]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--title", default="one ResNet-50 bs256 bf16 training step")
    a = ap.parse_args()
    root = a.root
    agg = defaultdict(lambda: defaultdict(float))
    for p in "ABC":
        per, dur = load_pass(os.path.join(root, "pass" + p))
        for i in (sorted(per) if a.all else last_step(per)):
            k = short(per[i]["name"])
            for c, v in per[i].items():
                if c != "name" and (p == "A" or c != "GRBM_GUI_ACTIVE"):
                    agg[k][c] += v
            if p == "A":
                agg[k]["ms"] += dur.get(i, 0.0)
                agg[k]["calls"] += 1
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["ms"])
    tot = sum(v["ms"] for _, v in rows)
    print(f"# {a.title}, MI355X, rocprofv3 --pmc (3 passes); total {tot:.2f} ms "
          f"(counter runs serialise kernels)")
    print(f"{'kernel':58s} {'calls':>5s} {'ms':>7s} {'MFMA%':>6s} {'TF':>5s} {'VALU/MFMA':>9s} {'LDSconf%':>8s} "
          f"{'rdGB':>6s} {'wrGB':>6s} {'TB/s':>5s} {'L2hit%':>6s}")
    for k, v in rows:
        g = v.get("GRBM_GUI_ACTIVE", 0.0)
        mf = 100.0 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g * 128.0) if g else 0.0
        tf = v.get("SQ_INSTS_MFMA", 0.0) * 16384 / (v["ms"] / 1e3) / 1e12 if v["ms"] else 0.0
        nm = v.get("SQ_INSTS_MFMA", 0.0)
        vpm = v.get("SQ_INSTS_VALU", 0.0) / nm if nm else float("nan")
        nl = v.get("SQ_INSTS_LDS", 0.0)
        lc = 100.0 * v.get("SQ_LDS_BANK_CONFLICT", 0.0) / nl if nl else 0.0
        rd = 2.0 * v.get("FETCH_SIZE", 0.0) * 1024 / 1e9
        wr = v.get("WRITE_SIZE", 0.0) * 1024 / 1e9
        bw = (rd + wr) / (v["ms"] / 1e3) / 1e3 if v["ms"] else 0.0
        h, m = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        hit = 100.0 * h / (h + m) if h + m else 0.0
        print(f"{k:58s} {int(v['calls']):5d} {v['ms']:7.3f} {mf:6.1f} {tf:5.0f} {vpm:9.2f} {lc:8.1f} {rd:6.2f} {wr:6.2f} "
              f"{bw:5.2f} {hit:6.1f}")


if __name__ == "__main__":
    main()
