"""Summarise bench/pmc_conv.sh: one line per (shape, config) for the conv kernel
(median dispatch of the last iterations).

    python bench/pmc_conv_summary.py gpurun_out/pmcc

  us      kernel time under the counter run (serialised, profiled clock)
  MFMA%   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  TF      SQ_INSTS_MFMA x 16384 FLOP (one 16x16x32 bf16 MFMA; the MF32 config undercounts 2x) / time
  wait%   SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)
  inst%   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: MFMA dependency / pipe busy)
  act%    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  ldsc%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  V/M L/M VALU and LDS instructions per MFMA;  vmlvl  SQ_INST_LEVEL_VMEM / SQ_ACTIVE_INST_VMEM
  L2hit%  TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv" not in r["Kernel_Name"] and "winograd" not in r["Kernel_Name"]:
                continue
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] = per[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv" in r["Kernel_Name"]:
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ids = sorted(per)[-4:]          # last dispatches: warm
    agg = defaultdict(float)
    for i in ids:
        for k, v in per[i].items():
            agg[k] += v / len(ids)
    us = sorted(dur[i] for i in ids if i in dur)
    agg["us"] = us[len(us) // 2] if us else float("nan")
    return agg


def main():
    root = sys.argv[1]
    print(f"{'shape/pass':>22} {'cfg':>6} {'us':>7} {'MFMA%':>6} {'TF':>6} {'wait%':>6} {'inst%':>6} "
          f"{'act%':>5} {'ldsc%':>6} {'V/M':>5} {'L/M':>5} {'vmlvl':>6} {'L2hit%':>6}")
    for tagdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(tagdir):
            continue
        cfgs = sorted({os.path.basename(p)[:-3] for p in glob.glob(os.path.join(tagdir, "*_p1"))})
        for c in cfgs:
            a, b = load(os.path.join(tagdir, c + "_p1")), load(os.path.join(tagdir, c + "_p2"))
            cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
            wc = a.get("SQ_WAVE_CYCLES", 0) or float("nan")
            mf = b.get("SQ_INSTS_MFMA", 0) or float("nan")
            print(f"{os.path.basename(tagdir):>22} {c:>6} {a['us']:7.1f} "
                  f"{100 * a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (1024 * cyc) if cyc else 0:6.1f} "
                  f"{mf * 16384 / (a['us'] * 1e6):6.0f} "
                  f"{100 * a.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * a.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
                  f"{100 * a.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.1f} "
                  f"{100 * a.get('SQ_LDS_BANK_CONFLICT', 0) / max(a.get('SQ_LDS_IDX_ACTIVE', 1), 1):6.1f} "
                  f"{b.get('SQ_INSTS_VALU', 0) / mf:5.2f} {b.get('SQ_INSTS_LDS', 0) / mf:5.2f} "
                  f"{b.get('SQ_INST_LEVEL_VMEM', 0) / max(b.get('SQ_ACTIVE_INST_VMEM', 1), 1):6.2f} "
                  f"{100 * b.get('TCC_HIT_sum', 0) / max(b.get('TCC_HIT_sum', 0) + b.get('TCC_MISS_sum', 0), 1):6.1f}")


if __name__ == "__main__":
    main()
