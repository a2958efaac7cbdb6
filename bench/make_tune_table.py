"""Build a committed kernel tuning table by MAJORITY VOTE over several
independent autotuning processes (each a fresh `bench.py --tune_table online`
run: step-0 timing of every candidate on the live two-stream step).  A single
process's choices are noisy on near-tied candidates; the vote is stable.

    python bench/make_tune_table.py --runs 5 --out pytorch_multiprocessing_distributed_amd/ops/tables/r50_bs256_gfx950.json \
        [-- extra bench.py args]
"""
import argparse
import collections
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--out", required=True)
    ap.add_argument("--tmp", default="gpurun_out/tune_votes")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    os.makedirs(a.tmp, exist_ok=True)
    tabs = []
    for r in range(a.runs):
        path = os.path.join(a.tmp, f"run{r}.json")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "2",
               "--tune_table", "online", "--save_tune_table", path, *a.extra]
        print("[tune-vote]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, timeout=300)
        with open(path) as f:
            tabs.append(json.load(f))
    out = dict(tabs[0])
    report = []
    for kind, klen in (("conv", 13), ("wgrad", 11)):
        votes = collections.defaultdict(collections.Counter)
        for t in tabs:
            for e in t.get(kind, []):
                votes[tuple(e[:klen])][e[klen]] += 1
        rows = []
        for key in sorted(votes):
            (choice, n), = votes[key].most_common(1)
            rows.append(list(key) + [choice])
            if n < a.runs:
                report.append(f"{kind} {key}: {dict(votes[key])} -> {choice}")
        out[kind] = rows
    out["votes"] = a.runs
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f)
    print(f"[tune-vote] {len(out['conv'])} conv + {len(out['wgrad'])} wgrad entries -> {a.out}")
    print(f"[tune-vote] {len(report)} non-unanimous keys:")
    for line in report:
        print("  " + line)


if __name__ == "__main__":
    main()
