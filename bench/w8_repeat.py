"""Repeat the 8-rank-on-one-GPU oracle step (tests/test_distributed_gpu.py _worker) K times in one
configuration and count the runs that break the per-tensor bound (diagnosis of an intermittent
deviation; see profiles/w8_intermittent_r06.txt).

    python bench/w8_repeat.py [--runs 10] [--det 0|1] [--streams 0|1] [--world 8]
"""
import argparse
import os
import sys
import tempfile

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--det", type=int, default=0)
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    import test_distributed_gpu as T
    import test_model_oracle_gpu as oracle
    ms, loss, grads = oracle._runs(train=True, model="res")
    nbad = 0
    for k in range(a.runs):
        out = os.path.join(tempfile.mkdtemp(), "r0.pt")
        mp.spawn(T._worker, args=(a.world, T._free_port(), out, "xgmi", "none", "res", bool(a.det), bool(a.streams)),
                 nprocs=a.world, join=True)
        got = torch.load(out, weights_only=True)
        bad, e1, e2 = T._oracle_violations(got, ms, loss, grads)
        worst = sorted(((e2[n] / max(e1[n], 1e-6), n) for n in e2), reverse=True)[:3]
        nbad += bool(bad)
        print(f"run {k}: {'BAD ' + str(bad) if bad else 'ok'}; worst e2/e1 "
              + ", ".join(f"{n} {r:.2f}" for r, n in worst), flush=True)
    print(f"[w8_repeat] world {a.world} det {a.det} streams {a.streams}: {nbad} of {a.runs} runs break the bound",
          flush=True)


if __name__ == "__main__":
    main()
