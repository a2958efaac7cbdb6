"""Achieved HBM bandwidth of the BN-family kernels on the ResNet-50 shapes.

    python bench/bn_bench.py [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = "cuda"
    print(f"{'shape':>18} | {'apply':>14} {'apply+res':>14} {'reduce':>14} {'elemt':>14}  (us, TB/s)")
    for hw, c in [(112, 64), (56, 64), (56, 256), (28, 128), (28, 512), (14, 256), (14, 1024),
                  (7, 512), (7, 2048)]:
        M = a.batch * hw * hw
        y = torch.randn(M, c, device=dev).to(torch.bfloat16)
        r = torch.randn(M, c, device=dev).to(torch.bfloat16)
        g = torch.rand(c, device=dev) + 0.5
        b = torch.randn(c, device=dev)
        yf = y[:4096].float()
        sums = torch.stack([yf.sum(0), (yf * yf).sum(0)]) * (M / 4096)
        cnt = torch.tensor([float(M)], device=dev)
        p = HP.bn_finalize(sums, cnt, g, b, 1e-5)
        out, mask = HP.bn_apply(y, p)
        nb = M * c * 2
        t1 = timeit(lambda: HP.bn_apply(y, p))
        t2 = timeit(lambda: HP.bn_apply(y, p, res=r))
        red = HP.stats_collapse(HP.bn_bwd_reduce(out, mask, y, p, True)).view(2, c)

        def reduce():
            HP._release(HP.bn_bwd_reduce(out, mask, y, p, True))   # timing only (no clear)
        t3 = timeit(reduce)
        t4 = timeit(lambda: HP.bn_bwd_elemt(out, mask, y, p, g, red, float(M), True))

        def bw(t, passes):
            return f"{t * 1e3:6.0f} {passes * nb / t / 1e9:5.2f}"
        print(f"{f'{hw}x{hw}x{c}':>18} | {bw(t1, 2.06):>14} {bw(t2, 3.06):>14} {bw(t3, 2.06):>14} "
              f"{bw(t4, 3.06):>14}", flush=True)


if __name__ == "__main__":
    main()
