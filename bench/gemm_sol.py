"""Speed-of-light check for the 1x1 convolutions: each ResNet-50 bs256 1x1
stride-1 conv IS a plain GEMM in NHWC (Y[M,K] = X[M,C] W^T), so time our
implicit-GEMM conv kernel (fwd, no BN statistics) against the vendor library
GEMM (torch.mm -> hipBLASLt) on the same bf16 operands, plus one large square
GEMM for the chip's practical bf16 MFMA ceiling.

    python bench/gemm_sol.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402

# (C, H, K): 1x1 stride-1 convs of ResNet-50 at batch 256
SHAPES = [(64, 56, 64), (64, 56, 256), (256, 56, 64), (256, 56, 128),
          (128, 28, 512), (512, 28, 128), (256, 14, 1024), (1024, 14, 256),
          (512, 7, 2048), (2048, 7, 512)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
    return us[len(us) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    torch.manual_seed(0)
    print(f"{'GEMM M x N x K':>26} {'ours us':>9} {'TF':>6} {'hipBLASLt us':>13} {'TF':>6} {'GB/s@ours':>10}")
    for n in (8192,):
        A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.mm(A, B), a.iters)
        print(f"{f'{n} x {n} x {n} (square)':>26} {'-':>9} {'-':>6} {t:13.1f} {2 * n ** 3 / t / 1e6:6.0f}")
    for C, H, K in SHAPES:
        M = a.batch * H * H
        x = torch.randn(a.batch, H, H, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5).contiguous(memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, C, True)
        ours = timeit(lambda: HP.conv_fwd(x, wp, 1, 0, False), a.iters)
        X = x.view(M, C)
        Wt = w.view(K, C).to(torch.bfloat16).t()
        lib = timeit(lambda: torch.mm(X, Wt), a.iters)
        fl = 2.0 * M * C * K
        by = 2.0 * M * (C + K)
        print(f"{f'{M} x {K} x {C}':>26} {ours:9.1f} {fl / ours / 1e6:6.0f} {lib:13.1f} {fl / lib / 1e6:6.0f} "
              f"{by / ours / 1e3:10.0f}")


if __name__ == "__main__":
    main()
