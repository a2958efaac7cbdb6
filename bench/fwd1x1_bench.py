"""Forward 1x1 stride-1 convolutions with the BN-statistics epilogue (ResNet-50 bs256
shapes): time and achieved HBM bandwidth on the exact bytes (read x, write y), tiled
implicit-GEMM kernel vs the persistent streaming kernel (kernels/conv1x1_stream.hip).

    python bench/fwd1x1_bench.py [--batch 256] [--iters 20] [--s1 0|2] [--s1bn 0|64|128]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C as _C  # noqa: E402

# (name, Cin, Cout, H, count in R50)
CASES = [
    ("l1.conv1a", 64, 64, 56, 1), ("l1.conv1", 256, 64, 56, 2), ("l1.conv3", 64, 256, 56, 3),
    ("l1.short", 64, 256, 56, 1), ("l2b1.conv1", 256, 128, 56, 1), ("l2.conv1", 512, 128, 28, 3),
    ("l2.conv3", 128, 512, 28, 4), ("l3b1.conv1", 512, 256, 28, 1), ("l3.conv1", 1024, 256, 14, 5),
    ("l3.conv3", 256, 1024, 14, 6), ("l4b1.conv1", 1024, 512, 14, 1), ("l4.conv1", 2048, 512, 7, 2),
    ("l4.conv3", 512, 2048, 7, 3),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--s1", type=int, default=0, help="streaming 1x1 policy (2 = forwards too)")
    ap.add_argument("--s1bn", type=int, default=0)
    a = ap.parse_args()
    _C.conv1x1_set_policy(a.s1)
    _C.conv1x1_set_bn(a.s1bn)
    dev = "cuda"
    N = a.batch
    tot = tot_ideal = 0.0
    print(f"{'case':>12} {'M':>8} {'Cin':>5} {'Cout':>5} | {'us':>7} {'GB':>6} {'TB/s':>5} {'TF':>6}")
    for (name, Cin, Cout, H, cnt) in CASES:
        M = N * H * H
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(N, H, H, Cin, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(Cout, Cin, 1, 1, device=dev, generator=g) / Cin ** 0.5).contiguous(
            memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, Cin, True)
        shift = torch.zeros(Cout, device=dev)
        buf = torch.zeros(64, 2, Cout, device=dev)     # statistics slots (accumulate across runs)

        def run():
            _C.conv_fwd(x, wp[0], 1, 0, True, buf, shift)
        t = timeit(run, a.iters)
        gb = (M * Cin * 2 + M * Cout * 2) / 1e9
        tf = 2.0 * M * Cin * Cout / (t * 1e-3) / 1e12
        print(f"{name:>12} {M:>8} {Cin:>5} {Cout:>5} | {t * 1e3:7.1f} {gb:6.3f} {gb / t:5.2f} {tf:6.0f}", flush=True)
        tot += cnt * t * 1e3
        tot_ideal += cnt * gb / 6.0 * 1e3
    print(f"R50 count-weighted: {tot:.0f} us (at 6 TB/s on the exact bytes: {tot_ideal:.0f} us)")


if __name__ == "__main__":
    main()
