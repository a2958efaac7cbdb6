"""FP8 vs bf16 weight (or, --dgrad, data) gradient per ResNet-50 layer (batch 256):
the e5m2 x e4m3 scaled-MFMA kernel (conv_wgrad_fp8 / conv_dgrad_fp8) against the bf16
kernel the tuner picks, median us and TFLOP/s, split reduce included for the wgrads.

    python bench/wgrad_fp8_bench.py [--iters 20] [--only 3x3|1x1] [--dgrad]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

# (C, H, K, R, stride) of the ResNet-50 block convs
SHAPES = [(64, 56, 64, 3, 1), (128, 56, 128, 3, 2), (128, 28, 128, 3, 1), (256, 28, 256, 3, 2),
          (256, 14, 256, 3, 1), (512, 14, 512, 3, 2), (512, 7, 512, 3, 1),
          (64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (128, 28, 512, 1, 1), (512, 28, 128, 1, 1),
          (256, 14, 1024, 1, 1), (1024, 14, 256, 1, 1), (512, 7, 2048, 1, 1), (2048, 7, 512, 1, 1)]


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
    ap.add_argument("--only", default="")
    ap.add_argument("--dgrad", action="store_true", help="time the data gradients instead")
    a = ap.parse_args()
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    tuning.load_default()
    torch.manual_seed(0)
    print(f"{'layer C_H_K_R_s':>22} {'bf16 us':>8} {'TF':>5} {'fp8 us':>8} {'TF':>5} {'speedup':>8}")
    tb = tf = 0.0
    for Cin, H, K, R, st in SHAPES:
        if a.only and a.only != f"{R}x{R}":
            continue
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(a.batch, H, H, Cin, device="cuda").relu().to(torch.bfloat16)
        dy = (torch.randn(a.batch, P, P, K, device="cuda") * 1e-3).to(torch.bfloat16)
        sx = torch.tensor([100.0], device="cuda")
        sdy = torch.tensor([1e6], device="cuda")
        xq = C.quant_bf16_fp8(x, sx, None)
        dyq = C.quant_bf16_fp8(dy, sdy, None, bf8=True)
        dw = torch.zeros(K, R, R, Cin, device="cuda")
        b = timeit(lambda: C.conv_wgrad(dy, x, R, R, st, pad, dw), a.iters)
        f = timeit(lambda: C.conv_wgrad_fp8(dyq, xq, sdy, sx, R, R, st, pad, dw), a.iters)
        if a.dgrad:
            # plain data gradients (no epilogue): the tuned bf16 kernel vs the fp8 one
            from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
            w = (torch.randn(K, Cin, R, R, device="cuda") / (Cin * R * R) ** 0.5).contiguous(
                memory_format=torch.channels_last)
            wp = HP.conv_weight(w, torch.bfloat16, Cin, True)
            sw = torch.tensor([64.0], device="cuda")
            _, wtq = C.quant_weight_fp8_t(w, Cin, sw, None)
            xs = (a.batch, H, H, Cin)
            b = timeit(lambda: HP.conv_dgrad(dy, wp, xs, st, pad), a.iters)
            f = timeit(lambda: HP.conv_dgrad_fp8(dyq, sdy, wtq, sw, xs, st, pad), a.iters)
        fl = 2.0 * a.batch * P * P * K * R * R * Cin
        tb += b
        tf += f
        print(f"{f'{Cin}_{H}_{K}_{R}_{st}':>22} {b:8.1f} {fl / b / 1e6:5.0f} {f:8.1f} {fl / f / 1e6:5.0f} "
              f"{b / f:8.2f}")
    print(f"{'sum':>22} {tb:8.1f} {'':5} {tf:8.1f} {'':5} {tb / tf:8.2f}")


if __name__ == "__main__":
    main()
