"""Winograd F(2x2,3x3) vs the implicit-GEMM MFMA conv on the ResNet-50 stride-1
3x3 layers at per-GPU batch 256: forward (+BN stats) and dgrad, with the
Winograd phase breakdown (filter / input transform / 16 GEMMs on the native MFMA kernel,
with hipBLASLt bmm timed alongside as a comparator / output), and the FUSED forward
(filter transform + one kernel, ops/winograd.py conv_fwd_fused).

    python bench/winograd_bench.py [--batch 256] > profiles/winograd_r01.txt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import winograd as WG  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    print(f"# batch {a.batch}; times in us; TF = useful direct-conv TFLOP/s")
    print(f"{'layer':>16} | {'igemm fwd':>9} {'wino fwd':>9} {'fused':>7} {'(kern)':>7} | {'filt':>6} {'in':>7} {'gemm':>7}"
          f" {'(bmm)':>8} {'out':>7} | {'igemm dg':>9} {'wino dg':>9}")
    for c, h in ((64, 56), (128, 28), (256, 14), (512, 7)):
        k = c
        x = torch.randn(a.batch, h, h, c, device="cuda").to(torch.bfloat16)
        w = (torch.randn(k, c, 3, 3, device="cuda") / (9 * c) ** 0.5).contiguous(
            memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, c, True)
        dy = torch.randn(a.batch, h, h, k, device="cuda").to(torch.bfloat16)
        flops = 2.0 * a.batch * h * h * k * c * 9

        def ig():
            y, st = HP.conv_fwd(x, wp, 1, 1, True)
            HP._release(st)

        def wg():
            y, st = WG.conv_fwd(x, wp[0], True, HP._acquire(k, x.device))
            HP._release(st)
        U = C.winograd_filter(wp[0], False)
        V = C.winograd_input(x)
        M = C.winograd_gemm(V, U)
        def fu():
            y, st = WG.conv_fwd_fused(x, wp[0], True, HP._acquire(k, x.device))
            HP._release(st)
        C.conv_set_tile(1)     # the implicit GEMM alone (the tuner's candidate 14 IS the fused kernel)
        t_ig = timeit(ig)
        C.conv_set_tile(0)
        t_wg, t_fu = timeit(wg), timeit(fu)
        t_fk = timeit(lambda: C.winograd_fused_fwd(x, U, False))
        t_f = timeit(lambda: C.winograd_filter(wp[0], False))
        t_i = timeit(lambda: C.winograd_input(x))
        t_b = timeit(lambda: C.winograd_gemm(V, U))
        t_bl = timeit(lambda: torch.bmm(V, U.transpose(1, 2)))
        t_o = timeit(lambda: C.winograd_output(M, a.batch, h, h, False, None))
        t_igd = timeit(lambda: HP.conv_dgrad(dy, wp, tuple(x.shape), 1, 1))
        t_wgd = timeit(lambda: WG.conv_dgrad(dy, wp[0], tuple(x.shape)))
        name = f"C{c}_H{h}_K{k}_R3"
        print(f"{name:>16} | {t_ig:9.1f} {t_wg:9.1f} {t_fu:7.1f} ({t_fk:5.1f}) | {t_f:6.1f} {t_i:7.1f} {t_b:7.1f} ({t_bl:6.1f}) {t_o:7.1f} |"
              f" {t_igd:9.1f} {t_wgd:9.1f}   (igemm {flops / t_ig / 1e6:.0f} TF, fused wino {flops / t_fu / 1e6:.0f} TF)",
              flush=True)


if __name__ == "__main__":
    main()
