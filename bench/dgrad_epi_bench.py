"""Short-reduction 1x1 dgrads with the fused block-backward epilogue (ResNet-50
bottleneck, per-GPU batch 256): times each (layer, operand set) as it runs in
the training step and reports achieved HBM bandwidth against the exact byte
count of the operands it must move:

    A = dY [M][K] bf16, out = dX [M][C] bf16, addend [M][C] bf16 (+ ReLU bitmask),
    BN-backward reduce over 1-2 (y [M][C] bf16, params) sets gated by a bitmask.

    python bench/dgrad_epi_bench.py [--batch 256] [--iters 20] [--choices 0,1,4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C as _C  # noqa: E402

# (name, C = dX channels, K = reduction, H, addend, addend_mask, nsets, count in R50)
CASES = [
    ("l1b1.conv1", 64, 64, 56, True, False, 0, 1),
    ("l1b2.conv1", 256, 64, 56, True, True, 2, 1),
    ("l1b3.conv1", 256, 64, 56, True, True, 1, 1),
    ("l1.conv3", 64, 256, 56, False, False, 1, 3),
    ("l2b1.conv1", 256, 128, 56, True, False, 1, 1),
    ("l2b2.conv1", 512, 128, 28, True, True, 2, 1),
    ("l2b3.conv1", 512, 128, 28, True, True, 1, 2),
    ("l2.conv3", 128, 512, 28, False, False, 1, 4),
    ("l3b1.conv1", 512, 256, 28, True, False, 1, 1),
    ("l3b2.conv1", 1024, 256, 14, True, True, 2, 1),
    ("l3b3.conv1", 1024, 256, 14, True, True, 1, 4),
    ("l4b1.conv1", 1024, 512, 14, True, False, 1, 1),
    ("l4b2.conv1", 2048, 512, 7, True, True, 2, 1),
    ("l4b3.conv1", 2048, 512, 7, True, True, 1, 1),
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
    ap.add_argument("--only", default="")
    ap.add_argument("--tile", type=int, default=0, help="conv_set_tile policy (0 = autotuned)")
    ap.add_argument("--fp8", action="store_true",
                    help="also time the fp8 dgrad (e5m2 dY x e4m3 transposed weights) with the same epilogue")
    ap.add_argument("--impl", type=int, default=5,
                    help="conv_set_impl staging (0 = register staging, 1 = LDS-DMA BK=64, 5 = per shape)")
    a = ap.parse_args()
    _C.conv_set_tile(a.tile)
    _C.conv_set_impl(a.impl)
    dev = "cuda"
    N = a.batch
    tot_us = tot_ideal = 0.0
    print(f"{'case':>12} {'M':>8} {'C':>5} {'K':>4} {'sets':>4} | {'us':>7} {'GB':>6} {'TB/s':>5} "
          f"| plain-dgrad us  TB/s")
    for (name, C, K, H, add, amask, nsets, cnt) in CASES:
        if a.only and a.only not in name:
            continue
        M = N * H * H
        g = torch.Generator(device=dev).manual_seed(0)
        dy = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(K, C, 1, 1, device=dev, generator=g) / K ** 0.5).contiguous(
            memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, C, True)
        xshape = (N, H, H, C)
        addend = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16) if add else None
        pid = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev),
                           torch.ones(C, device=dev), torch.zeros(C, device=dev)]).contiguous()
        am = None
        if amask:
            _, am = HP.bn_apply(torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16),
                                pid, relu=True)
        sets = [(torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16), pid)
                for _ in range(nsets)]
        mk = None
        if nsets:
            _, mk = HP.bn_apply(sets[0][0], pid, relu=True)

        def run():
            if nsets:
                _, rr = HP.conv_dgrad(dy, wp, xshape, 1, 0, addend, bnred=(mk, sets), addend_mask=am)
                HP._release(*rr)
            else:
                HP.conv_dgrad(dy, wp, xshape, 1, 0, addend, addend_mask=am)

        def plain():
            HP.conv_dgrad(dy, wp, xshape, 1, 0)
        t = timeit(run, a.iters)
        tp = timeit(plain, a.iters)
        f8s = ""
        if a.fp8:
            sdy = torch.tensor([1.0], device=dev)
            sw = torch.tensor([64.0], device=dev)
            dyq = _C.quant_bf16_fp8(dy, sdy, None, bf8=True)
            _, wtq = _C.quant_weight_fp8_t(w, C, sw, None)

            def run8():
                if nsets:
                    _, rr = HP.conv_dgrad_fp8(dyq, sdy, wtq, sw, xshape, 1, 0, addend, bnred=(mk, sets),
                                              addend_mask=am)
                    HP._release(*rr)
                else:
                    HP.conv_dgrad_fp8(dyq, sdy, wtq, sw, xshape, 1, 0, addend, addend_mask=am)
            f8s = f" | fp8 {timeit(run8, a.iters) * 1e3:7.1f}"
        gb = (M * K * 2 + M * C * 2 + (M * C * 2 if add else 0) + (M * C // 8 if amask else 0)
              + nsets * M * C * 2 + (M * C // 8 if nsets else 0)) / 1e9
        gbp = (M * K * 2 + M * C * 2) / 1e9
        print(f"{name:>12} {M:>8} {C:>5} {K:>4} {nsets:>4} | {t * 1e3:7.1f} {gb:6.3f} {gb / t:5.2f} "
              f"| {tp * 1e3:7.1f} {gbp / tp:5.2f}{f8s}", flush=True)
        tot_us += cnt * t * 1e3
        tot_ideal += cnt * gb / 6.0 * 1e3   # at ~6 TB/s achievable HBM
        del dy, addend, sets, am, mk
    print(f"R50 count-weighted: {tot_us:.0f} us (at 6 TB/s on the exact bytes: {tot_ideal:.0f} us)")


if __name__ == "__main__":
    main()
