"""BN-apply in the consumer conv's prologue, measured in
isolation on the ResNet-50 bs256 conv3 forwards (bn2 -> ReLU -> conv3, the cheapest
consumer: 1x1, stride 1, no padding):

  separate : bn_apply(y2) -> z2 (+ ReLU mask), then the tuned conv3 forward reads z2
  prologue : conv3 forward reads y2 and forms relu(y2 * scale + shift) on each A fragment
             (conv_igemm_kernel<..., PRO>, `_C.conv_fwd_pro`), z2 never written

Checks the prologue output is bit-identical to the separate path, then prints both
times.  Only the forward side: the backward of the prologue design (conv3 wgrad reading
y2 through the same transform, the ReLU mask re-derived from y2 in the fused-reduce dgrad)
can only add cost, so a forward that does not win here settles the question.

    python bench/bn_prologue_bench.py [--batch 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C as _C  # noqa: E402

# (name, C_mid, H, count in R50): conv3 is C_mid -> 4 C_mid
CASES = [("l1.conv3", 64, 56, 3), ("l2.conv3", 128, 28, 4), ("l3.conv3", 256, 14, 6), ("l4.conv3", 512, 7, 3)]


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
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    N = a.batch
    tot_sep = tot_pro = 0.0
    print(f"{'case':>9} {'M':>7} {'C':>4} {'K':>5} | {'bn_apply':>8} {'conv':>7} {'sep':>7} | {'pro':>7} "
          f"{'pro/sep':>7} exact")
    for (name, C, H, cnt) in CASES:
        K = 4 * C
        M = N * H * H
        g = torch.Generator(device=dev).manual_seed(0)
        y = (torch.randn(N, H, H, C, device=dev, generator=g) * 2 + 0.5).to(torch.bfloat16)
        p = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev),
                         torch.rand(C, device=dev, generator=g) + 0.5,
                         torch.randn(C, device=dev, generator=g) * 0.5]).contiguous()
        w = (torch.randn(K, C, 1, 1, device=dev, generator=g) / C ** 0.5).contiguous(
            memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, C, True)
        shift = torch.zeros(K, device=dev)
        buf = torch.zeros(64, 2, K, device=dev)
        z, _ = HP.bn_apply(y, p, relu=True)
        ref = _C.conv_fwd(z, wp[0], 1, 0, True, buf, shift)[0]
        out = _C.conv_fwd_pro(y, wp[0], p, True, buf, shift)[0]
        torch.cuda.synchronize()
        # the tuned separate-path kernel may differ from the prologue's tile: compare values
        exact = bool(torch.equal(out, ref))
        rel = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        assert rel < 5e-3, (name, rel)
        t_bn = timeit(lambda: HP.bn_apply(y, p, relu=True), a.iters)
        t_cv = timeit(lambda: _C.conv_fwd(z, wp[0], 1, 0, True, buf, shift), a.iters)
        t_sep = timeit(lambda: _C.conv_fwd(HP.bn_apply(y, p, relu=True)[0], wp[0], 1, 0, True, buf, shift),
                       a.iters)
        t_pro = timeit(lambda: _C.conv_fwd_pro(y, wp[0], p, True, buf, shift), a.iters)
        print(f"{name:>9} {M:>7} {C:>4} {K:>5} | {t_bn:8.1f} {t_cv:7.1f} {t_sep:7.1f} | {t_pro:7.1f} "
              f"{t_pro / t_sep:7.3f} {'yes' if exact else f'rel {rel:.1e}'}", flush=True)
        tot_sep += cnt * t_sep
        tot_pro += cnt * t_pro
    print(f"R50 conv3 forwards, count-weighted: separate {tot_sep:.0f} us, prologue {tot_pro:.0f} us "
          f"({tot_pro - tot_sep:+.0f} us per step)")


if __name__ == "__main__":
    main()
