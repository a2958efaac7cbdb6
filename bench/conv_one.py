"""Run ONE conv layer configuration repeatedly (for rocprofv3 --pmc passes).

    python bench/conv_one.py C H K R stride [--tile T] [--pipe P] [--impl I] [--pass fwd|dgrad|wgrad]
                             [--wimpl W]   (wgrad staging variant, conv_wgrad.hip; -1 = autotuned)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C as _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    for k in ("C", "H", "K", "R", "stride"):
        ap.add_argument(k, type=int)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tile", type=int, default=1)
    ap.add_argument("--pipe", type=int, default=0)
    ap.add_argument("--impl", type=int, default=5)
    ap.add_argument("--pass", dest="which", default="fwd")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nostats", action="store_true", help="forward without BN statistics")
    ap.add_argument("--wimpl", type=int, default=-1, help="wgrad staging variant (-1: autotuned)")
    a = ap.parse_args()
    _C.conv_set_autotune(0)
    _C.conv_set_tile(a.tile)
    _C.conv_set_big_pipe(a.pipe)
    _C.conv_set_impl(a.impl)
    pad = a.R // 2
    x = torch.randn(a.batch, a.H, a.H, a.C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(a.K, a.C, a.R, a.R, device="cuda") / (a.C * a.R * a.R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, a.C, True)
    y, s = HP.conv_fwd(x, wp, a.stride, pad, True)
    dy = torch.randn_like(y)
    dw = torch.zeros(tuple(wp[0].shape), device="cuda", dtype=torch.float32)
    if a.which == "wgrad" and a.wimpl >= 0:
        _C.conv_wgrad_set_impl(a.wimpl)
    ts = []
    for _ in range(a.iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        if a.which == "fwd":
            y, s = HP.conv_fwd(x, wp, a.stride, pad, not a.nostats)
            if s is not None:
                HP._release(s)
        elif a.which == "wgrad":
            HP.conv_wgrad(dy, x, tuple(wp[0].shape), a.stride, pad, out=dw)
        else:
            HP.conv_dgrad(dy, wp, tuple(x.shape), a.stride, pad)
        e1.record()
        ts.append((e0, e1))
    torch.cuda.synchronize()
    us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ts[2:])
    print(f"done {a.which} C{a.C} H{a.H} K{a.K} R{a.R} s{a.stride} tile {a.tile} impl {a.impl} "
          f"stats {not a.nostats}: {us[len(us) // 2]:.1f} us")


if __name__ == "__main__":
    main()
