"""Per-layer conv microbenchmark: gfx950 implicit-GEMM kernels vs MIOpen.

For each unique ResNet-50 (ImageNet, 224^2) conv shape at the per-GPU batch,
times fwd / dgrad / wgrad of our kernels and of PyTorch-ROCm (MIOpen,
channels_last bf16, cudnn.benchmark) and prints TFLOP/s.  Usage:

    python bench/conv_bench.py --batch 256 [--iters 20] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP  # noqa: E402

# (C, H, K, R, stride, count-in-R50)
SHAPES = [
    (8, 224, 64, 7, 2, 1), (64, 56, 64, 1, 1, 1), (64, 56, 64, 3, 1, 3), (64, 56, 256, 1, 1, 4),
    (256, 56, 64, 1, 1, 2), (256, 56, 128, 1, 1, 1), (128, 56, 128, 3, 2, 1), (256, 56, 512, 1, 2, 1),
    (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (128, 28, 128, 3, 1, 3), (512, 28, 256, 1, 1, 1),
    (256, 28, 256, 3, 2, 1), (512, 28, 1024, 1, 2, 1), (256, 14, 1024, 1, 1, 6),
    (1024, 14, 256, 1, 1, 5), (256, 14, 256, 3, 1, 5), (1024, 14, 512, 1, 1, 1),
    (512, 14, 512, 3, 2, 1), (1024, 14, 2048, 1, 2, 1), (512, 7, 2048, 1, 1, 3),
    (2048, 7, 512, 1, 1, 2), (512, 7, 512, 3, 1, 2),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
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
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--json", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--impls", default="5", help="conv staging/pipeline impls to time (see conv_igemm.hip; 5 = per-shape default)")
    ap.add_argument("--tiles", default="", help="also time fwd/dgrad with these conv tile policies "
                    "(conv_set_tile) as tile[:bigpipe], e.g. 1,2:0,2:1,3:0")
    ap.add_argument("--wimpls", default="", help="also time these wgrad staging impls (conv_wgrad.hip)")
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="also time the e4m3 scaled-MFMA forward conv")
    ap.add_argument("--bnred", action="store_true",
                    help="also time dgrad with the fused BN-backward reduce, and the separate reduce")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = "cuda"
    rows = []
    tot = {"ours": 0.0, "miopen": 0.0}
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    impls = [int(v) for v in a.impls.split(",")]
    print(f"{'shape':>24} | {'fwd ours':>9} {'miopen':>7} | {'dgrad':>9} {'miopen':>7} | "
          f"{'wgrad':>9} {'miopen':>7}   (TFLOP/s; ours per impl {impls})")
    for (C, H, K, R, st, cnt) in SHAPES:
        name = f"C{C}_H{H}_K{K}_R{R}_s{st}"
        if a.only and a.only not in name:
            continue
        pad = R // 2
        N = a.batch
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, C, R, R, device=dev) / (C * R * R) ** 0.5).contiguous(
            memory_format=torch.channels_last)
        wp = HP.conv_weight(w, torch.bfloat16, C, True)
        y, _ = HP.conv_fwd(x, wp, st, pad, True)
        P = y.shape[1]
        dy = torch.randn_like(y)
        flops = 2.0 * N * P * P * K * C * R * R

        def fwd():
            yy, ss = HP.conv_fwd(x, wp, st, pad, True)
            HP._release(ss)          # recycle without clearing: timing only
        per = {}
        for im in impls:
            _C.conv_set_impl(im)
            per[im] = (timeit(fwd, a.iters),
                       timeit(lambda: HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad), a.iters)
                       if C != 8 else 0.0,
                       timeit(lambda: HP.conv_wgrad(dy, x, tuple(wp[0].shape), st, pad), a.iters))
        t_f, t_d, t_w = per[impls[-1]]
        f8txt = ""
        if a.tiles and C != 8:
            tt = []
            for spec in a.tiles.split(","):
                tl, _, bp = spec.partition(":")
                _C.conv_set_tile(int(tl))
                _C.conv_set_big_pipe(int(bp or 0))
                tt.append((timeit(fwd, a.iters),
                           timeit(lambda: HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad), a.iters)))
            _C.conv_set_tile(0)
            _C.conv_set_big_pipe(0)
            f8txt += "   tiles fwd " + "/".join(f"{flops / t[0] / 1e9:.0f}" for t in tt)
            f8txt += " dgrad " + "/".join(f"{flops / t[1] / 1e9:.0f}" for t in tt)
        if a.wimpls:
            wt = []
            for wi in [int(v) for v in a.wimpls.split(",")]:
                _C.conv_wgrad_set_impl(wi)
                wt.append(timeit(lambda: HP.conv_wgrad(dy, x, tuple(wp[0].shape), st, pad), a.iters))
            _C.conv_wgrad_set_impl(1)
            f8txt += "   wgrad impls " + "/".join(f"{flops / t / 1e9:.0f}" for t in wt)
        if a.bnred and C != 8:
            yb = torch.randn_like(x)
            pb = torch.stack([torch.zeros(C, device=dev), torch.ones(C, device=dev),
                              torch.ones(C, device=dev), torch.zeros(C, device=dev)]).contiguous()
            _, mk = HP.bn_apply(yb, pb, relu=True)

            def dg_fused():
                _, rr = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad, None, bnred=(mk, [(yb, pb)]))
                HP._release(*rr)
            dxx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad)

            def red_sep():
                HP._release(HP.bn_bwd_reduce(dxx, mk, yb, pb, True))
            tdf = timeit(dg_fused, a.iters)
            trs = timeit(red_sep, a.iters)
            f8txt += f"   dgrad+fusedred {tdf * 1e3:6.0f}us  dgrad {t_d * 1e3:6.0f}us  sep.reduce {trs * 1e3:5.0f}us"
        if a.fp8 and C % 16 == 0:
            sx = torch.tensor([1.0], device=dev)
            sw = torch.tensor([64.0], device=dev)
            xq = _C.quant_bf16_fp8(x, sx, None)
            wq = _C.quant_weight_fp8(w, C, sw, None)

            def f8():
                yy, ss = HP.conv_fp8_fwd(xq, wq, sx, sw, st, pad, True)
                HP._release(ss)
            t8 = timeit(f8, a.iters)
            f8txt = f"   fp8 fwd {flops / t8 / 1e9:6.0f}"
        # MIOpen (NCHW-shaped channels_last views of the same data)
        xn = x.permute(0, 3, 1, 2)
        wn = w.to(torch.bfloat16)
        dyn = dy.permute(0, 3, 1, 2)
        if a.no_miopen:
            m_f = m_d = m_w = 0.0
        else:
            m_f = timeit(lambda: F.conv2d(xn, wn, stride=st, padding=pad), a.iters)
            m_d = timeit(lambda: torch.nn.grad.conv2d_input(xn.shape, wn, dyn, stride=st,
                                                            padding=pad), a.iters) if C != 8 else 0.0
            m_w = timeit(lambda: torch.nn.grad.conv2d_weight(xn, wn.shape, dyn, stride=st,
                                                             padding=pad), a.iters)

        def tf(t):
            return flops / t / 1e9 if t > 0 else 0.0

        def cell(k, m):
            ours = "/".join(f"{tf(per[im][k]):.0f}" for im in impls)
            return f"{ours:>9} {tf(m):7.0f}"
        print(f"{name:>24} | {cell(0, m_f)} | {cell(1, m_d)} | {cell(2, m_w)}{f8txt}", flush=True)
        tot["ours"] += cnt * (t_f + t_d + t_w)
        tot["miopen"] += cnt * (m_f + m_d + m_w)
        rows.append(dict(shape=name, count=cnt, ms=dict(fwd=t_f, dgrad=t_d, wgrad=t_w),
                         ms_by_impl={str(k): v for k, v in per.items()},
                         miopen_ms=dict(fwd=m_f, dgrad=m_d, wgrad=m_w), gflop=flops / 1e9))
    print(f"R50 conv total (count-weighted): ours {tot['ours']:.2f} ms, MIOpen {tot['miopen']:.2f} ms")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(batch=a.batch, rows=rows, total_ms=tot), f, indent=1)


if __name__ == "__main__":
    main()
