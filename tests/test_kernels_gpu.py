"""Numerics of every gfx950 kernel against the PyTorch fp32 reference
primitive of the same op (ops/torch_prims.py), on the same bf16 inputs.

Conv shapes cover the ResNet-18-ref CIFAR layers and all 23
unique ResNet-50 ImageNet layers at a small batch, in the
fwd, dgrad and wgrad passes.
"""
import pytest
import torch

from pytorch_multiprocessing_distributed_amd.ops import torch_prims as TP

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (C, H, K, R, stride)  pad = R // 2
R50_SHAPES = [
    (8, 224, 64, 7, 2),  # stem (C padded 3 -> 8)
    (64, 56, 64, 1, 1), (64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (256, 56, 64, 1, 1),
    (256, 56, 128, 1, 1), (128, 56, 128, 3, 2), (256, 56, 512, 1, 2), (128, 28, 512, 1, 1),
    (512, 28, 128, 1, 1), (128, 28, 128, 3, 1), (512, 28, 256, 1, 1), (256, 28, 256, 3, 2),
    (512, 28, 1024, 1, 2), (256, 14, 1024, 1, 1), (1024, 14, 256, 1, 1), (256, 14, 256, 3, 1),
    (1024, 14, 512, 1, 1), (512, 14, 512, 3, 2), (1024, 14, 2048, 1, 2), (512, 7, 2048, 1, 1),
    (2048, 7, 512, 1, 1), (512, 7, 512, 3, 1),
]
CIFAR_SHAPES = [(8, 32, 64, 3, 1), (64, 32, 64, 3, 1), (64, 32, 128, 3, 2), (64, 32, 128, 1, 2),
                (128, 16, 128, 3, 1), (512, 4, 512, 3, 1)]


def _hp():
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims
    return hip_prims


def _close(a, b, rel):
    a = a.float()
    b = b.float()
    scale = b.abs().max().clamp_min(1e-6)
    err = (a - b).abs().max() / scale
    assert err < rel, f"max rel err {err.item():.3e} >= {rel}"


def _close_norm(a, b, rel):
    """Relative Frobenius error: robust to the handful of elements whose ReLU
    mask flips between two bf16 roundings of a near-zero pre-activation."""
    a = a.float()
    b = b.float()
    err = (a - b).norm() / b.norm().clamp_min(1e-12)
    assert err < rel, f"relative L2 err {err.item():.3e} >= {rel}"


# Conv fwd / dgrad oracle: both sides are the same fp32 sums rounded to bf16, so the
# relative L2 error floor is ~1e-3; 5e-3 is tight enough that a kernel dropping ONE input
# channel of a 512-channel reduction (~1/sqrt(512) = 4.4% of the output energy) fails
# (tests below: test_conv_oracle_rejects_dropped_channel).
CONV_REL_L2 = 5e-3


def _close_conv(a, b, rel_max=2e-2):
    _close(a, b, rel_max)
    _close_norm(a, b, CONV_REL_L2)


def _batch_for(h):
    return 2 if h >= 112 else (4 if h >= 28 else 8)


@pytest.mark.parametrize("shape", R50_SHAPES + CIFAR_SHAPES, ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_fwd_dgrad_wgrad(shape):
    HP = _hp()
    torch.manual_seed(0)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    wref = TP.conv_weight(w, torch.bfloat16, C)
    assert torch.equal(wp[0], wref[0])
    assert torch.equal(wp[1], wref[0].permute(3, 1, 2, 0).contiguous())
    y, st_ = HP.conv_fwd(x, wp, st, pad, True)
    yr, sr = TP.conv_fwd(x, wref, st, pad, True)
    _close_conv(y, yr)
    _close(HP.stats_collapse(st_).view(2, -1), sr, 2e-2)
    dy = torch.randn_like(y)
    dx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad)
    dxr = TP.conv_dgrad(dy, wref, tuple(x.shape), st, pad)
    _close_conv(dx, dxr)
    dw = HP.conv_wgrad(dy, x, tuple(wp[0].shape), st, pad)
    dwr = TP.conv_wgrad(dy, x, tuple(wref[0].shape), st, pad)
    _close(dw, dwr, 2e-3)


@pytest.mark.parametrize("impl", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("shape", R50_SHAPES + CIFAR_SHAPES, ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_wgrad_variants(shape, impl):
    """Every operand-staging variant of the split-K wgrad kernel (register
    staging; LDS-DMA rings of 64-row x2 / 32-row x4 / 64-row x3 stages), with a
    batch large enough that several splits and ragged split tails occur."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(2)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H) + 1  # odd batch: the last split ends mid-chunk
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, P, P, K, device=DEV).to(torch.bfloat16)
    dwr = TP.conv_wgrad(dy, x, (K, R, R, C), st, pad)
    _C.conv_wgrad_set_impl(impl)
    try:
        dw = HP.conv_wgrad(dy, x, (K, R, R, C), st, pad)
        torch.cuda.synchronize()
    finally:
        _C.conv_wgrad_set_impl(1)
    _close(dw, dwr, 2e-3)


def test_wgrad_many_splits_reproducible():
    """A tiny weight gradient over a long reduction (ResNet-50 layer-1 1x1, K = 64:
    two output tiles, hundreds of split-K slices -> several reduction groups) is
    bitwise identical run to run (fixed-order two-stage group reduction, no fp32
    atomics) and matches fp32 conv2d_weight."""
    HP = _hp()
    torch.manual_seed(7)
    N, H, C, K = 64, 56, 256, 64
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    dy = torch.randn(N, H, H, K, device=DEV).to(torch.bfloat16)
    # M = 200,704 rows over 2 output tiles: the 384-block split plan gives 192 slices
    a = HP.conv_wgrad(dy, x, (K, 1, 1, C), 1, 0)
    b = HP.conv_wgrad(dy, x, (K, 1, 1, C), 1, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, b), "split-K weight gradient differs between two identical runs"
    _close(a, TP.conv_wgrad(dy, x, (K, 1, 1, C), 1, 0), 2e-3)


@pytest.mark.parametrize("N,H,C,R,pad,P", [
    (3, 112, 16, 4, 2, 112),   # the space-to-depth stem: 4x4 over 16 ch, output cropped to H
    (3, 56, 64, 3, 1, 56),     # layer1 3x3
    (5, 28, 64, 3, 1, 28),
    (3, 20, 64, 3, 1, 20),     # 11-row bands: a ragged last band per image
    (9, 7, 64, 3, 1, 7),
])
def test_wgrad_halo(N, H, C, R, pad, P):
    """The halo wgrad (conv_wgrad.hip conv_wgrad_halo_kernel, variant 6): one
    band of whole output rows + input halo staged per block step, all taps from
    LDS.  Against fp32 conv2d_weight on the same bf16 operands (a cropped output
    is the full output with zero gradient in the cropped rows/columns)."""
    import torch.nn.functional as F
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(5)
    K = 64
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    dy = torch.randn(N, P, P, K, device=DEV).to(torch.bfloat16)
    full = H + 2 * pad - R + 1
    dyf = F.pad(dy.float().permute(0, 3, 1, 2), (0, full - P, 0, full - P))
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, R, R), dyf,
                                      padding=pad).permute(0, 2, 3, 1)
    _C.conv_wgrad_set_impl(6)
    try:
        dw = _C.conv_wgrad(dy, x, R, R, 1, pad, None)
        base = torch.randn_like(dw)
        acc = base.clone()
        _C.conv_wgrad(dy, x, R, R, 1, pad, acc)          # accumulate into a target
        torch.cuda.synchronize()
    finally:
        _C.conv_wgrad_set_impl(1)
    _close(dw, ref, 2e-3)
    _close(acc - base, ref, 2e-3)


@pytest.mark.parametrize("impl", [0, 1, 3, 4, 6, 7])
@pytest.mark.parametrize("shape", R50_SHAPES + CIFAR_SHAPES, ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_pipeline_variants(shape, impl):
    """Every operand-staging / pipeline variant of the implicit-GEMM kernel
    (register staging; LDS-DMA with BK 64/32 and 2-4 stages) on fwd + dgrad."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(1)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    wref = TP.conv_weight(w, torch.bfloat16, C)
    yr, sr = TP.conv_fwd(x, wref, st, pad, True)
    dy = torch.randn_like(yr)
    dxr = TP.conv_dgrad(dy, wref, tuple(x.shape), st, pad)
    _C.conv_set_impl(impl)
    try:
        y, st_ = HP.conv_fwd(x, wp, st, pad, True)
        dx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad)
        torch.cuda.synchronize()
    finally:
        _C.conv_set_impl(5)
    _close_conv(y, yr)
    _close(HP.stats_collapse(st_).view(2, -1), sr, 2e-2)
    _close_conv(dx, dxr)


@pytest.mark.parametrize("tile,pipe", [(2, 0), (2, 1), (2, 2), (2, 3), (3, 0), (3, 2), (3, 3), (4, 0), (5, 0),
                                       (6, 0), (7, 0), (8, 0), (9, 0), (10, 0), (11, 0), (12, 0)])
@pytest.mark.parametrize("shape", R50_SHAPES + CIFAR_SHAPES, ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_big_tiles(shape, tile, pipe):
    """8-wave 256x128 / 256x256 tiles (forced wherever legal: Cs >= 64, Nout >= 128)
    with each LDS-DMA pipeline, the 8-wave 128-row tiles (policies 4/5, Cs >= 64) and
    the register-resident P8 pipeline shapes (policies 6-9), fwd (+BN stats
    epilogue) and dgrad."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(4)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    wref = TP.conv_weight(w, torch.bfloat16, C)
    yr, sr = TP.conv_fwd(x, wref, st, pad, True)
    dy = torch.randn_like(yr)
    dxr = TP.conv_dgrad(dy, wref, tuple(x.shape), st, pad)
    _C.conv_set_tile(tile)
    _C.conv_set_big_pipe(pipe)
    try:
        y, st_ = HP.conv_fwd(x, wp, st, pad, True)
        dx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad)
        torch.cuda.synchronize()
    finally:
        _C.conv_set_tile(0)
        _C.conv_set_big_pipe(0)
    _close_conv(y, yr)
    _close(HP.stats_collapse(st_).view(2, -1), sr, 2e-2)
    _close_conv(dx, dxr)


# every forced kernel variant of the fwd/dgrad tests above: ("impl", conv_set_impl) or
# ("tile", conv_set_tile, big_pipe)
_VARIANTS = ([("impl", i, 0) for i in (0, 1, 3, 4, 6, 7)]
             + [("tile", t, p) for (t, p) in ((2, 0), (2, 1), (2, 2), (2, 3), (3, 0), (3, 2), (3, 3), (4, 0),
                                              (5, 0), (6, 0), (7, 0), (8, 0), (9, 0), (10, 0), (11, 0),
                                              (12, 0))])


@pytest.mark.parametrize("variant", _VARIANTS, ids=lambda v: "%s%d_%d" % v)
@pytest.mark.parametrize("shape", [(512, 14, 512, 3, 2), (512, 28, 128, 1, 1), (512, 7, 512, 3, 1)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_oracle_rejects_dropped_channel(shape, variant):
    """Negative control of the conv oracle: the same kernel variant run with ONE input
    channel of a 512-channel reduction zeroed in its weight image must FAIL the check the
    positive tests use, in both passes (fwd drops input channel c; dgrad drops output
    channel c of dX), while the intact weights pass it."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(9)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wref = TP.conv_weight(w, torch.bfloat16, C)
    yr, _ = TP.conv_fwd(x, wref, st, pad, False)
    dy = torch.randn_like(yr)
    dxr = TP.conv_dgrad(dy, wref, tuple(x.shape), st, pad)
    wbad = w.clone()
    wbad[:, 137] = 0.0
    kind, v, pipe = variant
    if kind == "impl":
        _C.conv_set_impl(v)
    else:
        _C.conv_set_tile(v)
        _C.conv_set_big_pipe(pipe)
    try:
        outs = {}
        for name, ww in (("good", w), ("bad", wbad)):
            wp = HP.conv_weight(ww, torch.bfloat16, C, True)
            y, _ = HP.conv_fwd(x, wp, st, pad, False)
            dx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad)
            outs[name] = (y, dx)
        torch.cuda.synchronize()
    finally:
        _C.conv_set_impl(5)
        _C.conv_set_tile(0)
        _C.conv_set_big_pipe(0)
    _close_conv(outs["good"][0], yr)
    _close_conv(outs["good"][1], dxr)
    with pytest.raises(AssertionError):
        _close_conv(outs["bad"][0], yr)
    with pytest.raises(AssertionError):
        _close_conv(outs["bad"][1], dxr)


@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("N,H,C", [(4, 112, 64), (2, 15, 64), (2, 20, 128)])
def test_fused_stem_pool_matches_composite(train, N, H, C):
    """BN+ReLU+maxpool (one kernel) and its two-pass backward == bn_apply ->
    maxpool_fwd and maxpool_bwd -> bn_bwd_reduce -> bn_bwd_elemt on the same data
    (odd sizes: a last block with one input row and no second pooled row)."""
    HP = _hp()
    torch.manual_seed(6)
    y = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    p = torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5,
                     torch.randn(C, device=DEV), torch.randn(C, device=DEV) * 0.5]).contiguous()
    out, arg = HP.stem_pool_fwd(y, p)
    a, mask = HP.bn_apply(y, p, relu=True)
    out_r, arg_r = HP.maxpool_fwd(a)
    assert torch.equal(out, out_r)
    assert torch.equal(arg, arg_r)
    dout = torch.randn_like(out)
    da = HP.maxpool_bwd(dout, arg_r, tuple(a.shape))
    red = HP.stats_collapse(HP.stem_pool_bwd_reduce(dout, arg, y, p)).view(2, C)
    red_r = HP.stats_collapse(HP.bn_bwd_reduce(da, mask, y, p, True)).view(2, C)
    _close(red, red_r, 1e-4)
    gamma = torch.rand(C, device=DEV) + 0.5
    cnt = float(N * H * H)
    if train:
        dy = HP.stem_pool_bwd_elemt(dout, arg, y, p, gamma, red_r, cnt)
        dy_r, _ = HP.bn_bwd_elemt(da, mask, y, p, gamma, red_r, cnt, True)
    else:
        dy = HP.stem_pool_bwd_elemt(dout, arg, y, p, gamma, None, None, eval_mode=True)
        dy_r, _ = HP.bn_bwd_elemt_eval(da, mask, p, True)
    _close(dy, dy_r, 1e-2)


def test_resnet50_fused_stem_step_matches_composite():
    """One ResNet-50 (ImageNet stem) training step with the fused stem tail vs the
    composite conv_bn_act + max-pool path: same loss, same gradients (bf16 noise)."""
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    res = {}
    for fused in (True, False):
        OF.set_fused_stem(fused)
        try:
            torch.manual_seed(0)
            m = ResNet50(num_classes=1000, stem="imagenet").to(DEV)
            x, y = C.synth_images(4, 64, 64, 8, 3, 1000, 7, 0)
            loss = OF.cross_entropy(m(x), y)
            loss.backward()
            torch.cuda.synchronize()
            res[fused] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()},
                          m.bn1.running_mean.clone())
        finally:
            OF.set_fused_stem(True)
    assert abs(res[True][0] - res[False][0]) < 1e-3 * abs(res[False][0])
    torch.testing.assert_close(res[True][2], res[False][2], rtol=1e-5, atol=1e-6)
    # The head is exact; deep in the backward, fp32-atomic ordering in the BN
    # statistics flips single bf16 roundings, which BN backward at random init
    # and batch 4 amplifies (two runs of the SAME path differ by as much --
    # bench/dbg_stem2.py), so the stem end is checked by direction.
    for n, lim in (("linear.weight", 0.99999), ("layer4.2.conv3.weight", 0.9999),
                   ("layer1.0.conv1.weight", 0.97), ("bn1.weight", 0.97), ("conv1.weight", 0.97)):
        g, r = res[True][1][n], res[False][1][n]
        cos = torch.nn.functional.cosine_similarity(g.flatten(), r.flatten(), dim=0).item()
        assert cos > lim, (n, cos)


def test_conv_autotuner_caches_and_matches():
    """The per-shape autotuner (cudnn.benchmark equivalent) picks a kernel on the
    first call, caches it, and the tuned launch equals the untuned one up to
    bf16 rounding; BN statistics are not double-counted by the timing runs."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(5)
    C, H, K, R, st = 256, 14, 256, 3, 1
    x = torch.randn(8, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    _C.conv_set_autotune(0)
    try:
        y0, s0 = HP.conv_fwd(x, wp, st, 1, True)
        dy = torch.randn_like(y0)
        dx0 = HP.conv_dgrad(dy, wp, tuple(x.shape), st, 1)
        dw0 = HP.conv_wgrad(dy, x, tuple(wp[0].shape), st, 1)
        ref = HP.stats_collapse(s0).view(2, -1)
    finally:
        _C.conv_set_autotune(1)
    _C.conv_autotune_clear()
    y1, s1 = HP.conv_fwd(x, wp, st, 1, True)          # tunes
    assert _C.conv_autotune_entries() >= 1
    dx1 = HP.conv_dgrad(dy, wp, tuple(x.shape), st, 1)
    dw1 = HP.conv_wgrad(dy, x, tuple(wp[0].shape), st, 1)
    y2, s2 = HP.conv_fwd(x, wp, st, 1, True)          # cached
    _close(y1, y0, 1e-2)
    _close(HP.stats_collapse(s1).view(2, -1), ref, 1e-2)
    _close(HP.stats_collapse(s2).view(2, -1), ref, 1e-2)
    assert torch.equal(y1, y2)
    _close(dx1, dx0, 1e-2)
    _close(dw1, dw0, 1e-3)


@pytest.mark.parametrize("mode", ["plain", "res", "two", "norelu"])
@pytest.mark.parametrize("C", [64, 256, 2048])
def test_bn_family(mode, C):
    HP = _hp()
    torch.manual_seed(1)
    M = 4 * 7 * 7 * 3
    y1 = (torch.randn(M, C, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    y2 = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    res = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    yf = y1.float()
    sums = torch.stack([yf.sum(0), (yf * yf).sum(0)])
    count = torch.tensor([float(M)], device=DEV)
    rm1, rv1 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm1.clone(), rv1.clone()
    nb1 = torch.zeros((), dtype=torch.long, device=DEV)
    nb2 = nb1.clone()
    p = HP.bn_finalize(sums, count, g, b, 1e-5, rm1, rv1, 0.1, nb1)
    pr = TP.bn_finalize(sums, count, g, b, 1e-5, rm2, rv2, 0.1, nb2)
    _close(p, pr, 1e-5)
    _close(rm1, rm2, 1e-5)
    _close(rv1, rv2, 1e-5)
    assert nb1.item() == nb2.item() == 1
    relu = mode != "norelu"
    kw = {}
    if mode == "res":
        kw = dict(res=res)
    if mode == "two":
        kw = dict(y2=y2, p2=pr)
    out, mask = HP.bn_apply(y1, p, relu=relu, **kw)
    outr, maskr = TP.bn_apply(y1, pr, relu=relu, **kw)
    _close(out, outr, 1e-2)
    if relu:   # bitmask bit k of byte i == element 8i+k > 0
        bits = (mask.view(-1, 1).int() >> torch.arange(8, device=DEV).view(1, 8)) & 1
        assert torch.equal(bits.view(M, C).bool(), maskr), "relu bitmask mismatch"
    dout = torch.randn(M, C, device=DEV).to(torch.bfloat16)
    red = HP.stats_collapse(HP.bn_bwd_reduce(dout, mask, y1, pr, relu)).view(2, C)
    redr = TP.bn_bwd_reduce(dout, maskr, y1, pr, relu)
    _close(red, redr, 1e-3)
    dy, dzm = HP.bn_bwd_elemt(dout, mask, y1, pr, g, redr, count, relu, want_dzm=True)
    dyr, dzmr = TP.bn_bwd_elemt(dout, maskr, y1, pr, g, redr, count, relu, want_dzm=True)
    _close(dy, dyr, 1e-2)
    _close(dzm, dzmr, 1e-2)
    dye, _ = HP.bn_bwd_elemt_eval(dout, mask, pr, relu)
    dyer, _ = TP.bn_bwd_elemt_eval(dout, maskr, pr, relu)
    _close(dye, dyer, 1e-2)
    pe = HP.bn_eval_params(rm2, rv2, g, b, 1e-5)
    per = TP.bn_eval_params(rm2, rv2, g, b, 1e-5)
    _close(pe, per, 1e-5)


def test_pools_loss_sgd():
    HP = _hp()
    torch.manual_seed(2)
    # every 3x3 window sees the 9 distinct values of a per-channel permutation: no argmax ties
    perm = torch.stack([torch.randperm(9, device=DEV) for _ in range(64)], 1).float()  # [9, C]
    hh = torch.arange(112, device=DEV) % 3
    slot = (hh.view(112, 1) * 3 + hh.view(1, 112)).view(1, 112, 112, 1).expand(2, 112, 112, 64)
    x = torch.gather(perm.view(9, 1, 1, 64).expand(9, 112, 112, 64).unsqueeze(0).expand(2, -1, -1, -1, -1),
                     1, slot.unsqueeze(1)).squeeze(1).to(torch.bfloat16)
    o, a = HP.maxpool_fwd(x)
    orf, ar = TP.maxpool_fwd(x)
    assert torch.equal(o, orf)
    do = torch.randn_like(o)
    _close(HP.maxpool_bwd(do, a, tuple(x.shape)), TP.maxpool_bwd(do, ar, tuple(x.shape)), 1e-2)
    x7 = torch.randn(4, 7, 7, 2048, device=DEV).to(torch.bfloat16)
    _close(HP.avgpool_fwd(x7), TP.avgpool_fwd(x7), 1e-4)
    g = torch.randn(4, 2048, device=DEV)
    _close(HP.avgpool_bwd(g, tuple(x7.shape), torch.bfloat16),
           TP.avgpool_bwd(g, tuple(x7.shape), torch.bfloat16), 1e-2)
    logits = torch.randn(64, 1000, device=DEV) * 3
    tgt = torch.randint(0, 1000, (64,), device=DEV)
    tgt[:8] = logits[:8].argmax(1)
    loss, lse = HP.xent_fwd(logits, tgt)
    lossr, lser = TP.xent_fwd(logits, tgt)
    _close(loss, lossr, 1e-5)
    _close(lse, lser, 1e-5)
    gl = torch.ones(1, device=DEV)
    _close(HP.xent_bwd(gl, logits, tgt, lse), TP.xent_bwd(gl, logits, tgt, lser), 1e-5)
    assert HP.correct_count(logits, tgt).item() == TP.correct_count(logits, tgt).item()
    n = 1000003
    p = torch.randn(n, device=DEV)
    gg = torch.randn(n, device=DEV)
    b1 = torch.zeros(n, device=DEV)
    p2, b2 = p.clone(), b1.clone()
    for first in (True, False):
        HP.sgd_nesterov_(p, gg, b1, 0.1, 0.9, 1e-4, True, first)
        TP.sgd_nesterov_(p2, gg, b2, 0.1, 0.9, 1e-4, True, first)
    _close(p, p2, 1e-6)
    _close(b1, b2, 1e-6)


def test_data_kernels():
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    x, y = C.synth_images(4, 224, 224, 8, 3, 1000, 123, 0)
    assert x.shape == (4, 224, 224, 8) and y.shape == (4,)
    assert x[..., 3:].abs().max().item() == 0
    assert 0.5 < x[..., :3].float().std().item() < 1.5
    assert int(y.min()) >= 0 and int(y.max()) < 1000
    data = torch.randint(0, 256, (10, 32, 32, 3), dtype=torch.uint8, device=DEV)
    idx = torch.tensor([3, 1, 7], device=DEV)
    out = C.cifar_augment(data, idx, 3, False, 8, 0, 0, False)
    ref = (data[idx].float() / 255 - 0.5) / 0.5
    _close(out, ref, 1e-6)


def test_dgrad_addend_and_wgrad_accumulate():
    HP = _hp()
    torch.manual_seed(3)
    x = torch.randn(4, 28, 28, 128, device=DEV).to(torch.bfloat16)
    w = (torch.randn(256, 128, 3, 3, device=DEV) / 34).contiguous(memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, 128, True)
    wref = TP.conv_weight(w, torch.bfloat16, 128)
    dy = torch.randn(4, 14, 14, 256, device=DEV).to(torch.bfloat16)
    add = torch.randn(4, 28, 28, 128, device=DEV).to(torch.bfloat16)
    _close(HP.conv_dgrad(dy, wp, tuple(x.shape), 2, 1, add),
           TP.conv_dgrad(dy, wref, tuple(x.shape), 2, 1, add), 2e-2)
    base = torch.randn(256, 3, 3, 128, device=DEV)
    out = base.clone()
    HP.conv_wgrad(dy, x, tuple(wp[0].shape), 2, 1, out=out)
    _close(out, base + TP.conv_wgrad(dy, x, tuple(wref[0].shape), 2, 1), 2e-3)


def _grads_of(model):
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()
            if p.grad is not None}


@pytest.mark.parametrize("kind", ["bottleneck_identity", "bottleneck_proj_s2", "basic_proj_s2"])
def test_residual_block_hip_matches_torch_prims(kind):
    """One residual block (single autograd node: fused BN stats, dgrad with the
    residual-gradient addend, direct arena grads) on gfx950 kernels vs the same
    graph on torch primitives, same bf16 inputs.  (Whole deep nets at tiny
    batch amplify bf16 rounding differences chaotically, so numerics are
    pinned per block; the whole model is covered by the training test below.)"""
    from pytorch_multiprocessing_distributed_amd.models.resnet import BasicBlock, Bottleneck
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.flat import flatten_module
    torch.manual_seed(0)
    if kind == "bottleneck_identity":
        mk, cin, hw, args = Bottleneck, 256, 28, (256, 64, 1)
    elif kind == "bottleneck_proj_s2":
        mk, cin, hw, args = Bottleneck, 256, 28, (256, 128, 2)
    else:
        mk, cin, hw, args = BasicBlock, 64, 32, (64, 128, 2)
    base = mk(*args).to(DEV)
    x0 = torch.randn(8, hw, hw, cin, device=DEV).to(torch.bfloat16)
    dout = None
    res = {}
    for mode in ("hip", "torch"):
        blk = mk(*args).to(DEV)
        blk.load_state_dict(base.state_dict())
        flatten_module(blk)           # arena grads -> exercises the direct-write path
        x = x0.clone().requires_grad_(True)
        OF.force_torch_prims(mode == "torch")
        try:
            out = blk(x)
            if dout is None:
                dout = torch.randn_like(out)
            out.backward(dout)
            torch.cuda.synchronize()
        finally:
            OF.force_torch_prims(False)
        res[mode] = (out.float(), x.grad.float(),
                     {n: p.grad.float().clone() for n, p in blk.named_parameters()},
                     {k: v.clone() for k, v in blk.state_dict().items() if "running" in k})
    h, t = res["hip"], res["torch"]
    _close(h[0], t[0], 2e-2)
    _close_norm(h[1], t[1], 2e-2)
    for k, g in t[2].items():
        _close_norm(h[2][k], g, 2e-2)
    for k, v in t[3].items():
        _close(h[3][k], v, 1e-2)


def test_resnet50_trains_on_gpu():
    """End-to-end: the fused ResNet-50 (ImageNet stem) on the gfx950 kernels
    overfits a fixed batch -- loss must drop well below its initial value.

    lr 0.01: at lr >= 0.02 this batch-16 / 64x64 setup is unstable for ANY bf16
    implementation (bench/dbg_r50.py: the torch reference prims in bf16 and in
    fp32 spike and stall the same way), and first-step gradients of bf16 vs
    fp32 torch prims agree only to cosine ~0.2 here -- the net at random init is
    that sensitive to rounding, so convergence is the meaningful check."""
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    torch.manual_seed(0)
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
    x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
    y = torch.arange(16, device=DEV) % 10
    losses = []
    for _ in range(25):
        loss = OF.cross_entropy(m(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(map(lambda v: v == v, losses)), losses
    assert losses[-1] < 0.1 * losses[0], losses


@pytest.mark.parametrize("shape", [(64, 56, 256, 1, 1), (128, 28, 128, 3, 1), (256, 28, 512, 1, 2),
                                   (256, 28, 256, 3, 2), (512, 7, 2048, 1, 1)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
@pytest.mark.parametrize("two", [False, True])
@pytest.mark.parametrize("tile", [1, 2, 3, 6, 7, 8, 10, 11, 12])
def test_dgrad_fused_bn_reduce(shape, two, tile):
    """BN-backward reduce fused into the dgrad epilogue (one or two BN sets
    sharing the ReLU mask, with a residual addend) == dgrad then bn_bwd_reduce,
    on the 4-wave 128-row tiles and the 8-wave 256-row tiles."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    _C.conv_set_tile(tile)
    try:
        _dgrad_fused_bn_reduce(shape, two)
    finally:
        _C.conv_set_tile(0)


def _dgrad_fused_bn_reduce(shape, two):
    HP = _hp()
    torch.manual_seed(3)
    C, H, K, R, st = shape
    pad = R // 2
    N = _batch_for(H)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, R, R, device=DEV) / (C * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    yconv, _ = HP.conv_fwd(x, wp, st, pad, False)
    dy = torch.randn_like(yconv)
    add = torch.randn_like(x)
    sets = []
    for _ in range(2 if two else 1):
        yb = torch.randn_like(x)
        p = torch.stack([torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5,
                         torch.rand(C, device=DEV), torch.randn(C, device=DEV)]).contiguous()
        sets.append((yb, p))
    _, mask = HP.bn_apply(sets[0][0], sets[0][1], relu=True)
    dx_f, reds = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad, add, bnred=(mask, sets))
    dx = HP.conv_dgrad(dy, wp, tuple(x.shape), st, pad, add)
    # the fused-reduce dgrad stores its output (a BN site's dz) already gated by that
    # site's ReLU mask (bit k of byte i == element 8i+k), the form every consumer reads
    bits = (mask.view(-1, 1).int() >> torch.arange(8, device=DEV).view(1, 8)) & 1
    assert torch.equal(dx_f, dx * bits.view(dx.shape).to(dx.dtype))
    for (yb, p), r in zip(sets, reds):
        got = HP.stats_collapse(r).view(2, C)
        want = HP.stats_collapse(HP.bn_bwd_reduce(dx, mask, yb, p, True)).view(2, C)  # unfused
        _close(got, want, 1e-3)


def test_bn_stats_large_mean_shift():
    """|mean|/std = 100: the conv-epilogue statistics are
    taken about the BN's shift (previous batch mean, common.h bn_moments), so
    from step 2 on the variance matches an fp64 reference on the SAME bf16
    outputs; the unshifted first step shows the cancellation it avoids.  Then
    the fused conv->BN->ReLU path on the HIP kernels against torch.nn.BatchNorm2d
    in fp64 over three training steps (outputs and running statistics)."""
    import torch.nn as nn
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    HP = _hp()
    torch.manual_seed(5)
    N, H, C, K = 16, 15, 64, 64     # M = 3600: the last 128-row tile is partial

    def inp(seed):
        g = torch.Generator(device=DEV).manual_seed(seed)
        x = torch.randn(N, H, H, C, device=DEV, generator=g)
        x[..., 0] = 1.0
        return x.to(torch.bfloat16)
    from pytorch_multiprocessing_distributed_amd.models.resnet import Conv2d
    conv = Conv2d(C, K, 1, stride=1, padding=0).to(DEV)
    with torch.no_grad():
        conv.weight.normal_(0, (1.0 / (C - 1)) ** 0.5)
        conv.weight[:, 0] = 100.0
    x = inp(0)
    wp = HP.conv_weight(conv.weight, torch.bfloat16, C, False)
    y, _ = HP.conv_fwd(x, wp, 1, 0, False)
    t = y.double().reshape(-1, K)
    tvar = t.var(0, unbiased=False)
    shift = torch.zeros(K, device=DEV)
    errs = []
    for _ in range(2):
        _, st = HP.conv_fwd(x, wp, 1, 0, shift)
        p = HP.stats_finalize_local(st, t.shape[0], torch.ones(K, device=DEV), torch.zeros(K, device=DEV),
                                    0.0, shift=shift)
        errs.append(((1.0 / p[1].double() ** 2 - tvar).abs() / tvar).max().item())
    assert errs[1] < 1e-4 and errs[1] < errs[0] / 10, errs
    # the module path (fused BN finalize on the HIP kernels) vs nn.BatchNorm2d
    bn = nn.BatchNorm2d(K).to(DEV)
    ref_bn = nn.BatchNorm2d(K).to(DEV).double()
    for step in range(3):
        xs = inp(step + 1)
        out = OF.conv_bn_act(xs, conv, bn, relu=True)
        with torch.no_grad():
            yy, _ = HP.conv_fwd(xs, wp, 1, 0, False)       # the same bf16 conv output
            ref = torch.relu(ref_bn(yy.double().permute(0, 3, 1, 2))).permute(0, 2, 3, 1)
        if step >= 1:
            # bf16 output rounding only: relative L2 ~ 2^-9
            _close_norm(out.double(), ref, 5e-3)
    torch.testing.assert_close(bn.running_mean.double(), ref_bn.running_mean, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(bn.running_var.double(), ref_bn.running_var, rtol=5e-3, atol=1e-4)


@pytest.mark.parametrize("N,K,V", [(256, 2048, 1000), (32, 512, 10), (7, 64, 33)])
def test_linear_mfma(N, K, V):
    """Classifier GEMMs (kernels/linear.hip, bf16 MFMA with fp32 accumulation)
    against fp32 torch: forward (+bias), dgrad, and dW/db accumulated into
    existing targets (the grad-arena contract)."""
    HP = _hp()
    torch.manual_seed(3)
    x = torch.randn(N, K, device=DEV)
    w = torch.randn(V, K, device=DEV) / K ** 0.5
    b = torch.randn(V, device=DEV)
    dout = torch.randn(N, V, device=DEV)
    _close_norm(HP.linear_fwd(x, w, b), TP.linear_fwd(x, w, b), 1e-2)
    _close_norm(HP.linear_dgrad(dout, w), TP.linear_dgrad(dout, w), 1e-2)
    dw0, db0 = torch.randn(V, K, device=DEV), torch.randn(V, device=DEV)
    dw1, db1 = dw0.clone(), db0.clone()
    HP.linear_wgrad(dout, x, dw0, db0, True)
    TP.linear_wgrad(dout, x, dw1, db1, True)
    _close_norm(dw0, dw1, 1e-2)
    _close(db0, db1, 1e-5)


@pytest.mark.parametrize("N,K,V", [(256, 2048, 1000), (64, 512, 10)])
def test_linear_split_k_deterministic(N, K, V):
    """The split-K classifier combines its partial products in a fixed order
    (workspace slabs, no fp32 atomics): repeated products are bitwise equal,
    including dW accumulated into an existing target."""
    HP = _hp()
    torch.manual_seed(4)
    x = torch.randn(N, K, device=DEV)
    w = torch.randn(V, K, device=DEV) / K ** 0.5
    b = torch.randn(V, device=DEV)
    dout = torch.randn(N, V, device=DEV)
    f = [HP.linear_fwd(x, w, b) for _ in range(3)]
    d = [HP.linear_dgrad(dout, w) for _ in range(3)]
    base = torch.randn(V, K, device=DEV)
    g = []
    for _ in range(3):
        t = base.clone()
        HP.linear_wgrad(dout, x, t, None, True)
        g.append(t)
    for seq in (f, d, g):
        for t in seq[1:]:
            assert torch.equal(t, seq[0])


@pytest.mark.parametrize("n,off", [(1, 0), (15, 3), (4096, 0), (1000003, 5)])
def test_zero_kernel(n, off):
    """The framework's fill kernel (gradient-arena zero_grad, fresh accumulators):
    unaligned head, 16-B bulk and byte tail; bytes outside the view untouched."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    buf = torch.full((n + off + 7,), 7, dtype=torch.uint8, device=DEV)
    C.zero_(buf[off:off + n])
    torch.cuda.synchronize()
    assert int(buf[off:off + n].sum()) == 0
    assert bool((buf[:off] == 7).all()) and bool((buf[off + n:] == 7).all())



def test_tuning_table_roundtrip(tmp_path):
    """Per-shape tuning tables (ops/tuning.py): the tuned choices of a conv
    fwd/dgrad/wgrad export, survive clear + load from JSON, and an imported
    table is used as-is (no re-tuning: the entry count does not grow)."""
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    _C.conv_autotune_clear()
    _C.wgrad_autotune_clear()
    x = torch.randn(4, 14, 14, 64, device=DEV).to(torch.bfloat16)
    w = (torch.randn(128, 64, 3, 3, device=DEV) / 24).contiguous(memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, 64, True)
    y, _ = HP.conv_fwd(x, wp, 1, 1, False)
    HP.conv_dgrad(torch.randn_like(y), wp, tuple(x.shape), 1, 1)
    HP.conv_wgrad(torch.randn_like(y), x, (128, 3, 3, 64), 1, 1)
    torch.cuda.synchronize()
    tab = tuning.export_table()
    assert len(tab["conv"]) == 2 and len(tab["wgrad"]) == 1, tab
    path = str(tmp_path / "t.json")
    tuning.save(path)
    _C.conv_autotune_clear()
    _C.wgrad_autotune_clear()
    assert tuning.load(path) == 3
    assert tuning.export_table()["conv"] == tab["conv"]
    y2, _ = HP.conv_fwd(x, wp, 1, 1, False)
    torch.cuda.synchronize()
    assert _C.conv_autotune_entries() == 2 and torch.equal(y, y2)


def test_wgrad_deferred_grouped_reduce_matches_immediate():
    """Deferred split-K reductions (wgrad_set_defer + ONE grouped wgrad_flush launch, as a
    block backward issues them on the side stream) == each weight gradient reducing on its
    own, bit for bit (same fixed summation order), for a mix of split counts."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C as _C
    HP = _hp()
    torch.manual_seed(13)
    shapes = [(8, 56, 256, 64, 1, 1), (8, 28, 128, 128, 3, 1), (8, 14, 256, 1024, 1, 1), (4, 56, 64, 64, 3, 1)]
    ops = []
    for (N, H, C, K, R, st) in shapes:
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
        dy = torch.randn(N, P, P, K, device=DEV).to(torch.bfloat16)
        ops.append((dy, x, (K, R, R, C), st, pad))
    ref = [HP.conv_wgrad(dy, x, ks, st, pad) for (dy, x, ks, st, pad) in ops]
    outs = [torch.zeros_like(r) for r in ref]
    _C.wgrad_set_defer(True)
    try:
        for (dy, x, ks, st, pad), o in zip(ops, outs):
            HP.conv_wgrad(dy, x, ks, st, pad, out=o)
        assert _C.wgrad_pending() >= 3
    finally:
        _C.wgrad_set_defer(False)
    _C.wgrad_flush()
    assert _C.wgrad_pending() == 0
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_grouped_weight_images_exact(mode):
    """The grouped per-step weight-image refresh (runtime/weights.cpp -> the LDS-tiled
    transpose of conv_weight_prep_grouped_kernel) reproduces both layouts exactly:
    wk [K][R][S][Cp] and wkt [Cp][R][S][K], zero in the padded channels; shapes with K and C
    off the 64-tile grid, 1x1 / 3x3 / 7x7 taps."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    shapes = [(64, 3, 7, 8), (256, 64, 1, 64), (72, 40, 3, 48), (512, 512, 3, 512), (2048, 512, 1, 512),
              (100, 130, 3, 136)]
    g = torch.Generator(device="cpu").manual_seed(3)
    ws = [torch.randn(k, c, r, r, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
          for k, c, r, _ in shapes]
    imgs = C.WeightImages(ws, [cp for *_, cp in shapes], [True] * len(shapes))
    imgs.refresh(3)
    torch.cuda.synchronize()
    pre = [[t.clone() for t in imgs.get(i)] for i in range(len(shapes))]
    for w in ws:
        w.mul_(-0.5)
    imgs.refresh(mode)
    torch.cuda.synchronize()
    for i, ((k, c, r, cp), w) in enumerate(zip(shapes, ws)):
        ref = torch.zeros(k, r, r, cp, device=DEV, dtype=torch.bfloat16)
        ref[..., :c] = w.permute(0, 2, 3, 1).to(torch.bfloat16)
        wk, wkt = imgs.get(i)
        want_wk = ref if mode & 1 else pre[i][0]
        want_wkt = ref.permute(3, 1, 2, 0) if mode & 2 else pre[i][1]
        assert torch.equal(wk, want_wk), f"wk mismatch at {shapes[i]}"
        assert torch.equal(wkt, want_wkt), f"wkt mismatch at {shapes[i]}"


def test_grouped_fp8_weight_images_exact():
    """fp8 counterpart (quant_weight_fp8_grouped_kernel, tiled with an LDS transpose): e4m3 of
    w * scale (saturated, round-to-nearest-even like torch's cast) in both layouts, zero
    padded channels, and the weight's amax in its own slots."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    shapes = [(256, 64, 1, 64), (72, 40, 3, 48), (512, 512, 3, 512), (100, 130, 3, 136), (64, 8, 7, 8)]
    g = torch.Generator(device="cpu").manual_seed(5)
    ws = [torch.randn(k, c, r, r, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
          for k, c, r, _ in shapes]
    scales = [torch.full((1,), 37.0 * (i + 1), device=DEV) for i in range(len(shapes))]
    amaxes = [torch.zeros(64, device=DEV) for _ in shapes]
    imgs = C.Fp8WeightImages(ws, [cp for *_, cp in shapes], scales, amaxes, [i % 2 == 0 for i in range(len(shapes))])
    imgs.refresh()
    torch.cuda.synchronize()
    for i, ((k, c, r, cp), w) in enumerate(zip(shapes, ws)):
        ref = torch.zeros(k, r, r, cp, device=DEV)
        ref[..., :c] = w.permute(0, 2, 3, 1) * scales[i]
        ref = ref.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(imgs.get(i), ref), f"q mismatch at {shapes[i]}"
        qt = imgs.get_t(i)
        if i % 2 == 0:
            assert torch.equal(qt, ref.permute(3, 1, 2, 0)), f"qt mismatch at {shapes[i]}"
        else:
            assert qt is None
        assert amaxes[i].max().item() == w.abs().max().item()
