"""FP8 (OCP e4m3) path on gfx950 (BASELINE config 5): the scaled-MFMA operand
lane map (exact integer data), per-tensor quantisation with amax tracking,
and the fp8 implicit-GEMM forward conv against an fp32 conv of the same
dequantised operands."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _C():
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    return C


def _e4m3(t):
    return t.to(torch.float8_e4m3fn).view(torch.uint8)


def test_scaled_mfma_16x16x128_lane_map():
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-3, 4, (16, 128), generator=g).float()
    Bt = torch.randint(-3, 4, (16, 128), generator=g).float()
    Bt[3, 77] = 7.0       # asymmetric markers
    A[5, 120] = -6.0
    got = _C().fp8_mfma_probe(_e4m3(A).to(DEV), _e4m3(Bt).to(DEV)).cpu()
    torch.testing.assert_close(got, A @ Bt.T, rtol=0, atol=0)


def test_quant_bf16_fp8_matches_torch_and_tracks_amax():
    C = _C()
    x = (torch.randn(4096, device=DEV) * 3).to(torch.bfloat16)
    scale = torch.tensor([2.0], device=DEV)
    amax = torch.zeros(64, device=DEV)
    q = C.quant_bf16_fp8(x, scale, amax)
    want = _e4m3((x.float() * 2.0).clamp(-448, 448))
    assert torch.equal(q, want)
    assert amax.max().item() == x.float().abs().max().item()
    back = C.dequant_fp8(q, torch.tensor([0.5], device=DEV))
    torch.testing.assert_close(back, x.float(), rtol=0.07, atol=1e-2)
    # out-of-range values saturate to +-448 (the hardware convert alone would give NaN)
    big = torch.tensor([1000.0, -1000.0, 448.0, 500.0] * 4, device=DEV).to(torch.bfloat16)
    qb = C.quant_bf16_fp8(big, torch.tensor([1.0], device=DEV), None)
    vals = C.dequant_fp8(qb, None)
    assert torch.equal(vals, torch.tensor([448.0, -448.0, 448.0, 448.0] * 4, device=DEV))


def test_bn_apply_fp8_copy_saturates():
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    y = (torch.randn(8, 4, 4, 64, device=DEV) * 4).to(torch.bfloat16)
    p = torch.stack([torch.zeros(64, device=DEV), torch.ones(64, device=DEV),
                     torch.ones(64, device=DEV), torch.zeros(64, device=DEV)]).contiguous()
    amax = torch.zeros(64, device=DEV)
    out, mask, q = HP.bn_apply(y, p, relu=True, fp8=(torch.tensor([100.0], device=DEV), amax))
    d = _C().dequant_fp8(q, torch.tensor([0.01], device=DEV))
    assert torch.isfinite(d).all()
    want = (out.float() * 100).clamp(max=448) / 100
    torch.testing.assert_close(d, want, rtol=0.07, atol=1e-3)
    assert amax.max().item() == out.float().max().item()


@pytest.mark.parametrize("shape", [(16, 56, 64, 7, 2), (64, 56, 64, 1, 1), (64, 56, 64, 3, 1),
                                   (256, 56, 128, 1, 1), (128, 28, 128, 3, 2), (512, 7, 2048, 1, 1),
                                   (256, 14, 256, 3, 1)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
@pytest.mark.parametrize("impl", [0, 1], ids=["fp8kernel", "igemm"])
def test_conv_fp8_fwd(shape, impl):
    """conv_fp8_fwd on both implementations: conv_fp8_fwd_kernel (fp8.hip) and the
    implicit-GEMM kernel's e4m3 path (conv_igemm_kernel<..., F8>, PMD_FP8_FWD_IMPL=1)."""
    C = _C()
    C.conv_fp8_fwd_set_impl(impl)
    try:
        _conv_fp8_fwd_case(C, shape)
    finally:
        C.conv_fp8_fwd_set_impl(-1)


def _conv_fp8_fwd_case(C, shape):
    torch.manual_seed(0)
    Cin, H, K, R, st = shape
    pad = R // 2
    N = 2 if H >= 56 else 4
    x = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, Cin, R, R, device=DEV) / (Cin * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    sx = torch.tensor([448.0 / x.float().abs().max().item()], device=DEV)
    sw = torch.tensor([448.0 / w.abs().max().item()], device=DEV)
    amax_x = torch.zeros(64, device=DEV)
    amax_w = torch.zeros(64, device=DEV)
    xq = C.quant_bf16_fp8(x, sx, amax_x)
    wq = C.quant_weight_fp8(w, Cin, sw, amax_w)
    assert abs(amax_w.max().item() - w.abs().max().item()) < 1e-7
    y, stats = C.conv_fp8_fwd(xq, wq, sx, sw, st, pad, True, None)
    # reference: fp32 conv of the dequantised operands
    xd = C.dequant_fp8(xq, 1.0 / sx).permute(0, 3, 1, 2)
    wd = C.dequant_fp8(wq, 1.0 / sw).permute(0, 3, 1, 2)
    yr = F.conv2d(xd, wd, stride=st, padding=pad).permute(0, 2, 3, 1)
    err = (y.float() - yr).abs().max() / yr.abs().max()
    assert err < 1e-2, err
    # relative L2 at the bf16 output-rounding floor (same oracle contract as the bf16 convs,
    # tests/test_kernels_gpu.py CONV_REL_L2)
    rel2 = (y.float() - yr).norm() / yr.norm()
    assert rel2 < 5e-3, rel2
    s = stats.sum(0)
    yb = y.float().reshape(-1, K)
    torch.testing.assert_close(s[0], yb.sum(0), rtol=1e-3, atol=1e-2)
    # fp8 vs the bf16 conv of the ORIGINAL operands: quantisation error only
    y16 = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), stride=st, padding=pad).permute(0, 2, 3, 1)
    rel = (y.float() - y16).norm() / y16.norm()
    assert rel < 0.1, rel


def test_quant_bf16_bf8_e5m2_matches_torch():
    """The e5m2 (bf8) gradient quantiser: bytes equal torch's float8_e5m2 cast of the
    scaled value, out-of-range values saturate to +-57344, dequant round-trips."""
    C = _C()
    x = (torch.randn(4096, device=DEV) * 30).to(torch.bfloat16)
    scale = torch.tensor([4.0], device=DEV)
    amax = torch.zeros(64, device=DEV)
    q = C.quant_bf16_fp8(x, scale, amax, bf8=True)
    want = (x.float() * 4.0).to(torch.float8_e5m2).view(torch.uint8)
    assert torch.equal(q, want)
    assert amax.max().item() == x.float().abs().max().item()
    back = C.dequant_fp8(q, torch.tensor([0.25], device=DEV), bf8=True)
    torch.testing.assert_close(back, x.float(), rtol=0.13, atol=1e-3)
    big = torch.tensor([1e5, -1e5, 57344.0, 6e4] * 4, device=DEV).to(torch.bfloat16)
    vals = C.dequant_fp8(C.quant_bf16_fp8(big, torch.tensor([1.0], device=DEV), None, bf8=True), None, bf8=True)
    assert torch.equal(vals, torch.tensor([57344.0, -57344.0, 57344.0, 57344.0] * 4, device=DEV))


@pytest.mark.parametrize("shape", [(64, 56, 64, 3, 1), (128, 28, 128, 3, 1), (256, 14, 256, 3, 1),
                                   (512, 7, 512, 3, 1), (128, 56, 128, 3, 2), (256, 14, 1024, 1, 1),
                                   (64, 56, 256, 1, 1), (1024, 14, 512, 1, 2)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_wgrad_fp8(shape):
    """e5m2 dY x e4m3 X weight gradient on the scaled 16x16x128 MFMA (transposed
    ds_read_b64_tr_b8 fragments, split-K + ordered reduce) == the fp32 weight gradient
    of the same dequantised operands; accumulates into ``out``."""
    C = _C()
    torch.manual_seed(1)
    Cin, H, K, R, st = shape
    pad = R // 2
    N = 2 if H >= 56 else (4 if H >= 28 else 16)
    x = torch.randn(N, H, H, Cin, device=DEV).relu().to(torch.bfloat16)
    P = (H + 2 * pad - R) // st + 1
    dy = (torch.randn(N, P, P, K, device=DEV) * 1e-3).to(torch.bfloat16)
    sx = torch.tensor([448.0 / x.float().abs().max().item()], device=DEV)
    sdy = torch.tensor([57344.0 / 4 / dy.float().abs().max().item()], device=DEV)
    xq = C.quant_bf16_fp8(x, sx, None)
    dyq = C.quant_bf16_fp8(dy, sdy, None, bf8=True)
    base = torch.randn(K, R, R, Cin, device=DEV)
    dw = C.conv_wgrad_fp8(dyq, xq, sdy, sx, R, R, st, pad, base.clone())
    xd = C.dequant_fp8(xq, 1.0 / sx).permute(0, 3, 1, 2)
    dyd = C.dequant_fp8(dyq, 1.0 / sdy, bf8=True).permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xd.double(), (K, Cin, R, R), dyd.double(), stride=st,
                                      padding=pad).permute(0, 2, 3, 1).float()
    err = ((dw - base) - ref).abs().max() / ref.abs().max()
    assert err < 1e-4, err


@pytest.mark.parametrize("shape", [(64, 56, 64, 3, 1), (64, 56, 256, 1, 1), (256, 56, 64, 1, 1),
                                   (128, 28, 128, 3, 1), (128, 56, 128, 3, 2), (256, 14, 256, 3, 1),
                                   (1024, 14, 256, 1, 1), (256, 14, 1024, 1, 1), (512, 28, 1024, 1, 2),
                                   (512, 7, 512, 3, 1)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_dgrad_fp8(shape):
    """e5m2 dY x e4m3 transposed weight image on the scaled MFMA inside the implicit-GEMM
    dgrad kernel == the fp32 data gradient of the same dequantised operands; with an
    addend and the fused BN-backward reduce, == the unfused bf16 epilogue ops."""
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    C = _C()
    torch.manual_seed(2)
    Cin, H, K, R, st = shape
    pad = R // 2
    N = 2 if H >= 56 else (4 if H >= 28 else 8)
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, P, P, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, Cin, R, R, device=DEV) / (Cin * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    sw = torch.tensor([448.0 / w.abs().max().item()], device=DEV)
    sdy = torch.tensor([57344.0 / 4 / dy.float().abs().max().item()], device=DEV)
    wq, wtq = C.quant_weight_fp8_t(w, Cin, sw, None)
    dyq = C.quant_bf16_fp8(dy, sdy, None, bf8=True)
    # the transposed image is the forward image with K and C swapped
    assert torch.equal(wtq, wq.permute(3, 1, 2, 0))
    dx = HP.conv_dgrad_fp8(dyq, sdy, wtq, sw, (N, H, H, Cin), st, pad)
    wd = C.dequant_fp8(wq, 1.0 / sw).permute(0, 3, 1, 2).double()
    dyd = C.dequant_fp8(dyq, 1.0 / sdy, bf8=True).permute(0, 3, 1, 2).double()
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), wd, dyd, stride=st, padding=pad).permute(0, 2, 3, 1)
    err = (dx.double() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, err
    rel2 = (dx.double() - ref).norm() / ref.norm()
    assert rel2 < 5e-3, rel2
    # a weight image with one input channel zeroed must fail that bound (negative control
    # of the oracle at the smallest reduction under test as well as the largest)
    if Cin >= 256:
        wbad = w.clone()
        wbad[:, 7] = 0.0
        _, wtq_bad = C.quant_weight_fp8_t(wbad, Cin, sw, None)
        dxb = HP.conv_dgrad_fp8(dyq, sdy, wtq_bad, sw, (N, H, H, Cin), st, pad)
        assert (dxb.double() - ref).norm() / ref.norm() > 5e-3
    # fused epilogue: addend + BN-backward reduce over one BN input
    add = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    yb = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    p = torch.stack([torch.randn(Cin, device=DEV) * 0.1, torch.rand(Cin, device=DEV) + 0.5,
                     torch.rand(Cin, device=DEV), torch.randn(Cin, device=DEV)]).contiguous()
    _, mask = HP.bn_apply(yb, p, relu=True)
    dx_f, reds = HP.conv_dgrad_fp8(dyq, sdy, wtq, sw, (N, H, H, Cin), st, pad, add, bnred=(mask, [(yb, p)]))
    bits = (mask.view(-1, 1).int() >> torch.arange(8, device=DEV).view(1, 8)) & 1
    want = ((dx.float() + add.float()) * bits.view(dx.shape).float())
    torch.testing.assert_close(dx_f.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())
    got = HP.stats_collapse(reds[0]).view(2, Cin)
    exp = HP.stats_collapse(HP.bn_bwd_reduce(dx_f, mask, yb, p, True)).view(2, Cin)
    torch.testing.assert_close(got, exp, rtol=1e-3, atol=1e-3 * exp.abs().max().item())


def test_resnet50_fp8_trains():
    """Config 5 path: ResNet-50 with every block conv in fp8 (e4m3 forwards, e5m2 x e4m3
    data and weight gradients, delayed scaling) converges on a fixed batch like the bf16 model, and its first-step
    loss matches bf16 to quantisation accuracy."""
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
    C = _C()
    x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
    y = torch.arange(16, device=DEV) % 10
    first = {}
    for mode in ("bf16", "fp8"):
        torch.manual_seed(0)
        m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
        f8 = Fp8Scaling(DEV) if mode == "fp8" else None
        OF.set_fp8(f8)
        try:
            opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
            losses = []
            for _ in range(25):
                loss = OF.cross_entropy(m(x), y)
                opt.zero_grad()
                loss.backward()
                opt.step()
                losses.append(loss.item())
        finally:
            OF.set_fp8(None)
        first[mode] = losses[0]
        assert all(v == v for v in losses), losses
        assert losses[-1] < 0.1 * losses[0], (mode, losses)
        if f8 is not None:
            # a weight site per fp8-eligible conv (default policy "all" with the fp8
            # gradients and PMD_FP8_MIN_KG=0: every one of ResNet-50's 52 block convs --
            # 16 blocks x 3 + 4 projection shortcuts; the stem stays bf16) plus the
            # activation sites of their inputs
            n_elig = sum(1 for mod in m.modules() if getattr(mod, "weight", None) is not None
                         and mod.weight.dim() == 4 and mod is not m.conv1
                         and OF.fp8_eligible(mod, mod.weight.shape[1]))
            if OF.FP8_CONVS == "all" and OF.FP8_MIN_KG == 0:
                assert n_elig == 52, n_elig
            assert len(f8.sites) > n_elig, (n_elig, len(f8.sites))
            if OF.FP8_WGRAD:
                # the e5m2 dY sites of the fp8 weight / data gradients: the gradient path ran
                assert f8.grads is not None and len(f8.grads.sites) > 0
            assert f8.steps == 24                              # first update() precedes any site
            n = len(f8.sites)
            assert torch.isfinite(f8.scale[:n]).all() and (f8.scale[:n] > 0).all()
    # At 64 px / batch 16 the random-init network is numerically chaotic (layer-4 BN
    # over 64 values per channel): any fp8 quantisation pattern moves the first
    # logits by rel-L2 ~0.45 vs bf16 and the first loss by a few percent
    # (bench/fp8_probe.py -> profiles/fp8_probe_r02.txt: 2.4% with every eligible
    # conv in fp8, 8.0% with the 3x3 convs only, whose logits are the closer ones)
    assert abs(first["fp8"] - first["bf16"]) < 0.12 * first["bf16"], first


def test_grouped_fp8_weight_images_match_per_conv():
    """Fp8WeightSet (one grouped launch for every block conv) == quant_weight_fp8
    per conv: identical e4m3 bytes and amax, for every ResNet-50 block conv."""
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.models.resnet import Conv2d
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
    C = _C()
    torch.manual_seed(0)
    m = ResNet50(num_classes=1000, stem="imagenet").to(DEV)
    convs = [mod for mod in m.modules() if isinstance(mod, Conv2d) and mod is not m.conv1]
    f8 = Fp8Scaling(DEV)
    ws = OF.Fp8WeightSet([(c, c.in_channels) for c in convs], f8)
    ws.refresh()
    torch.cuda.synchronize()
    for c in convs:
        sw, aw = f8.site(("w", id(c)))
        ref_amax = torch.zeros(64, device=DEV)
        ref = C.quant_weight_fp8(c.weight.detach(), c.in_channels, sw, ref_amax)
        got = ws.lookup(c, c.in_channels)
        assert torch.equal(got, ref)
        assert torch.equal(aw.max(), ref_amax.max())


def test_fp8_update_scales_native_matches_torch():
    """Fp8Scaling.update() (one native launch) == the torch formula: scale = 448 /
    max over the 64 amax slots where one was observed, unchanged elsewhere, slots
    cleared; sites past n untouched."""
    from pytorch_multiprocessing_distributed_amd.ops.fp8 import E4M3_MAX
    C = _C()
    torch.manual_seed(0)
    cap, n = 40, 37
    amax = torch.rand(cap, 64, device=DEV) * 10
    amax[5].zero_()                          # no observation: keep its scale
    scale = torch.rand(cap, device=DEV) + 0.5
    a_ref = amax[:n].amax(dim=1)
    s_ref = torch.where(a_ref > 0, E4M3_MAX / a_ref.clamp_min(1e-12), scale[:n])
    tail_a, tail_s = amax[n:].clone(), scale[n:].clone()
    C.fp8_update_scales(amax, scale, n, E4M3_MAX)
    torch.cuda.synchronize()
    assert torch.allclose(scale[:n], s_ref, rtol=1e-6, atol=0)
    assert torch.count_nonzero(amax[:n]).item() == 0
    assert torch.equal(amax[n:], tail_a) and torch.equal(scale[n:], tail_s)


def test_basicblock_resnet_fp8_step():
    """fp8 in BasicBlock networks (ResNet-34, ImageNet stem): every block conv is 3x3,
    so block outputs carry e4m3 copies to the next block; a few SGD steps stay finite
    and reduce the loss on a fixed batch, and fp8 sites exist for the 3x3 convs."""
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
    C = _C()
    x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
    y = torch.arange(16, device=DEV) % 10
    torch.manual_seed(0)
    m = build_model("resnet34", num_classes=10, stem="imagenet").to(DEV)
    f8 = Fp8Scaling(DEV)
    OF.set_fp8(f8)
    try:
        opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
        losses = []
        for _ in range(15):
            loss = OF.cross_entropy(m(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
    finally:
        OF.set_fp8(None)
    assert all(v == v for v in losses), losses
    assert losses[-1] < 0.5 * losses[0], losses
    n33 = sum(1 for mod in m.modules() if getattr(mod, "weight", None) is not None
              and mod.weight.dim() == 4 and mod is not m.conv1 and tuple(mod.weight.shape[2:]) == (3, 3))
    assert n33 == 32 and len(f8.sites) >= n33, (n33, len(f8.sites))
