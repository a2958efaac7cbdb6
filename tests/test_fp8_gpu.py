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
    amax = torch.zeros(1, device=DEV)
    q = C.quant_bf16_fp8(x, scale, amax)
    want = _e4m3((x.float() * 2.0).clamp(-448, 448))
    assert torch.equal(q, want)
    assert amax.item() == x.float().abs().max().item()
    back = C.dequant_fp8(q, torch.tensor([0.5], device=DEV))
    torch.testing.assert_close(back, x.float(), rtol=0.07, atol=1e-2)


@pytest.mark.parametrize("shape", [(16, 56, 64, 7, 2), (64, 56, 64, 1, 1), (64, 56, 64, 3, 1),
                                   (256, 56, 128, 1, 1), (128, 28, 128, 3, 2), (512, 7, 2048, 1, 1),
                                   (256, 14, 256, 3, 1)],
                         ids=lambda s: "C%d_H%d_K%d_R%d_s%d" % s)
def test_conv_fp8_fwd(shape):
    C = _C()
    torch.manual_seed(0)
    Cin, H, K, R, st = shape
    pad = R // 2
    N = 2 if H >= 56 else 4
    x = torch.randn(N, H, H, Cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, Cin, R, R, device=DEV) / (Cin * R * R) ** 0.5).contiguous(
        memory_format=torch.channels_last)
    sx = torch.tensor([448.0 / x.float().abs().max().item()], device=DEV)
    sw = torch.tensor([448.0 / w.abs().max().item()], device=DEV)
    amax_x = torch.zeros(1, device=DEV)
    amax_w = torch.zeros(1, device=DEV)
    xq = C.quant_bf16_fp8(x, sx, amax_x)
    wq = C.quant_weight_fp8(w, Cin, sw, amax_w)
    assert abs(amax_w.item() - w.abs().max().item()) < 1e-7
    descale = 1.0 / (sx * sw)
    y, stats = C.conv_fp8_fwd(xq, wq, descale, st, pad, True, None)
    # reference: fp32 conv of the dequantised operands
    xd = C.dequant_fp8(xq, 1.0 / sx).permute(0, 3, 1, 2)
    wd = C.dequant_fp8(wq, 1.0 / sw).permute(0, 3, 1, 2)
    yr = F.conv2d(xd, wd, stride=st, padding=pad).permute(0, 2, 3, 1)
    err = (y.float() - yr).abs().max() / yr.abs().max()
    assert err < 1e-2, err
    s = stats.sum(0)
    yb = y.float().reshape(-1, K)
    torch.testing.assert_close(s[0], yb.sum(0), rtol=1e-3, atol=1e-2)
    # fp8 vs the bf16 conv of the ORIGINAL operands: quantisation error only
    y16 = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), stride=st, padding=pad).permute(0, 2, 3, 1)
    rel = (y.float() - y16).norm() / y16.norm()
    assert rel < 0.1, rel
