"""gfx950 Winograd F(2x2,3x3) path (csrc/kernels/winograd.hip + the 16 GEMMs on conv_igemm)
against the PyTorch fp32 conv of the same bf16 operands: forward with the fused
BN statistics, dgrad, dispatch through hip_prims, and a ResNet step."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_multiprocessing_distributed_amd.ops import winograd as WG

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("t,c,k", [(3136, 64, 64), (1000, 128, 256), (96, 512, 512), (17, 64, 32)])
def test_winograd_gemm_native(t, c, k):
    """The 16 transformed-domain GEMMs on the implicit-GEMM MFMA kernel vs fp32 bmm of
    the same bf16 operands (bf16 output: one rounding, rel-L2 < 1e-2)."""
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    torch.manual_seed(0)
    V = torch.randn(16, t, c, device=DEV).to(torch.bfloat16)
    U = (torch.randn(16, k, c, device=DEV) / c ** 0.5).to(torch.bfloat16)
    M = C.winograd_gemm(V, U)
    ref = torch.bmm(V.float(), U.float().transpose(1, 2))
    assert M.shape == (16, t, k) and M.dtype == torch.bfloat16
    assert _rel(M, ref) < 1e-2


@pytest.mark.parametrize("n,h,c,k", [(4, 56, 64, 64), (4, 28, 128, 128), (8, 14, 256, 256),
                                     (8, 7, 512, 512), (2, 9, 64, 32)])
def test_winograd_fwd_stats(n, h, c, k):
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    torch.manual_seed(0)
    x = torch.randn(n, h, h, c, device=DEV).to(torch.bfloat16)
    w = (torch.randn(k, c, 3, 3, device=DEV) / (9 * c) ** 0.5).contiguous(memory_format=torch.channels_last)
    wk = HP.conv_weight(w, torch.bfloat16, c, True)[0]
    y, st = WG.conv_fwd(x, wk, True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wk.float().permute(0, 3, 1, 2), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 2e-2
    yf = y.float().reshape(-1, k)
    s = st.sum(0)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-3, atol=1e-2 * n * h * h ** 0.5)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("n,h,c,k", [(4, 56, 64, 64), (8, 14, 256, 128), (2, 7, 64, 64)])
def test_winograd_dgrad(n, h, c, k):
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    torch.manual_seed(1)
    dy = torch.randn(n, h, h, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(k, c, 3, 3, device=DEV) / (9 * c) ** 0.5).contiguous(memory_format=torch.channels_last)
    wk = HP.conv_weight(w, torch.bfloat16, c, True)[0]
    dx = WG.conv_dgrad(dy, wk, (n, h, h, c))
    ref = torch.nn.grad.conv2d_input((n, c, h, h), wk.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 2e-2


# the fused forward (one kernel: input transform -> LDS -> 16 MFMA GEMMs -> output transform + stats),
# at every stride-1 3x3 shape family of ResNet-50 / ResNet-18 (7x7 and odd sizes: partial 2x2 tiles)
FUSED_SHAPES = [(4, 56, 64, 64), (4, 28, 128, 128), (8, 14, 256, 256), (8, 7, 512, 512), (3, 9, 64, 128),
                (2, 32, 64, 64), (4, 16, 128, 128), (16, 4, 512, 512), (1, 5, 192, 64)]


@pytest.mark.parametrize("n,h,c,k", FUSED_SHAPES)
@pytest.mark.parametrize("shifted", [False, True])
def test_winograd_fused_fwd_vs_fp32(n, h, c, k, shifted):
    """Output against the fp32 conv of the same bf16 operands, and the statistics against
    the fp32 sums of the kernel's own bf16 outputs about the shift (the conv_fwd contract)."""
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    torch.manual_seed(n * h + c + k)
    x = torch.randn(n, h, h, c, device=DEV).to(torch.bfloat16)
    w = (torch.randn(k, c, 3, 3, device=DEV) / (9 * c) ** 0.5).contiguous(memory_format=torch.channels_last)
    wk = HP.conv_weight(w, torch.bfloat16, c, True)[0]
    shift = (torch.randn(k, device=DEV) * 0.1) if shifted else None
    y, st = WG.conv_fwd_fused(x, wk, True, None, shift)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wk.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert y.shape == ref.shape and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 1e-2, _rel(y, ref)
    yf = y.float().reshape(-1, k) - (shift if shifted else 0.0)
    s = st.sum(0)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=1e-4, atol=1e-3 * yf.shape[0] ** 0.5)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
    y2, _ = WG.conv_fwd_fused(x, wk, False)
    assert torch.equal(y2, y)


def test_winograd_fused_is_a_conv_candidate():
    """Candidate 14 through the production conv entry (hip_prims.conv_fwd with the forced tile
    policy): same output and statistics as the explicit fused API, also in the deterministic
    statistics mode (bit-identical across two calls)."""
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    torch.manual_seed(5)
    x = torch.randn(8, 14, 14, 256, device=DEV).to(torch.bfloat16)
    w = (torch.randn(256, 256, 3, 3, device=DEV) / 48.0).contiguous(memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, 256, True)
    y_ref, st_ref = WG.conv_fwd_fused(x, wp[0], True)
    C.conv_set_tile(14)
    try:
        y, st = HP.conv_fwd(x, wp, 1, 1, True)
        assert torch.equal(y, y_ref)
        torch.testing.assert_close(st.sum(0), st_ref.sum(0), rtol=1e-5, atol=1e-2)
        OF.set_deterministic(True)
        try:
            a = HP.conv_fwd(x, wp, 1, 1, True)[1].sum(0)
            b = HP.conv_fwd(x, wp, 1, 1, True)[1].sum(0)
            assert torch.equal(a, b)
        finally:
            OF.set_deterministic(False)
    finally:
        C.conv_set_tile(0)

