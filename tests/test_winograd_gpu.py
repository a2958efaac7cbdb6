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
