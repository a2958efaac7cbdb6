"""Winograd F(2x2,3x3) transform algebra (ops/winograd.py::conv_ref, the CPU
reference of csrc/kernels/winograd.hip) against PyTorch fp32 conv2d: forward
and the flipped-filter dgrad, even and odd spatial sizes."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_multiprocessing_distributed_amd.ops import winograd as WG


@pytest.mark.parametrize("n,h,w,c,k", [(2, 8, 8, 8, 16), (1, 7, 5, 16, 8), (3, 4, 6, 8, 8), (1, 1, 1, 8, 8)])
def test_winograd_ref_fwd(n, h, w, c, k):
    torch.manual_seed(0)
    x = torch.randn(n, h, w, c, dtype=torch.float64)
    wk = torch.randn(k, 3, 3, c, dtype=torch.float64)
    y = WG.conv_ref(x, wk)
    ref = F.conv2d(x.permute(0, 3, 1, 2), wk.permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,h,w,c,k", [(2, 8, 8, 8, 16), (1, 7, 5, 16, 8)])
def test_winograd_ref_dgrad(n, h, w, c, k):
    torch.manual_seed(1)
    dy = torch.randn(n, h, w, k, dtype=torch.float64)
    wk = torch.randn(k, 3, 3, c, dtype=torch.float64)
    dx = WG.conv_ref(dy, wk, flip=True)
    ref = torch.nn.grad.conv2d_input((n, c, h, w), wk.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2),
                                     padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(dx.double(), ref, rtol=1e-5, atol=1e-5)


def test_winograd_eligibility():
    assert WG.eligible((64, 3, 3, 64), 1, 1)
    assert WG.eligible((512, 3, 3, 512), 1, 1, 512)
    assert not WG.eligible((64, 3, 3, 64), 2, 1)       # strided: implicit GEMM
    assert not WG.eligible((64, 1, 1, 64), 1, 0)       # 1x1
    assert not WG.eligible((64, 3, 3, 24), 1, 1)       # 3 chunks: grid contract
    assert not WG.eligible((64, 3, 3, 64), 1, 1, 32)   # channel mismatch
