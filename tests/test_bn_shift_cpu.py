"""BatchNorm statistics about a per-channel shift (csrc/kernels/common.h
bn_moments; ops/functional.py bn_stat_shift) on the PyTorch reference
primitives: with |mean|/std = 100 the plain fp32 E[y^2] - E[y]^2 loses
(mean/std)^2 = 1e4 of its relative precision; accumulated about the previous
step's batch mean the variance is exact to fp32 rounding from step 2 on, and
the training-mode BN matches torch.nn.BatchNorm2d (fp64) step for step."""
import torch
import torch.nn as nn

from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.ops import torch_prims as TP


def _offset_conv(C=16, K=8, offset=100.0):
    """1x1 conv whose outputs have mean ~offset and std ~1 in every channel
    (input channel 0 is constant 1, its weight column = offset)."""
    conv = nn.Conv2d(C, K, 1, bias=False)
    with torch.no_grad():
        conv.weight.normal_(0, (1.0 / (C - 1)) ** 0.5)
        conv.weight[:, 0] = offset
    return conv


def _input(N=16, C=16, H=8, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, H, C, generator=g)
    x[..., 0] = 1.0
    return x


def test_stats_about_shift_exact():
    conv = _offset_conv()
    x = _input()
    wk = TP.conv_weight(conv.weight, torch.float32, 16)
    y, _ = TP.conv_fwd(x, wk, 1, 0, False)
    truth = y.double().reshape(-1, 8)
    tvar, tmean = truth.var(0, unbiased=False), truth.mean(0)
    shift = torch.zeros(8)
    n = truth.shape[0]
    errs = []
    for _ in range(2):
        _, st = TP.conv_fwd(x, wk, 1, 0, shift)
        p = TP.stats_finalize_local(st, n, torch.ones(8), torch.zeros(8), 0.0, shift=shift)
        var = 1.0 / p[1].double() ** 2
        errs.append(((var - tvar).abs() / tvar).max().item())
        assert ((p[0].double() - tmean).abs() / tvar.sqrt()).max() < 1e-4
        assert torch.allclose(shift.double(), p[0].double())     # next step's shift = batch mean
    # step 1 (shift 0) pays the cancellation, step 2 (shift = mean) does not
    assert errs[1] < 1e-5, errs
    assert errs[1] < errs[0] / 10, errs


def test_training_bn_matches_torch_at_large_mean():
    torch.manual_seed(0)
    conv = _offset_conv()
    bn = nn.BatchNorm2d(8)
    ref_bn = nn.BatchNorm2d(8).double()
    conv.train()
    bn.train()
    ref_bn.train()
    for step in range(3):
        x = _input(seed=step)
        out = OF.conv_bn_act(x, conv, bn, relu=False)                 # NHWC, torch prims (CPU)
        with torch.no_grad():
            y = conv.double()(x.permute(0, 3, 1, 2).double())
            conv.float()
            ref = ref_bn(y).permute(0, 2, 3, 1)
        if step >= 1:   # the shift has converged to the batch mean (previous step's)
            rel = ((out.double() - ref).norm() / ref.norm()).item()
            assert rel < 1e-4, (step, rel)
    assert torch.allclose(bn.running_mean.double(), ref_bn.running_mean, rtol=1e-6, atol=1e-5)
    assert torch.allclose(bn.running_var.double(), ref_bn.running_var, rtol=2e-4)
