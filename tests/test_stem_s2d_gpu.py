"""gfx950 space-to-depth stem conv (csrc/kernels/stem.hip + conv_fwd_hw +
cropped wgrad) against the direct 7x7/s2 implicit-GEMM path and the fp32
PyTorch conv: output, BN statistics, weight gradient (returned and arena-
accumulated), and a full ResNet-50 step with the s2d stem on vs off."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("n,h", [(2, 224), (4, 64), (3, 32)])
def test_s2d_stem_conv_matches_direct(n, h):
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    torch.manual_seed(0)
    from pytorch_multiprocessing_distributed_amd.models.resnet import Conv2d
    conv = Conv2d(3, 64, 7, stride=2, padding=3).to(DEV)
    x, _ = C.synth_images(n, h, h, 8, 3, 10, 3, 0)
    assert OF._s2d_stem_ok(x, conv)
    outs = {}
    for flag in (True, False):
        OF.set_s2d_stem(flag)
        try:
            conv.weight.grad = None
            w = conv.weight
            y, st = OF.conv(x, conv, want_stats=True)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(5)).to(y.dtype)
            (y.float() * g.float()).sum().backward()
            torch.cuda.synchronize()
            from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
            outs[flag] = (y.clone(), HP.stats_collapse(st).view(2, -1).clone(), w.grad.clone())
        finally:
            OF.set_s2d_stem(True)
    (y1, s1, g1), (y0, s0, g0) = outs[True], outs[False]
    ref = F.conv2d(x[..., :3].float().permute(0, 3, 1, 2), conv.weight.detach().to(torch.bfloat16).float(),
                   stride=2, padding=3).permute(0, 2, 3, 1)
    assert y1.shape == y0.shape == ref.shape
    assert _rel(y1, ref) < 1e-2 and _rel(y0, ref) < 1e-2
    assert _rel(s1, s0) < 1e-2
    assert _rel(g1, g0) < 1e-2


def test_s2d_stem_resnet50_step():
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    x, y = C.synth_images(4, 64, 64, 8, 3, 1000, 7, 0)
    res = {}
    for flag in (True, False):
        OF.set_s2d_stem(flag)
        try:
            torch.manual_seed(0)
            m = ResNet50(num_classes=1000, stem="imagenet").to(DEV)
            loss = OF.cross_entropy(m(x), y)
            loss.backward()
            torch.cuda.synchronize()
            res[flag] = (loss.item(), m.conv1.weight.grad.clone())
        finally:
            OF.set_s2d_stem(True)
    assert abs(res[True][0] - res[False][0]) < 1e-2 * max(1.0, abs(res[False][0]))
    assert _rel(res[True][1], res[False][1]) < 5e-2


@pytest.mark.parametrize("n,h,fused", [(3, 224, True), (2, 96, False)])
def test_fused_stem_backward_matches_two_pass(n, h, fused, monkeypatch):
    """The stem's max-pool + BN(+ReLU) backward elementwise pass run INSIDE the stem weight
    gradient (stem_wgrad_fused: dy never materialised) == the two-pass path (stem_pool_bwd_elemt
    writes dy, the halo wgrad reads it back): bit for bit, in the deterministic statistics mode
    with the halo weight-gradient variant pinned.  96x96 inputs are outside the fused plan
    (3-row bands): the stand-in dy falls back to the two passes."""
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims as HP
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    x, y = C.synth_images(n, h, h, 8, 3, 1000, 11, 0)
    calls = {"fused": 0}
    orig = HP.stem_wgrad_fused

    def spy(*a, **k):
        r = orig(*a, **k)
        calls["fused"] += r is not None
        return r
    monkeypatch.setattr(HP, "stem_wgrad_fused", spy)
    C.conv_wgrad_set_impl(6)
    OF.set_deterministic(True)
    res = {}
    try:
        for lazy in (True, False):
            monkeypatch.setattr(OF, "_STEM_LAZY", lazy)
            torch.manual_seed(0)
            m = ResNet50(num_classes=1000, stem="imagenet").to(DEV)
            loss = OF.cross_entropy(m(x), y)
            loss.backward()
            torch.cuda.synchronize()
            res[lazy] = (loss.detach().clone(), m.conv1.weight.grad.clone(), m.bn1.weight.grad.clone(),
                         m.bn1.bias.grad.clone())
    finally:
        OF.set_deterministic(False)
        C.conv_wgrad_set_impl(-1)
    assert calls["fused"] == (1 if fused else 0)
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)


def test_s2d_input_prefetched_with_the_batch_is_bit_exact():
    """The stem's space-to-depth input layout made by the data prefetch on the side stream
    (ops/functional.py s2d_input_prefetch, data/loader.py prefetch transform) gives the same
    two-stream ResNet-50 steps, bit for bit (deterministic statistics mode), as the stem laying
    the batch out itself -- and the prefetched layout is what the stem consumed."""
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.models import ResNet50
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    dev = torch.device(DEV, 0)
    OF.init_step_streams(dev)
    OF.set_deterministic(True)
    try:
        res = []
        for pre in (False, True):
            torch.manual_seed(0)
            m = ResNet50(num_classes=1000, stem="imagenet").to(dev)
            data = SyntheticImageNet(4, 64, 1000, steps=3, device=dev, dtype=torch.bfloat16, cpad=8, seed=5)
            tf = OF.s2d_input_prefetch(m) if pre else None
            assert (tf is not None) == pre
            data.prefetch(OF._wgrad_stream(dev), transform=tf)
            losses = []
            for i in range(3):
                x, y = data.next_batch(i)
                assert (getattr(x, "_pmd_s2d_in", None) is not None) == pre
                loss = OF.cross_entropy(m(x), y)
                assert getattr(x, "_pmd_s2d_in", None) is None      # consumed by the stem
                loss.backward(OF.loss_seed(loss))
                losses.append(loss.detach().clone())
            torch.cuda.synchronize()
            res.append((torch.stack(losses), m.conv1.weight.grad.clone(), m.bn1.running_mean.clone()))
    finally:
        OF.set_deterministic(False)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
