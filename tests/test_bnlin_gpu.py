"""Linear-BN backward on the gfx950 path (kernels/bnlin.hip + the dgrad epilogue's addend bias
and sum-only reduce): each primitive against its fp32 PyTorch twin (ops/torch_prims.py), and a
whole ResNet-50 training step with every eligible block on the linear path against the fp32
oracle, no worse than the elementwise path on the same tensors."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hp():
    from pytorch_multiprocessing_distributed_amd.ops import hip_prims
    return hip_prims


def _tp():
    from pytorch_multiprocessing_distributed_amd.ops import torch_prims
    return torch_prims


@pytest.mark.parametrize("K,C", [(256, 64), (512, 128), (1024, 256), (2048, 512)])
def test_bnlin_prims_match_torch(K, C):
    HP, TP = _hp(), _tp()
    torch.manual_seed(K + C)
    wk = (torch.randn(K, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
    T = torch.randn(K, 1, 1, C, device=DEV)
    p = torch.stack([torch.randn(K, device=DEV) * 0.1, torch.rand(K, device=DEV) + 0.5,
                     torch.zeros(K, device=DEV), torch.zeros(K, device=DEV)]).contiguous()
    # coefficients, scaled dgrad image, G, bias
    red = torch.randn(2, K, device=DEV) * 100
    gamma = torch.rand(K, device=DEV) + 0.5
    cnt = torch.full((1,), 4096.0, device=DEV)
    (_, g), bias, abc = HP.bnlin_coeff(red, cnt, gamma, p, wk, C)
    (g_r,), bias_r, abc_r = TP.bnlin_coeff(red.double(), cnt.double(), gamma.double(), p.double(),
                                           wk.double(), C)
    torch.testing.assert_close(abc.double(), abc_r, rtol=1e-5, atol=1e-6)
    (_, wkt_a) = HP.bnlin_dimg(gamma, p, wk, C)
    (wk_a,) = TP.bnlin_dimg(gamma.double(), p.double(), wk.double(), C)
    torch.testing.assert_close(wkt_a.double(), wk_a.reshape(K, C).t().reshape(C, 1, 1, K), rtol=1e-2, atol=1e-3)
    torch.testing.assert_close(g.double(), g_r, rtol=2e-2, atol=2e-2 * g_r.abs().max().item())
    torch.testing.assert_close(bias.double(), bias_r, rtol=1e-4, atol=1e-4 * bias_r.abs().max().item())
    # colsum
    x = torch.randn(3, 7, 9, C, device=DEV).to(torch.bfloat16)
    torch.testing.assert_close(HP.colsum(x), x.float().reshape(-1, C).sum(0), rtol=1e-4, atol=1e-3)
    # weight-gradient combine
    gz = torch.randn(C, 1, 1, C, device=DEV)
    cs = torch.randn(C, device=DEV)
    out = torch.randn(K, 1, 1, C, device=DEV)
    want = out.double().clone()
    HP.bnlin_wgrad_(out, abc, T, wk, gz, cs)
    TP.bnlin_wgrad_(want, abc.double(), T.double(), wk.double(), gz.double(), cs.double())
    torch.testing.assert_close(out.double(), want, rtol=1e-4, atol=1e-3 * want.abs().max().item())


def test_dgrad_addend_bias_and_sum_only_reduce():
    """conv_dgrad(addend, addend_bias) == dgrad + addend + bias; a y-less BN set reduces
    (sum dz, -mean * invstd * sum dz) of the masked output."""
    HP = _hp()
    torch.manual_seed(3)
    N, H, C, K = 4, 14, 128, 512
    dy = torch.randn(N, H, H, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, C, 1, 1, device=DEV) / K ** 0.5).contiguous(memory_format=torch.channels_last)
    wp = HP.conv_weight(w, torch.bfloat16, C, True)
    add = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    bias = torch.randn(C, device=DEV)
    base = HP.conv_dgrad(dy, wp, (N, H, H, C), 1, 0)
    out = HP.conv_dgrad(dy, wp, (N, H, H, C), 1, 0, add, addend_bias=bias)
    want = base.float() + add.float() + bias
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2)
    # sum-only reduce with a mask
    p = torch.stack([torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5,
                     torch.ones(C, device=DEV), torch.zeros(C, device=DEV)]).contiguous()
    mbool = torch.rand(N, H, H, C, device=DEV) > 0.4
    bits = (mbool.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=DEV, dtype=torch.uint8)).sum(1,
                                                                                             dtype=torch.uint8)
    dx, bufs = HP.conv_dgrad(dy, wp, (N, H, H, C), 1, 0, bnred=(bits.reshape(N, H, H, C // 8), [(None, p)]))
    r = bufs[0].sum(0)
    dzm = dx.float().reshape(-1, C)
    torch.testing.assert_close(dzm, (base.float() * mbool).reshape(-1, C), rtol=0, atol=0)
    s = dzm.sum(0)
    torch.testing.assert_close(r[0], s, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(r[1], -p[0] * p[1] * s, rtol=1e-4, atol=1e-2)
    HP._release(*bufs)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("arena", [False, True])
def test_resnet50_train_step_linear_bn_vs_fp32_oracle(monkeypatch, arena):
    """Every identity bottleneck block on the linear path (PMD_BNLIN=all) vs the elementwise
    path, both against the fp32 PyTorch-primitive oracle on the same weights and batch: loss,
    running statistics, and the per-tensor gradient error no worse than the elementwise path's
    (median, 90th percentile; the conv3 / bn3 tensors of the linear blocks individually)."""
    import copy
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.manual_seed(0)
    m0 = build_model("resnet50", num_classes=1000, stem="imagenet").to(DEV)
    x, y = C.synth_images(32, 112, 112, 8, 3, 1000, 7, 0)
    m0.train()
    ms = {k: copy.deepcopy(m0) for k in ("lin", "elt", "f32")}
    grads, loss = {}, {}
    for k, m in ms.items():
        monkeypatch.setattr(OF, "_BNLIN", "all" if k == "lin" else "0")
        mm = DataParallel(m, None) if arena else m
        OF.force_torch_prims(k == "f32")
        try:
            lo = OF.cross_entropy(mm(x.float() if k == "f32" else x), y)
            lo.backward()
        finally:
            OF.force_torch_prims(False)
        torch.cuda.synchronize()
        loss[k] = float(lo)
        grads[k] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    ee = {n: _rel(g, grads["f32"][n]) for n, g in grads["elt"].items()}

    def q(v, f):
        v = sorted(v)
        return v[min(int(len(v) * f), len(v) - 1)]
    for k in ("lin",):
        assert abs(loss[k] - loss["f32"]) / loss["f32"] < 1e-2, (k, loss)
        el = {n: _rel(g, grads["f32"][n]) for n, g in grads[k].items()}
        for f in (0.5, 0.9):
            assert q(el.values(), f) < 1.2 * q(ee.values(), f) + 1e-3, (k, f, q(el.values(), f), q(ee.values(), f))
        bad = [(n, el[n], ee[n]) for n in el if ("conv3" in n or "bn3" in n) and el[n] > 2.0 * ee[n] + 2e-2]
        assert not bad, (k, bad)
        for (n, b1), b2, b3 in zip(ms[k].named_buffers(), ms["f32"].buffers(), ms["elt"].buffers()):
            if b1.dtype.is_floating_point and n.endswith("running_var"):
                assert _rel(b1, b2) < 1e-2, (k, n)
            if b1.dtype.is_floating_point and n.endswith("running_mean"):
                # means near zero: bounded by the elementwise path's own error
                assert _rel(b1, b2) < 1.5 * _rel(b3, b2) + 1e-3, (k, n, _rel(b1, b2), _rel(b3, b2))
