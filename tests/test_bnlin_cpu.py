"""Linear-BN backward (ops/functional.py _bnlin_final): the final BN of a bottleneck block
back-propagated through its 1x1 conv3 -- without reading the BN input y and without ever
forming dy -- equals the stock PyTorch model's gradients in fp64, on the CPU backend, with and
without the flat gradient arena, and with the fused statistics path both hit and missed.
(The GPU kernels of the same prims: tests/test_kernels_gpu.py::test_bnlin_*.)"""
import pytest
import torch

from pytorch_multiprocessing_distributed_amd.models import build_model
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel


@pytest.fixture
def bnlin_all(monkeypatch):
    monkeypatch.setattr(OF, "_BNLIN", "all")
    yield


def _copy_into_stock(fused, stock):
    with torch.no_grad():
        sd = stock.state_dict()
        for k, v in fused.state_dict().items():
            sd[k].copy_(v)


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("arena", [False, True])
def test_bnlin_matches_stock_resnet50(bnlin_all, arena, fold, monkeypatch):
    # fold: the final conv3 output y never exists (statistics-only conv3, then conv3 with the
    # BN-apply epilogue; backward: sum-only fused reduce + the recomputed y part, _bnfold_dot)
    monkeypatch.setattr(OF, "_BNFOLD", fold)
    torch.manual_seed(0)
    f = build_model("resnet50", num_classes=10, stem="imagenet").double()
    s = build_model("resnet50", num_classes=10, stem="imagenet", impl="stock").double()
    _copy_into_stock(f, s)
    fm = DataParallel(f, None) if arena else f
    x = torch.randn(3, 3, 64, 64, dtype=torch.float64)
    y = torch.randint(0, 10, (3,))
    for step in range(2):
        lf = OF.cross_entropy(fm(x.permute(0, 2, 3, 1).contiguous()), y)
        ls = torch.nn.functional.cross_entropy(s(x), y)
        torch.testing.assert_close(lf, ls, rtol=1e-9, atol=1e-9)
        fm.zero_grad()
        s.zero_grad()
        lf.backward()
        ls.backward()
        for (n, pf), ps in zip(f.named_parameters(), s.parameters()):
            torch.testing.assert_close(pf.grad, ps.grad, rtol=1e-7, atol=1e-9, msg=n)
    for (n, bf), bs in zip(f.named_buffers(), s.buffers()):
        torch.testing.assert_close(bf, bs, rtol=1e-9, atol=1e-9, msg=n)


def test_bnlin_path_is_taken(bnlin_all, monkeypatch):
    """Every identity bottleneck block whose output feeds another block's fused dgrad takes
    the linear path (ResNet-50: 12 identity blocks, the last one has no fused producer)."""
    calls = []
    orig = OF._bnlin_final

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    monkeypatch.setattr(OF, "_bnlin_final", spy)
    torch.manual_seed(0)
    f = build_model("resnet50", num_classes=10, stem="imagenet").double()
    x = torch.randn(2, 64, 64, 3, dtype=torch.float64)
    OF.cross_entropy(f(x), torch.tensor([1, 2])).backward()
    assert len(calls) == 11


def test_bnlin_off_by_default_below_threshold():
    # "auto": only BN inputs of >= 200704 x 512 elements (ResNet-50 l1 / l2 at batch 256)
    assert OF._BNLIN == "auto"
    conv = torch.nn.Conv2d(64, 256, 1, bias=False)
    small = torch.empty(50176, 1, 1, 1024, device="meta")      # l3: 51.4M elements
    assert not OF._bnlin_eligible(conv, small, None, True, True, None, None)
    big = torch.empty(200704, 1, 1, 512, device="meta")        # l2: 102.8M elements
    assert OF._bnlin_eligible(conv, big, None, True, True, None, None)
    assert not OF._bnlin_eligible(conv, big, None, False, True, None, None)      # eval
    assert not OF._bnlin_eligible(conv, big, None, True, True, ("proj",), None)  # projection block
    assert not OF._bnlin_eligible(torch.nn.Conv2d(64, 256, 3, padding=1), big, None, True, True, None, None)


def test_bnfold_path_is_taken(bnlin_all, monkeypatch):
    """With the fold on, every identity block's final conv runs as statistics-only + BN-apply
    epilogue passes (12 in ResNet-50); 11 of them complete their reduce from z (the 12th, the
    last block, has no fused producer and recomputes y)."""
    from pytorch_multiprocessing_distributed_amd.ops import torch_prims as TP
    counts = {"apply": 0, "dot": 0, "stats": 0}
    for name in ("conv_fwd_apply", "conv_bn_dot_", "conv_fwd_stats"):
        orig = getattr(TP, name)

        def spy(*a, _o=orig, _n=name, **k):
            counts[{"conv_fwd_apply": "apply", "conv_bn_dot_": "dot", "conv_fwd_stats": "stats"}[_n]] += 1
            return _o(*a, **k)
        monkeypatch.setattr(TP, name, spy)
    monkeypatch.setattr(OF, "_BNFOLD", True)
    torch.manual_seed(0)
    f = build_model("resnet50", num_classes=10, stem="imagenet").double()
    x = torch.randn(2, 64, 64, 3, dtype=torch.float64)
    OF.cross_entropy(f(x), torch.tensor([1, 2])).backward()
    assert counts == {"apply": 12, "dot": 11, "stats": 12}


def test_bnfold_prims_match_unfused():
    """conv_fwd_apply == bn_apply(conv_fwd), conv_fwd_stats == conv_fwd's statistics, and the
    sum-only reduce + conv_bn_dot_ == the full reduce (fp64, torch prims)."""
    from pytorch_multiprocessing_distributed_amd.ops import torch_prims as TP
    torch.manual_seed(1)
    z = torch.randn(2, 5, 6, 16, dtype=torch.float64).relu()
    wk = (TP.conv_weight(torch.randn(32, 16, 1, 1, dtype=torch.float64), torch.float64, 16)[0],)
    res = torch.randn(2, 5, 6, 32, dtype=torch.float64)
    shift = torch.randn(32, dtype=torch.float64)
    y, st = TP.conv_fwd(z, wk, 1, 0, shift)
    torch.testing.assert_close(TP.conv_fwd_stats(z, wk, 1, 0, shift), st)
    p = TP.stats_finalize_local(st.clone(), y.numel() // 32, torch.rand(32, dtype=torch.float64) + 0.5,
                                torch.randn(32, dtype=torch.float64), 1e-5, shift=shift.clone())
    o1, m1 = TP.bn_apply(y, p, res)
    o2, m2 = TP.conv_fwd_apply(z, wk, 1, 0, p, res)
    torch.testing.assert_close(o2, o1)
    assert torch.equal(m1, m2)
    dz = torch.randn_like(y)
    full = TP.bn_bwd_reduce(dz, None, y, p, False)
    part = TP.bn_bwd_reduce(dz, None, None, p, False)
    TP.conv_bn_dot_(z, wk, dz, p, part)
    torch.testing.assert_close(part, full, rtol=1e-10, atol=1e-10)
