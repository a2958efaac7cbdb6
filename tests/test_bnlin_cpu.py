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


@pytest.mark.parametrize("arena", [False, True])
def test_bnlin_matches_stock_resnet50(bnlin_all, arena):
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
