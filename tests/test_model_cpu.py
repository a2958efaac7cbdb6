"""Model structure / numerics on the CPU (torch-primitive) backend.

* key set, order, shapes and counts equal the stock nn.Conv2d/nn.BatchNorm2d
  tree (= the reference's module naming);
* the fused NHWC op graph (conv+stats, BN+add+ReLU autograd Functions) gives
  the same loss, gradients and running statistics as the stock NCHW model;
* the saved checkpoint is the reference format: ``module.`` keys, fp32,
  ``_metadata`` versions, loads strict into the stock model.
"""
import collections

import pytest
import torch

from pytorch_multiprocessing_distributed_amd.models import build_model
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
from pytorch_multiprocessing_distributed_amd.utils.checkpoint import load_model, save_model


def _copy_into_stock(fused, stock):
    with torch.no_grad():
        sd = stock.state_dict()
        for k, v in fused.state_dict().items():
            sd[k].copy_(v)


@pytest.mark.parametrize("name,stem,nkeys,nparams", [
    ("res", "cifar", 74, 4903242),
    ("resnet34", "cifar", None, 21282122),
    ("resnet50", "cifar", 320, 23520842),
    ("resnet50", "imagenet", 320, 25557032),
    ("resnet152", "imagenet", 932, 60192808),
])
def test_keys_and_sizes(name, stem, nkeys, nparams):
    nc = 1000 if stem == "imagenet" else 10
    f = build_model(name, num_classes=nc, stem=stem)
    s = build_model(name, num_classes=nc, stem=stem, impl="stock")
    fk, sk = f.state_dict(), s.state_dict()
    assert list(fk.keys()) == list(sk.keys())
    for k in fk:
        assert fk[k].shape == sk[k].shape and fk[k].dtype == sk[k].dtype, k
    if nkeys:
        assert len(fk) == nkeys
    assert sum(p.numel() for p in f.parameters()) == nparams
    assert fk._metadata["bn1"]["version"] == 2


@pytest.mark.parametrize("name,stem,hw", [("res", "cifar", 32), ("resnet50", "imagenet", 64),
                                          ("resnet34", "cifar", 32)])
def test_fused_matches_stock_train_step(name, stem, hw):
    torch.manual_seed(0)
    nc = 1000 if stem == "imagenet" else 10
    f = build_model(name, num_classes=nc, stem=stem).double()
    s = build_model(name, num_classes=nc, stem=stem, impl="stock").double()
    _copy_into_stock(f, s)
    x = torch.randn(4, 3, hw, hw, dtype=torch.float64)
    y = torch.randint(0, nc, (4,))
    for step in range(2):
        lf = OF.cross_entropy(f(x.permute(0, 2, 3, 1).contiguous()), y)
        ls = torch.nn.functional.cross_entropy(s(x), y)
        torch.testing.assert_close(lf, ls, rtol=1e-9, atol=1e-9)
        f.zero_grad()
        s.zero_grad()
        lf.backward()
        ls.backward()
        for (n, pf), ps in zip(f.named_parameters(), s.parameters()):
            torch.testing.assert_close(pf.grad, ps.grad, rtol=1e-7, atol=1e-9, msg=n)
    for (n, bf), bs in zip(f.named_buffers(), s.buffers()):
        torch.testing.assert_close(bf, bs, rtol=1e-9, atol=1e-9, msg=n)
    f.eval()
    s.eval()
    with torch.no_grad():
        torch.testing.assert_close(f(x.permute(0, 2, 3, 1).contiguous()), s(x), rtol=1e-8,
                                   atol=1e-8)


@pytest.mark.parametrize("name,stem,hw", [("res", "cifar", 32), ("resnet50", "imagenet", 64)])
def test_eval_mode_backward_matches_stock(name, stem, hw):
    torch.manual_seed(1)
    nc = 1000 if stem == "imagenet" else 10
    f = build_model(name, num_classes=nc, stem=stem).double().eval()
    s = build_model(name, num_classes=nc, stem=stem, impl="stock").double().eval()
    _copy_into_stock(f, s)
    x = torch.randn(2, 3, hw, hw, dtype=torch.float64)
    f(x.permute(0, 2, 3, 1).contiguous()).sum().backward()
    s(x).sum().backward()
    for (n, pf), ps in zip(f.named_parameters(), s.parameters()):
        torch.testing.assert_close(pf.grad, ps.grad, rtol=1e-7, atol=1e-9, msg=n)


def test_reference_checkpoint_format(tmp_path):
    m = DataParallel(build_model("res"), comm=None)
    path = save_model(m, str(tmp_path), 20)
    assert path.endswith("model_20.pth")
    sd = torch.load(path, weights_only=True)
    assert isinstance(sd, collections.OrderedDict)
    assert len(sd) == 74 and all(k.startswith("module.") for k in sd)
    assert sd["module.conv1.weight"].shape == (64, 3, 3, 3)
    assert sd["module.conv1.weight"].is_contiguous()
    assert sd["module.linear.weight"].shape == (10, 512)
    assert sd["module.bn1.num_batches_tracked"].dtype == torch.int64
    assert sd._metadata["module.bn1"]["version"] == 2
    # loads strict into the stock (reference-structured) model after stripping module.
    stock = build_model("res", impl="stock")
    stock.load_state_dict({k[7:]: v for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        for k, v in stock.state_dict().items():
            assert torch.equal(v, m.module.state_dict()[k])
    # and back into our own model through the arena-preserving loader
    m2 = DataParallel(build_model("res"), comm=None)
    load_model(m2, path)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    # one storage per tensor, like the reference's zip container
    import zipfile
    with zipfile.ZipFile(path) as z:
        blobs = [n for n in z.namelist() if "/data/" in n and not n.endswith("serialization_id")]
    assert len(blobs) == 74


def test_flat_arena_views_and_grads():
    m = build_model("res")
    dp = DataParallel(m, comm=None)
    fp = dp.flat
    w = m.conv1.weight
    assert w.is_contiguous(memory_format=torch.channels_last)
    assert w.data_ptr() >= fp.param_arena.data_ptr()
    x = torch.randn(2, 32, 32, 3)
    OF.cross_entropy(dp(x), torch.tensor([1, 2])).backward()
    assert w.grad.data_ptr() >= fp.grad_arena.data_ptr()
    assert fp.grad_arena.abs().sum() > 0
    # buckets tile the arena contiguously
    assert dp.buckets[0].start == 0 and dp.buckets[-1].end == fp.numel
    for a, b in zip(dp.buckets, dp.buckets[1:]):
        assert a.end == b.start


@pytest.mark.parametrize("arch", ["res", "resnet50"])
def test_fused_bn_reduce_matches_unfused(arch):
    """BN-backward reduces fused into the dgrad epilogues (intra-block and across
    blocks through the _BnSite hand-off) give the same gradients as the
    separate bn_bwd_reduce passes (fp64 torch prims)."""
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    grads = {}
    for fuse in (False, True):
        OF.set_fuse_bn_reduce(fuse)
        torch.manual_seed(0)
        stem = "cifar" if arch == "res" else "imagenet"
        m = build_model(arch, num_classes=10, stem=stem).double()
        g = torch.Generator().manual_seed(1)
        hw = 32 if stem == "cifar" else 64
        x = torch.randn(4, hw, hw, 3, generator=g, dtype=torch.float64)
        y = torch.randint(0, 10, (4,), generator=g)
        hits0 = OF._state["fused_site_hits"]
        OF.cross_entropy(m(x), y).backward()
        if fuse:
            assert OF._state["fused_site_hits"] > hits0     # cross-block hand-off happened
        grads[fuse] = {n: p.grad.clone() for n, p in m.named_parameters()}
    OF.set_fuse_bn_reduce(True)
    for n, g0 in grads[False].items():
        torch.testing.assert_close(grads[True][n], g0, rtol=1e-9, atol=1e-12, msg=n)


REF_RESNET = "/root/reference/model/resnet.py"


@pytest.mark.skipif(not __import__("os").path.exists(REF_RESNET), reason="reference tree not mounted")
def test_checkpoint_loads_into_reference_model_class(tmp_path):
    """SURVEY §4.2 format compatibility: our model_<E>.pth, with ``module.``
    stripped, loads strict=True into the reference's own ``ResNet18()`` and
    gives the same forward (fp32, eval)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_resnet", REF_RESNET)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)           # plain source: class definitions only
    torch.manual_seed(0)
    m = DataParallel(build_model("res"), comm=None)
    path = save_model(m, str(tmp_path), 3)
    sd = torch.load(path, weights_only=True)
    rm = ref.ResNet18()
    rm.load_state_dict({k[7:]: v for k, v in sd.items()}, strict=True)
    rm.eval()
    m.module.eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        want = rm(x)
        got = m.module(x.permute(0, 2, 3, 1).contiguous())
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-5)


def test_weight_image_set_covers_every_conv(monkeypatch):
    """The grouped weight-image refresh must serve EVERY conv of the model (one
    prep launch per forward); a conv whose lookup misses falls back to its own
    per-conv prep launch.  Simulated on CPU with a stand-in for the native
    image table (the lookup keys are what is under test)."""
    from pytorch_multiprocessing_distributed_amd.ops import torch_prims as TP
    from pytorch_multiprocessing_distributed_amd.ops.native import C

    class FakeImages:
        def __init__(self, ws, cps, wts):
            self.e = list(zip(ws, cps, wts))

        def refresh(self, mode=3):
            pass

        def get(self, i):
            w, cp, wt = self.e[i]
            return list(TP.conv_weight(w, torch.float32, cp, wt))

    monkeypatch.setattr(C, "WeightImages", FakeImages, raising=False)
    monkeypatch.setattr(TP, "SUPPORTS_FP8", True, raising=False)
    calls = {"hit": 0, "miss": 0}
    orig = OF.WeightImageSet.lookup

    def lookup(self, w, cin, want_t):
        r = orig(self, w, cin, want_t)
        calls["hit" if r is not None else "miss"] += 1
        return r
    monkeypatch.setattr(OF.WeightImageSet, "lookup", lookup)
    for name, stem, hw in [("resnet50", "imagenet", 64), ("res", "cifar", 32)]:
        calls.update(hit=0, miss=0)
        m = build_model(name, num_classes=10, stem=stem)
        m(torch.randn(2, hw, hw, 8 if stem == "imagenet" else 3)).sum().backward()
        nconv = sum(1 for mod in m.modules() if hasattr(mod, "kernel_size"))
        assert calls == {"hit": nconv, "miss": 0}, (name, calls, nconv)
