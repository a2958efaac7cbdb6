"""Determinism check: ResNet-50 step repeated, fused vs composite stem tail."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

res = {True: [], False: []}
for fused in (True, False) * 4:
    OF.set_fused_stem(fused)
    torch.manual_seed(0)
    m = ResNet50(num_classes=1000, stem="imagenet").cuda()
    x, y = C.synth_images(4, 64, 64, 8, 3, 1000, 7, 0)
    cap = {}
    h = m.layer1.register_forward_pre_hook(lambda mod, inp: cap.update(inp=inp[0].detach().clone()))
    loss = OF.cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    h.remove()
    r = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    r["_loss"] = loss.detach().reshape(1).float()
    print("fused", fused, "site hits/misses", OF._state["fused_site_hits"], OF._state["fused_site_misses"])
    r["_stem_out"] = cap["inp"].float()
    res[fused].append(r)
for fused in (True, False):
    base = res[fused][0]
    for i, r in enumerate(res[fused][1:]):
        bad = {n: (r[n] - base[n]).abs().max().item() for n in base if not torch.equal(r[n], base[n])}
        worst = sorted(bad.items(), key=lambda kv: -kv[1])[:4]
        print(f"fused={fused} run {i + 1} vs run 0: {len(bad)} params differ; worst {worst}")
a, b = res[True][0], res[False][0]
bad = {n: (a[n] - b[n]).abs().max().item() for n in a if not torch.equal(a[n], b[n])}
print("fused vs composite: differing params", len(bad), sorted(bad.items(), key=lambda kv: -kv[1])[:5])
