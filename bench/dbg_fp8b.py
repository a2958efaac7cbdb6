import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

DEV = "cuda"
x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
yl = torch.arange(16, device=DEV) % 10
res = {}
for mode in ("bf16", "fp8"):
    torch.manual_seed(0)
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    OF.set_fp8(Fp8Scaling(DEV) if mode == "fp8" else None)
    acts = {}
    hooks = []
    for nm, mod in m.named_children():
        if nm.startswith("layer"):
            for bi, blk in enumerate(mod):
                hooks.append(blk.register_forward_hook(
                    lambda mod_, i, o, key=f"{nm}.{bi}": acts.__setitem__(key, o.detach().float().clone())))
    logits = m(x)
    loss = OF.cross_entropy(logits, yl)
    loss.backward()
    res[mode] = (acts, {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}, logits.detach())
    OF.set_fp8(None)
a0, g0, l0 = res["bf16"]
a1, g1, l1 = res["fp8"]
for k in a0:
    print(k, "act rel", ((a1[k] - a0[k]).norm() / a0[k].norm()).item())
print("logits rel", ((l1 - l0).norm() / l0.norm()).item())
rows = []
for n in g0:
    r = g1[n].norm() / g0[n].norm().clamp_min(1e-20)
    cos = torch.nn.functional.cosine_similarity(g1[n].flatten(), g0[n].flatten(), dim=0).item()
    rows.append((r.item(), cos, n))
rows.sort(reverse=True)
for r in rows[:10]:
    print("grad norm ratio", r)
for r in rows[-5:]:
    print("grad norm ratio", r)
