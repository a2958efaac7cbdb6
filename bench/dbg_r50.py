"""Debug: ResNet-50 (ImageNet stem) gradients + short training on the gfx950
kernels vs the torch reference prims (bf16 and fp32 activations), from
identical weights."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD  # noqa: E402
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
base = ResNet50(num_classes=10, stem="imagenet").to(DEV)
sd = {k: v.clone() for k, v in base.state_dict().items()}
x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
y = torch.arange(16, device=DEV) % 10


def run(mode, lr, steps):
    OF.force_torch_prims(mode != "hip")
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    m.load_state_dict(sd)
    opt = FusedSGD(m, lr=lr, momentum=0.9, weight_decay=0.0, nesterov=True)
    xin = x.float() if mode == "torch32" else x
    ls, g0 = [], None
    for it in range(steps):
        loss = OF.cross_entropy(m(xin), y)
        opt.zero_grad()
        loss.backward()
        if it == 0:
            g0 = {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}
        opt.step()
        ls.append(round(loss.item(), 3))
    OF.force_torch_prims(False)
    return ls, g0


grads = {}
for mode in ("hip", "torch", "torch32"):
    ls, grads[mode] = run(mode, 0.05, 1)
for a, b in (("hip", "torch32"), ("torch", "torch32"), ("hip", "torch")):
    cs = []
    for n in grads[a]:
        g, r = grads[a][n], grads[b][n]
        cs.append((torch.nn.functional.cosine_similarity(g.flatten(), r.flatten(), dim=0).item(), n))
    cs.sort()
    print(f"{a} vs {b}: median cos {cs[len(cs)//2][0]:.4f}  worst {cs[:4]}")
for lr in (0.05, 0.02, 0.01):
    for mode in ("hip", "torch", "torch32"):
        ls, _ = run(mode, lr, 25)
        print(f"lr {lr} {mode:8s} ratio {ls[-1] / ls[0]:.3f} {ls}", flush=True)
