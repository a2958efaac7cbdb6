"""Debug the fp8 (config 5) path: per-step logits/scales, bn_apply fp8 copy check."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD  # noqa: E402
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF, hip_prims as HP  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

DEV = "cuda"
# 1) bn_apply fp8 copy
y = torch.randn(64, 8, 8, 256, device=DEV).to(torch.bfloat16)
p = torch.stack([torch.zeros(256, device=DEV), torch.ones(256, device=DEV),
                 torch.ones(256, device=DEV), torch.zeros(256, device=DEV)]).contiguous()
sc = torch.tensor([4.0], device=DEV)
am = torch.zeros(64, device=DEV)
out, mask, q = HP.bn_apply(y, p, relu=True, fp8=(sc, am))
deq = C.dequant_fp8(q.contiguous(), torch.tensor([0.25], device=DEV))
print("bn_apply q8 rel err", ((deq - out.float()).norm() / out.float().norm()).item(),
      "amax", am.max().item(), out.float().abs().max().item())
# 2) training trace
x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
yl = torch.arange(16, device=DEV) % 10
torch.manual_seed(0)
m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
f8 = Fp8Scaling(DEV)
OF.set_fp8(f8)
opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
names = {}
for nm, mod in m.named_modules():
    names[id(mod)] = nm
for it in range(6):
    logits = m(x)
    loss = OF.cross_entropy(logits, yl)
    opt.zero_grad()
    loss.backward()
    opt.step()
    n = len(f8.sites)
    inv = {v: k for k, v in f8.sites.items()}
    sc = f8.scale[:n].cpu()
    am = f8.amax[:n].cpu()
    print(f"it {it} loss {loss.item():.4f} logits std {logits.float().std().item():.4f} "
          f"scale min {sc.min().item():.3g} max {sc.max().item():.3g} amax max {am.max().item():.3g}")
    if it in (0, 2, 5):
        for i in range(n):
            k = inv[i]
            print("   ", k[0], names.get(k[1], "?"), f"scale {sc[i].item():.4g} amax {am[i].item():.4g}")
