import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD  # noqa: E402
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402

DEV = "cuda"
x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
yl = torch.arange(16, device=DEV) % 10
torch.manual_seed(0)
base = ResNet50(num_classes=10, stem="imagenet").to(DEV)
sd = {k: v.clone() for k, v in base.state_dict().items()}
outs = {}
for mode in ("fp32", "bf16", "fp8"):
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    m.load_state_dict(sd)
    m.eval()
    OF.force_torch_prims(mode == "fp32")
    OF.set_fp8(Fp8Scaling(DEV) if mode == "fp8" else None)
    with torch.no_grad():
        outs[mode] = m(x.float() if mode == "fp32" else x).float()
    OF.set_fp8(None)
    OF.force_torch_prims(False)
for a, b in (("bf16", "fp32"), ("fp8", "fp32"), ("fp8", "bf16")):
    print("eval logits", a, "vs", b, ((outs[a] - outs[b]).norm() / outs[b].norm()).item())
for lr in (0.01, 0.003):
    for mode in ("bf16", "fp8"):
        m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
        m.load_state_dict(sd)
        OF.set_fp8(Fp8Scaling(DEV) if mode == "fp8" else None)
        opt = FusedSGD(m, lr=lr, momentum=0.9, weight_decay=0.0, nesterov=True)
        ls = []
        for it in range(25):
            loss = OF.cross_entropy(m(x), yl)
            opt.zero_grad()
            loss.backward()
            opt.step()
            ls.append(round(loss.item(), 3))
        OF.set_fp8(None)
        print("train lr", lr, mode, ls, flush=True)
