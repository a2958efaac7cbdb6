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


class Frozen(Fp8Scaling):
    def update(self):
        self.amax.zero_()
        self.steps += 1


for name, mk, lr in (("frozen", lambda: Frozen(DEV), 0.01), ("margin4", lambda: Fp8Scaling(DEV, margin=4.0), 0.01),
                     ("delayed-lr1e-3", lambda: Fp8Scaling(DEV), 0.001), ("bf16-lr1e-3", lambda: None, 0.001)):
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    m.load_state_dict(sd)
    OF.set_fp8(mk())
    opt = FusedSGD(m, lr=lr, momentum=0.9, weight_decay=0.0, nesterov=True)
    ls = []
    for it in range(25):
        loss = OF.cross_entropy(m(x), yl)
        opt.zero_grad()
        loss.backward()
        opt.step()
        ls.append(round(loss.item(), 3))
    OF.set_fp8(None)
    print(name, ls, flush=True)
# which weights/acts go dead: per-block output stats at step 3 of the delayed run
m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
m.load_state_dict(sd)
OF.set_fp8(Fp8Scaling(DEV))
opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
stats = {}
for nm, mod in m.named_children():
    if nm.startswith("layer"):
        for bi, blk in enumerate(mod):
            blk.register_forward_hook(lambda mod_, i, o, key=f"{nm}.{bi}": stats.__setitem__(
                key, (o.float().mean().item(), (o.float() > 0).float().mean().item())))
for it in range(3):
    loss = OF.cross_entropy(m(x), yl)
    print("it", it, loss.item(), {k: tuple(round(v, 4) for v in s) for k, s in stats.items()})
    opt.zero_grad()
    loss.backward()
    opt.step()
bn = {n: (p.min().item(), p.max().item()) for n, p in m.named_parameters() if "bn" in n and "bias" in n}
print("bn bias ranges", list(bn.items())[:12])
