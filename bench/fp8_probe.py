"""fp8 forward numerics per conv policy: ResNet-50 logits / first loss with every
eligible block conv in fp8 (policy "all") or only the 3x3 convs ("spatial"), vs the
bf16 model of the same weights, for the first forward and after a few steps."""
import torch

from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
from pytorch_multiprocessing_distributed_amd.models import ResNet50
from pytorch_multiprocessing_distributed_amd.ops import functional as OF
from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
from pytorch_multiprocessing_distributed_amd.ops.native import C

DEV = "cuda"


def run(mode, policy, x, y, steps=4):
    torch.manual_seed(0)
    m = ResNet50(num_classes=10, stem="imagenet").to(DEV)
    OF.FP8_CONVS = policy
    f8 = Fp8Scaling(DEV) if mode == "fp8" else None
    OF.set_fp8(f8)
    outs, losses = [], []
    try:
        opt = FusedSGD(m, lr=0.01, momentum=0.9, weight_decay=0.0, nesterov=True)
        for _ in range(steps):
            out = m(x)
            loss = OF.cross_entropy(out, y)
            outs.append(out.float().detach().clone())
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
    finally:
        OF.set_fp8(None)
        OF.FP8_CONVS = "spatial"
    return outs, losses, (len(f8.sites) if f8 else 0)


def main():
    x, _ = C.synth_images(16, 64, 64, 8, 3, 10, 5, 0)
    y = torch.arange(16, device=DEV) % 10
    ref, lref, _ = run("bf16", "spatial", x, y)
    print("bf16 losses", [round(v, 4) for v in lref])
    for pol in ("all", "spatial"):
        o, l, ns = run("fp8", pol, x, y)
        rel = [((a - b).norm() / b.norm()).item() for a, b in zip(o, ref)]
        print(f"fp8 {pol:8s} sites={ns} losses", [round(v, 4) for v in l], "logit relL2 per step",
              [round(r, 4) for r in rel])


if __name__ == "__main__":
    main()
