"""Diagnose whole-model gradient agreement: per-parameter relative L2 between
(a) the gfx950 path and the fp32 torch-prims oracle, and (b) the fp32 oracle
and itself on an input perturbed at bf16 rounding level (chaos floor).

    python bench/oracle_probe.py [--batch 32] [--image 224] [--classes 1000]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import ResNet50  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops import functional as OF  # noqa: E402
from pytorch_multiprocessing_distributed_amd.ops.native import C  # noqa: E402


def grads(m, x, y, torch_prims):
    OF.force_torch_prims(torch_prims)
    try:
        m.zero_grad(set_to_none=True)
        loss = OF.cross_entropy(m(x), y)
        loss.backward()
    finally:
        OF.force_torch_prims(False)
    return float(loss), {n: p.grad.detach().double().clone() for n, p in m.named_parameters()}


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--gamma3", type=float, default=-1.0, help="init every block's last BN gamma")
    ap.add_argument("--eval", action="store_true", help="BN in eval mode (running statistics)")
    ap.add_argument("--summary", action="store_true")
    a = ap.parse_args()
    torch.manual_seed(0)
    m0 = ResNet50(num_classes=a.classes, stem="imagenet").cuda()
    m0.train(not a.eval)
    if a.gamma3 >= 0:
        for mod in m0.modules():
            if hasattr(mod, "bn3"):
                torch.nn.init.constant_(mod.bn3.weight, a.gamma3)
    x, y = C.synth_images(a.batch, a.image, a.image, 8, 3, a.classes, 7, 0)
    runs = {}
    runs["hip"] = grads(copy.deepcopy(m0), x, y, False)
    runs["f32"] = grads(copy.deepcopy(m0), x.float(), y, True)
    runs["f32b"] = grads(copy.deepcopy(m0), x.float(), y, True)    # determinism of the oracle
    xp = x.float() * (1 + 2 ** -9 * torch.randn_like(x.float()))
    runs["f32p"] = grads(copy.deepcopy(m0), xp, y, True)           # chaos floor
    runs["bf16tp"] = grads(copy.deepcopy(m0), x, y, True)          # torch prims on bf16 activations
    print(f"gamma3={a.gamma3} eval={a.eval} losses", {k: v[0] for k, v in runs.items()})
    ref = runs["f32"][1]
    if a.summary:
        for k in ("hip", "f32b", "f32p", "bf16tp"):
            e = sorted(rel(runs[k][1][n], ref[n]) for n in ref)
            print(f"  {k:7} median {e[len(e) // 2]:.2e}  p90 {e[int(len(e) * 0.9)]:.2e}  max {e[-1]:.2e}")
        return
    print(f"{'param':40} {'hip':>9} {'f32b':>9} {'f32pert':>9} {'bf16tp':>9} {'hip-vs-bf16tp':>13}")
    for n in ref:
        print(f"{n:40} {rel(runs['hip'][1][n], ref[n]):9.2e} {rel(runs['f32b'][1][n], ref[n]):9.2e} "
              f"{rel(runs['f32p'][1][n], ref[n]):9.2e} {rel(runs['bf16tp'][1][n], ref[n]):9.2e} "
              f"{rel(runs['hip'][1][n], runs['bf16tp'][1][n]):13.2e}")


if __name__ == "__main__":
    main()
