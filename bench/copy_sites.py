"""Where do the per-step device copies (``__amd_rocclr_copyBuffer`` in a rocprofv3 trace)
come from?  Runs bench.py's ResNet-50 step under torch.profiler with Python stacks and
prints every Memcpy / Memset event of ONE steady-state step with the innermost frames of
the framework code that issued it.

    python bench/copy_sites.py [--steps 1] [--model resnet50] [--batch 256] [--rehearsal]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    torch.manual_seed(0)
    model = DataParallel(build_model(a.model, num_classes=1000, stem="imagenet").to(dev), None)
    opt = FusedSGD(model, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    data = SyntheticImageNet(a.batch, 224, 1000, steps=10, device=dev, dtype=torch.bfloat16, cpad=8)
    tuning.load_default()
    model.train()

    def step(i):
        x, y = data.batch_at(i)
        loss = OF.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward(OF.loss_seed(loss))
        opt.step()

    for i in range(4):
        step(i)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(a.steps):
            step(4 + i)
        torch.cuda.synchronize()
    evs = prof.events()
    by_id = {e.id: e for e in evs}
    rows = collections.Counter()
    for e in evs:
        name = e.name
        if not ("Memcpy" in name or "Memset" in name or "copyBuffer" in name or "fillBuffer" in name):
            continue
        # walk up to the CPU op that launched it and print its framework frames
        cpu = e.cpu_parent if getattr(e, "cpu_parent", None) is not None else None
        chain = []
        c = cpu
        while c is not None and len(chain) < 6:
            chain.append(c.name)
            c = c.cpu_parent
        stack = [f for f in (cpu.stack if cpu is not None and cpu.stack else [])
                 if "pytorch_multiprocessing_distributed_amd" in f or "bench" in f][:4]
        rows[(name, " <- ".join(chain[:3]), " | ".join(stack))] += 1
    print(f"# device copies / fills per step ({a.steps} step(s) profiled, {a.model} bs{a.batch})")
    for (name, chain, stack), n in rows.most_common():
        print(f"{n / a.steps:6.1f}  {name}\n        ops: {chain}\n        at: {stack}")
    print(prof.key_averages(group_by_stack_n=4).table(sort_by="cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
