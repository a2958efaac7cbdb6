"""Eager vs HIP-graph replay of one training step at a given model / batch (single GPU):
the launch-bound small configurations (the reference's own CIFAR-10 ResNet18 at batch 32) are
where a captured step can win; at ResNet-50 bs256 the eager step is device-bound and the
graph executor's queue re-dealing loses (profiles/hip_graph_r05.txt).

    python bench/graph_step.py --model res --stem cifar --batch 32 --image 32 --classes 10
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="res")
    ap.add_argument("--stem", default="cifar")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--image", type=int, default=32)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    OF.init_step_streams(dev)
    tuning.load_default()
    torch.manual_seed(0)
    model = DataParallel(build_model(a.model, num_classes=a.classes, stem=a.stem).to(dev), None)
    opt = FusedSGD(model, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    data = SyntheticImageNet(a.batch, a.image, a.classes, steps=a.warmup + a.steps, device=dev,
                             dtype=torch.bfloat16, cpad=8, seed=0)
    model.train()

    def step_on(x, y):
        out = model(x)
        loss = OF.cross_entropy(out, y)
        opt.zero_grad()
        loss.backward(OF.loss_seed(loss))
        opt.step()
        return loss

    def timed(fn):
        for i in range(a.warmup):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            loss = fn(a.warmup + i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps, float(loss)

    eager_dt, eager_loss = timed(lambda i: step_on(*data.batch_at(i)))

    opt.graph_safe()
    sx, sy = data.batch_at(0)
    sx, sy = sx.clone(), sy.clone()
    main = torch.cuda.current_stream()
    for _ in range(3):                       # warm the capture's allocations and streams
        step_on(sx, sy)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=main):
        static_loss = step_on(sx, sy)
    torch.cuda.synchronize()

    def replay(i):
        x, y = data.batch_at(i)
        sx.copy_(x)
        sy.copy_(y)
        graph.replay()
        return static_loss
    graph_dt, graph_loss = timed(replay)
    rec = {"model": a.model, "batch": a.batch, "image": a.image,
           "eager_ms": round(1e3 * eager_dt, 3), "eager_img_s": round(a.batch / eager_dt, 1),
           "graph_ms": round(1e3 * graph_dt, 3), "graph_img_s": round(a.batch / graph_dt, 1),
           "eager_loss": eager_loss, "graph_loss": graph_loss}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
