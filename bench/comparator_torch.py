"""Comparator: the reference's own code path on stock PyTorch-ROCm.

BASELINE.md protocol: DistributedDataParallel (25 MiB buckets) + SyncBatchNorm
+ MIOpen convolutions with ``cudnn.benchmark=True`` + foreach SGD-nesterov
(reference main.py:42-59, 97-110), patched only where the reference cannot
run the target config: ImageNet stem + 1000 classes for 224x224, bf16
autocast, synthetic on-device data.  channels_last is used because it is the
fast MIOpen layout for bf16 on gfx950.

Launch like bench.py (single process, or torch.distributed.run for N>1).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_multiprocessing_distributed_amd.models import build_model  # noqa: E402


def measure_stock(model_name="resnet50", batch=256, image=224, steps=20, warmup=10, dev=None,
                  channels_last=True, ddp_device=None):
    """Images/sec of the reference's code path on stock PyTorch-ROCm on ``dev``
    (per process; DDP + SyncBN when torch.distributed is initialised with
    ``ddp_device``).  Used by ``bench.py --with_stock`` so the comparator is
    measured in the same run, on the same box, as the framework."""
    dev = dev or torch.device("cuda", torch.cuda.current_device())
    torch.backends.cudnn.benchmark = True
    model = build_model(model_name, num_classes=1000, stem="imagenet", impl="stock").to(dev)
    mf = torch.channels_last if channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    if ddp_device is not None:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
        model = nn.parallel.DistributedDataParallel(model, device_ids=[ddp_device])
    crit = nn.CrossEntropyLoss().to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4,
                          nesterov=True, foreach=True)
    x = torch.randn(batch, 3, image, image, device=dev).to(memory_format=mf)
    y = torch.randint(0, 1000, (batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = crit(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    import sys
    import threading
    tw = time.perf_counter()
    done = threading.Event()

    def heartbeat():                      # MIOpen's find prints nothing for minutes
        while not done.wait(30.0):
            print(f"[stock] ... {time.perf_counter() - tw:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(warmup):
        step()
        torch.cuda.synchronize()
        # progress (the first steps run MIOpen's find for every conv shape: minutes)
        print(f"[stock] warmup step {i + 1}/{warmup} done at {time.perf_counter() - tw:.0f} s",
              file=sys.stderr, flush=True)
    done.set()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del model, opt, x, y
    torch.cuda.empty_cache()
    return batch * steps / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--profile", default="")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", local)
    model = build_model(a.model, num_classes=1000, stem="imagenet", impl="stock").to(dev)
    mf = torch.contiguous_format if a.no_channels_last else torch.channels_last
    model = model.to(memory_format=mf)
    if world > 1:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
        model = nn.parallel.DistributedDataParallel(model, device_ids=[local])
    crit = nn.CrossEntropyLoss().to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4,
                          nesterov=True, foreach=True)
    x = torch.randn(a.batch, 3, a.image, a.image, device=dev).to(memory_format=mf)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
            loss = crit(out, y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    if rank == 0:
        ips = a.batch * world * a.steps / dt
        print(json.dumps({"metric": "comparator_stock_torch_images_per_sec", "value": round(ips, 1),
                          "n_gpus": world, "ms_per_step": round(1000 * dt / a.steps, 3),
                          "model": a.model, "batch_per_gpu": a.batch,
                          "channels_last": not a.no_channels_last, "loss": float(loss)}))
    if a.profile and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for _ in range(3):
                step()
            torch.cuda.synchronize()
        with open(a.profile, "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
