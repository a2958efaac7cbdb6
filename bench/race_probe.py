"""Run-to-run determinism of the 2-rank (one GPU, gloo) data-parallel step under
configurable schedules: prints, per step, the relative L2 between two runs of
the SAME configuration (BN in eval mode, lr 0: only fp32-atomic ordering
should differ).  Used to localise scheduling races.

    python bench/race_probe.py "name:ENV=V,ENV=V:rebuild" ...
"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out, env, rebuild):
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    OF._WGRAD_STREAM["on"] = env.get("PMD_WGRAD_STREAM", "1") != "0"
    OF._WGRAD_STREAM["defer"] = int(env.get("PMD_WGRAD_DEFER", "1"))
    comm = get_comm()
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=10, stem="imagenet").cuda()
    dp = DataParallel(model, comm, bucket_mb=2.0, first_bucket_mb=0.5, rebuild_buckets=rebuild)
    dp.module.eval()
    opt = FusedSGD(dp, lr=0.0, momentum=0.9, nesterov=True)
    x, _ = C.synth_images(8, 64, 64, 8, 3, 10, 11, 0)
    y = torch.arange(8, device="cuda") % 10
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    grads = []
    for _ in range(4):
        loss = OF.cross_entropy(dp(xs), ys)
        opt.zero_grad()
        loss.backward()
        opt.step()
        grads.append({n: p.grad.detach().float().cpu() for n, p in dp.module.named_parameters()})
    torch.cuda.synchronize()
    if rank == 0:
        torch.save(grads, out)
    dist.destroy_process_group()


def rel(x, y):
    num = sum(((x[k] - y[k]) ** 2).sum() for k in x)
    den = sum((y[k] ** 2).sum() for k in y)
    return (num / den).sqrt().item()


def main():
    for spec in sys.argv[1:]:
        name, envs, rb = spec.split(":")
        env = dict(kv.split("=") for kv in envs.split(",") if kv)
        runs = []
        for i in range(2):
            out = f"/tmp/race_{name}_{i}.pt"
            mp.spawn(worker, args=(2, _port(), out, env, rb == "1"), nprocs=2, join=True)
            runs.append(torch.load(out, weights_only=True))
        print(name, env, "rebuild" if rb == "1" else "no-rebuild",
              [f"{rel(a, b):.2e}" for a, b in zip(runs[0], runs[1])], flush=True)
        worst = sorted(((rel({k: runs[0][1][k]}, {k: runs[1][1][k]}), k) for k in runs[0][1]),
                       reverse=True)[:4]
        print("   step-1 worst tensors:", [(k, f"{e:.2e}") for e, k in worst], flush=True)


if __name__ == "__main__":
    main()
