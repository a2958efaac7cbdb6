"""Run-to-run determinism probe of the W=8 step rehearsed on ONE GPU (8 processes, gloo process
group, SyncBN over the xGMI kernel, native reducer): every rank repeats the same ResNet-18-ref
training step (same batch, grads zeroed, no optimizer) N times in the deterministic statistics
mode with unshifted BN sums (PMD_BN_SHIFT=0), so every iteration after the first (which ends
with the ready-order arena relayout, i.e. new bucket bounds) must give bit-identical gradients;
any tensor that differs from iteration 1 names a hand-off race.

    python bench/w8_race.py [--world 8] [--iters 6] [--syncbn xgmi|gloo] [--wgrad_stream 1|0]
"""
import argparse
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, a, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["PMD_BN_SHIFT"] = "0"
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel import dp as DP
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    OF.init_step_streams(dev)
    OF.set_wgrad_stream(a.wgrad_stream == 1)
    OF.set_deterministic(not a.fresh)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    if a.syncbn == "xgmi":
        comm.enable_xgmi(timeout_s=20.0)
        comm.xgmi.select_ordering(verbose=False)
    OF.set_bn_sync(comm)
    if a.tables:
        from pytorch_multiprocessing_distributed_amd.ops import tuning
        tuning.load_default()
    x, y = C.synth_images(8 * world, 32, 32, 8, 3, 10, 7, 0)
    if a.fresh:
        per = x.shape[0] // world
        xs, ys = x[rank * per:(rank + 1) * per].contiguous(), y[rank * per:(rank + 1) * per].contiguous()
        g0, report = None, []
        for r in range(a.fresh):
            torch.manual_seed(0 if rank == 0 else 77 + r)
            m = build_model("res", num_classes=10, stem="cifar").cuda()
            dpm = DP.DataParallel(m, comm, bucket_mb=1.0, first_bucket_mb=0.25)
            dpm.train()
            loss = OF.cross_entropy(dpm(xs), ys)
            loss.backward()
            torch.cuda.synchronize()
            g = {n: p.grad.detach().float().cpu().clone() for n, p in dpm.module.named_parameters()}
            if g0 is None:
                g0 = g
                continue
            rel = {n: ((g0[n] - g[n]).norm() / g0[n].norm().clamp_min(1e-30)).item() for n in g}
            worst = sorted(((v, n) for n, v in rel.items()), reverse=True)[:3]
            report.append((r, [f"{n} {v:.2e}" for v, n in worst], -2 if worst[0][0] > 1e-2 else -3))
            del dpm, m
        q.put((rank, report))
        OF.set_bn_sync(None)
        dist.destroy_process_group()
        return
    torch.manual_seed(0)
    model = build_model("res", num_classes=10, stem="cifar").cuda()
    per = x.shape[0] // world
    dpm = DP.DataParallel(model, comm, bucket_mb=1.0, first_bucket_mb=0.25)
    dpm.train()
    xs, ys = x[rank * per:(rank + 1) * per].contiguous(), y[rank * per:(rank + 1) * per].contiguous()
    ref = None
    report = []
    for it in range(a.iters):
        dpm.module.zero_grad(set_to_none=False)
        for p in dpm.module.parameters():
            if p.grad is not None:
                p.grad.zero_()
        loss = OF.cross_entropy(dpm(xs), ys)
        loss.backward()
        torch.cuda.synchronize()
        g = {n: p.grad.detach().float().cpu().clone() for n, p in dpm.module.named_parameters()}
        g["loss"] = loss.detach().float().cpu().reshape(1).clone()
        if it == 0:
            g0 = g
            continue          # iteration 1 re-lays the arena out in ready order (new buckets)
        if ref is None:
            ref = g
            # iteration 0 (online tuning unless --tables, first-step state) vs 1: relative size
            rel = {n: ((g0[n] - g[n]).norm() / g[n].norm().clamp_min(1e-30)).item() for n in g}
            worst = sorted(((v, n) for n, v in rel.items()), reverse=True)[:3]
            report.append((0, [f"{n} {v:.2e}" for v, n in worst], -1))
        else:
            bad = [n for n in ref if not torch.equal(ref[n], g[n])]
            report.append((it, bad[:8], len(bad)))
    q.put((rank, report))
    OF.set_bn_sync(None)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--syncbn", default="xgmi", choices=["xgmi", "gloo"])
    ap.add_argument("--wgrad_stream", type=int, default=1)
    ap.add_argument("--tables", type=int, default=0, help="1: load the committed tuning tables (no online tuning)")
    ap.add_argument("--fresh", type=int, default=0,
                    help="N > 0: N repetitions of a FRESH DataParallel's first step (ranks != 0 start from "
                         "other weights; rank-0 broadcast), statistics in the production (atomic) mode; "
                         "reports each repetition's largest relative gradient difference from repetition 0")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    mp.spawn(worker, args=(a.world, _free_port(), a, q), nprocs=a.world, join=True)
    res = sorted(q.get() for _ in range(a.world))
    nbad = 0
    for rank, rep in res:
        for it, names, n in rep:
            if n == -2 or (n == -3 and rank == 0):
                print(f"rank {rank} repetition {it} vs 0{' GROSS' if n == -2 else ''}: {names}")
                nbad += n == -2
            elif n < 0:
                print(f"rank {rank} iteration 0 vs 1, largest relative differences: {names}")
            elif n:
                nbad += 1
                print(f"rank {rank} iteration {it}: {n} tensors differ from iteration 1, e.g. {names}")
    print(f"[w8_race] world {a.world} syncbn {a.syncbn} wgrad_stream {a.wgrad_stream}: "
          f"{nbad} (rank, iteration) pairs differ out of {a.world * (a.iters - 2)}", flush=True)


if __name__ == "__main__":
    main()
