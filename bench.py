"""Flagship benchmark: ResNet-50 (ImageNet stem, 224x224, 1000 classes) bf16
training throughput, one process per MI355X, synchronous data parallel with
SyncBN + bucketed RCCL gradient all-reduce, fused SGD-nesterov -- the
BASELINE.json metric/config.  Synthetic on-device data, random-init weights.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Every rank does W untimed steps, then K timed steps bracketed by a barrier +
device synchronize on both sides; the step time is the MAX over ranks and
rank 0 prints ONE JSON line.  Per-GPU batch is fixed (256) -> weak scaling.
Each timed step is the full step: forward, loss, backward with overlapped
gradient all-reduce, optimizer update (nothing cached or skipped).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("images/sec (whole node) ResNet-50 224×224 bf16 at 1/2/4/8 MI355X; "
          "DDP scaling efficiency")
# stock PyTorch-ROCm reference path (DDP+SyncBN+MIOpen, bench/comparator_torch.py),
# re-measured on one MI355X at per-GPU batch 256 in round 5, in the same process as a
# 13,386 img/s run of ours (profiles/bench_r05_with_stock.jsonl; round 1: 6612.5); reported
# as a RECORDED figure unless --with_stock measures it in the same run
STOCK_IPS_PER_GPU_RECORDED = 6622.0
STOCK_RECORDED_SOURCE = "profiles/bench_r05_with_stock.jsonl (1x MI355X, round 5, same lease as ours)"
_MODEL_NAMES = {"resnet50": "ResNet-50", "resnet101": "ResNet-101", "resnet152": "ResNet-152",
                "resnet34": "ResNet-34", "resnet18": "ResNet-18-ref", "res": "ResNet-18-ref"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--stem", default="imagenet", choices=["imagenet", "cifar"],
                    help="cifar = the reference's 3x3 stem (ResNet-18-ref CIFAR shapes: --model res "
                         "--image 32 --classes 10)")
    ap.add_argument("--sync_bn", default="on", choices=["on", "off"])
    ap.add_argument("--bucket_mb", type=float, default=25.0)
    ap.add_argument("--first_bucket_mb", type=float, default=1.0)
    ap.add_argument("--last_bucket_mb", type=float, default=2.0,
                    help="cap of the last bucket (earliest layers, launched at the end of backward)")
    ap.add_argument("--syncbn_comm", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="SyncBN statistics transport (auto: one-shot xGMI kernel when W>1)")
    ap.add_argument("--grad_compress", default="none", choices=["none", "bf16"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8 = BASELINE config 5: every block conv's forward, data gradient and "
                         "weight gradient on the scaled fp8 MFMA (e4m3 weights/activations, e5m2 "
                         "gradients, delayed per-tensor scaling); stem, classifier, BN in bf16/fp32")
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend for W>1 (auto: nccl = RCCL)")
    ap.add_argument("--same_device", action="store_true",
                    help="W>1 ranks all on GPU 0 (with --backend gloo: rehearses the exact "
                         "multi-rank code path -- DataParallel, native reducer, xGMI SyncBN -- "
                         "on a one-GPU box; not a throughput number)")
    ap.add_argument("--comm", default="auto", choices=["auto", "c10d", "rccl"],
                    help="gradient-bucket transport: auto = the native RCCL communicator "
                         "(csrc/runtime/rccl_comm.cpp) when it can be the only in-step communicator "
                         "and its self-test passes, else torch ProcessGroupNCCL (c10d)")
    ap.add_argument("--dp_rehearsal", action="store_true",
                    help="W=1 only: run the production W>1 per-rank step on a single-rank process "
                         "group -- DataParallel hooks, native reducer, bucket all-reduces (--comm), "
                         "SyncBN through the one-shot xGMI kernel -- to measure its per-rank cost")
    ap.add_argument("--tune_table", default="",
                    help="kernel tuning table loaded before warmup: '' = the committed table(s) for "
                         "this device (ops/tables/, deterministic kernel choices), 'online' = "
                         "autotune every shape in step 0, or a JSON path (ops/tuning.py)")
    ap.add_argument("--save_tune_table", default="", help="rank 0 writes the tuning table after warmup")
    ap.add_argument("--with_stock", action="store_true",
                    help="also measure the stock PyTorch-ROCm comparator in this run (W=1)")
    ap.add_argument("--timeline", action="store_true",
                    help="print the gradient-bucket launch/overlap timeline of the last step")
    ap.add_argument("--profile", default="", help="write a torch.profiler table here (rank 0)")
    ap.add_argument("--data_prefetch", default="on", choices=["on", "off"],
                    help="two-stream steps: generate each synthetic batch one step ahead on the side stream")
    ap.add_argument("--step_mode", default="auto", choices=["auto", "two_stream", "one_stream", "graph"],
                    help="GPU step schedule (engine/train.py resolve_step_mode): auto = two_stream for the "
                         "224x224 headline, graph (W=1) / one_stream (W>1) for small images")
    ap.add_argument("--host_profile", default="",
                    help="after the timed run: cProfile the host side of 10 more steps (rank 0) and "
                         "write the top functions by own time here")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def syncbn_label(comm, sync_bn):
    """What actually carried the SyncBN statistics: the one-shot xGMI kernel, or
    the process group's own backend (RCCL = torch 'nccl', or gloo)."""
    if comm is None or sync_bn != "on":
        return None
    if comm.xgmi is not None:
        return "xgmi"
    return {"nccl": "rccl"}.get(comm.backend, comm.backend)


def native_build_info():
    """Provenance of the loaded extension (library digest and compile flags): a variant
    build (e.g. the timing-only -DPMD_TIMING_NO_ATOMICS) is refused at import unless
    PMD_ALLOW_VARIANT=1, and shows here when it was allowed."""
    from pytorch_multiprocessing_distributed_amd.ops import native
    return native.stamp_info()


def bench_rank(rank, world, a):
    from pytorch_multiprocessing_distributed_amd import launch
    from pytorch_multiprocessing_distributed_amd.data.loader import SyntheticImageNet
    from pytorch_multiprocessing_distributed_amd.engine.train import setup_syncbn
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel

    rehearsal = a.dp_rehearsal and world == 1
    if world > 1 or rehearsal:
        backend = "nccl" if a.backend == "auto" else a.backend
        if a.same_device or rehearsal:
            os.environ["LOCAL_RANK"] = "0"
        if rehearsal:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dev = launch.init_process(rank, world, backend, "cuda")
    else:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
    if not (world > 1 or rehearsal):
        # (init_process does this for the distributed runs, before the process group exists)
        OF.init_step_streams(dev)
    torch.manual_seed(0)
    model = build_model(a.model, num_classes=a.classes, stem=a.stem).to(dev)
    if rehearsal:
        # the W>1 machinery on a single-rank group: get_comm() would return None at W=1
        from pytorch_multiprocessing_distributed_amd.parallel.comm import Comm
        comm = Comm()
        if a.syncbn_comm == "auto":
            a.syncbn_comm = "xgmi"          # the production W>1 SyncBN transport
    else:
        comm = get_comm()
    setup_syncbn(comm, a.sync_bn, a.syncbn_comm, True)
    from pytorch_multiprocessing_distributed_amd.engine.train import GraphedStep, resolve_step_mode
    step_mode = resolve_step_mode(a.step_mode, 2 if rehearsal else world, True, a.image, a.dtype)
    OF.set_wgrad_stream(step_mode == "two_stream")
    model = DataParallel(model, comm, bucket_mb=a.bucket_mb, first_bucket_mb=a.first_bucket_mb,
                         compress=a.grad_compress, transport=a.comm if comm is not None else "c10d",
                         timeline=a.timeline, last_bucket_mb=a.last_bucket_mb)
    if a.dtype == "fp8":
        from pytorch_multiprocessing_distributed_amd.ops.fp8 import Fp8Scaling
        OF.set_fp8(Fp8Scaling(dev))
    opt = FusedSGD(model, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    data = SyntheticImageNet(a.batch, a.image, a.classes, steps=a.warmup + a.steps, device=dev,
                             dtype=torch.bfloat16, cpad=8, seed=rank)
    model.train()
    # kernel choices fixed before anything runs
    from pytorch_multiprocessing_distributed_amd.ops import tuning
    if a.tune_table == "online":
        tune_source = "online"
    elif a.tune_table:
        tuning.load(a.tune_table)
        tune_source = "table:" + os.path.basename(a.tune_table)
    else:
        tune_source, _ = tuning.load_default()

    graphed = {}

    prefetch = step_mode == "two_stream" and a.data_prefetch == "on"
    if prefetch:
        # each step's batch is generated one step ahead on the side stream (idle in the forward)
        data.prefetch(OF._wgrad_stream(dev), transform=OF.s2d_input_prefetch(model))

    def step(i):
        x, y = data.next_batch(i) if prefetch else data.batch_at(i)
        g = graphed.get("g")
        if g is not None:
            return g(x, y)[1]               # the captured step, replayed on this batch
        out = model(x)
        loss = OF.cross_entropy(out, y)
        opt.zero_grad()
        loss.backward(OF.loss_seed(loss))
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
        if i == 0 and comm is not None:
            tuning.sync(comm.group)         # every rank runs rank 0's kernel choices
    if step_mode == "graph":
        # captured after the eager warmup (kernel choices tuned, lazy state initialised) and
        # before the timed region, whose every step is then one copy-in + one graph replay
        x, y = data.batch_at(0)
        graphed["g"] = GraphedStep(model, opt, x, y)
    if a.save_tune_table and rank == 0:
        tuning.save(a.save_tune_table)
    torch.cuda.synchronize()
    if comm is not None:
        comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    from pytorch_multiprocessing_distributed_amd.utils import trace as _trace
    sync_debug = _trace.sync_debug_enabled()
    for i in range(a.steps):
        loss = step(a.warmup + i)
        if comm is not None:
            comm.raise_if_failed()          # host-mapped xGMI error word, no device sync
        if sync_debug:
            _trace.check_stream_budget(comm, model)
    # host time to ENQUEUE the timed steps (nothing in the loop waits on the device): when
    # it approaches ms_per_step the step is launch-/host-bound, not device-bound
    host_dt = time.perf_counter() - t0
    torch.cuda.synchronize()
    if comm is not None:
        comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if comm is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    final_loss = float(loss.item())
    # host cost of ONE step from an idle device (nothing queued ahead, so no enqueue ever
    # blocks on a full hardware queue): the pure host side of the step, after the timed
    # region; host_enqueue_ms_per_step above includes such blocking once the host runs
    # ahead of the device
    iso = []
    for i in range(3):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step(i)
        iso.append(time.perf_counter() - t1)
        if comm is not None:
            comm.raise_if_failed()
    torch.cuda.synchronize()
    host_iso_ms = 1000.0 * min(iso)
    if comm is not None and comm.xgmi is not None:
        comm.xgmi.check()         # raises if any statistics exchange timed out
    choice_hash = tuning.table_hash()
    if a.timeline and rank == 0 and comm is not None:
        for row in model.bucket_timeline():
            print("[bench] bucket %d: host launch %.0f us after first grad, finalize at %.0f us; "
                  "device all-reduce %.3f .. %.3f ms vs end of backward" % row, file=sys.stderr)
    stock = None
    if a.with_stock and world == 1 and a.dtype == "bf16":
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from comparator_torch import measure_stock
        stock = measure_stock(a.model, a.batch, a.image, steps=max(a.steps, 10), warmup=5, dev=dev)
    if rank == 0:
        ips = a.batch * world * a.steps / dt
        model_name = _MODEL_NAMES.get(a.model.lower(), a.model)
        metric = METRIC if (model_name == "ResNet-50" and a.dtype == "bf16" and a.image == 224) else (
            f"images/sec (whole node) {model_name} {a.image}×{a.image} {a.dtype} at 1/2/4/8 MI355X; "
            "DDP scaling efficiency")
        parallelism = f"dp{world}"
        if world > 1 and a.same_device:
            parallelism += f"-same-gpu-{dist.get_backend()}"
        if rehearsal:
            parallelism += "-rehearsal"
        rec = {
            "metric": metric, "value": round(ips, 1), "unit": "images/sec",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic (ImageNet-shaped batches generated on device every step" +
                    (", one step ahead on the side stream" if prefetch else "") + "; random-init weights)",
            "config": {"model": model_name, "global_batch": a.batch * world,
                       "seq_len": None,
                       "image_size": a.image, "per_gpu_batch": a.batch,
                       "parallelism": parallelism,
                       "sync_bn": a.sync_bn == "on" and (world > 1 or rehearsal),
                       "bucket_mb": a.bucket_mb, "step_mode": step_mode,
                       "syncbn_comm": syncbn_label(comm, a.sync_bn),
                       "syncbn_ordering": (comm.xgmi.ordering if comm is not None and comm.xgmi is not None
                                           else None),
                       "grad_compress": a.grad_compress,
                       "grad_transport": model.transport,
                       "grad_buckets_mb": ([round(m, 2) for m in model.bucket_sizes_mb()]
                                           if comm is not None else None)},
            "final_loss": round(final_loss, 4),
            "tune_source": tune_source,
            "kernel_choice_hash": choice_hash,
            **native_build_info(),
            "host_enqueue_ms_per_step": round(1000.0 * host_dt / a.steps, 3),
            "host_ms_per_step_idle_device": round(host_iso_ms, 3),
        }
        if stock is not None:
            rec["stock_pytorch_rocm_ips_measured"] = round(stock, 1)
            rec["vs_stock_pytorch_rocm_measured"] = round(ips / stock, 3)
        elif model_name == "ResNet-50" and a.dtype == "bf16" and world == 1:
            rec["vs_stock_pytorch_rocm_recorded"] = round(ips / STOCK_IPS_PER_GPU_RECORDED, 3)
            rec["stock_recorded_source"] = STOCK_RECORDED_SOURCE
        print(json.dumps(rec), flush=True)
    if a.host_profile:
        # host cost of the step alone (the JSON above is unaffected): where the enqueue
        # time goes, per Python function and per native call, over 10 steps
        import cProfile
        import io
        import pstats
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for i in range(10):
            step(i)
            if comm is not None:
                comm.raise_if_failed()
        pr.disable()
        torch.cuda.synchronize()
        if rank == 0:
            buf = io.StringIO()
            pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(60)
            pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(60)
            with open(a.host_profile, "w") as f:
                f.write(f"# bench.py host profile, 10 steps, {a.model} batch {a.batch}, "
                        f"parallelism {parallelism}\n")
                f.write(buf.getvalue())
    if a.profile and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            for i in range(3):
                step(i)
            torch.cuda.synchronize()
        with open(a.profile, "w") as f:
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=80))
    if world > 1 or rehearsal:
        model.close()           # the native reducer holds the process group: release it first
        launch.shutdown()


def _spawn_entry(rank, world, a):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    os.environ["LOCAL_RANK"] = str(rank)
    bench_rank(rank, world, a)


def main():
    a = parse()
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        if world != a.gpus and rank == 0:
            print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
                  file=sys.stderr)
        bench_rank(rank, world, a)
    elif a.gpus > 1:
        import torch.multiprocessing as mp
        mp.spawn(_spawn_entry, args=(a.gpus, a), nprocs=a.gpus, join=True)
    else:
        bench_rank(0, 1, a)


if __name__ == "__main__":
    main()
