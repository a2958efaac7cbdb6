"""Training engine: per-rank orchestration, train and validate epochs.

Mirrors the reference's L5 (main.py:32-171) with the same stdout formats and
log files, minus its bugs: the LR schedule steps on every rank
(B4), the sampler epoch advances (B5, ``--fixed_order`` keeps the reference
behaviour), and test accuracy is all-reduced over ranks (B2,
``--compat_metrics`` reproduces the reference number).  The hot loop keeps
loss/accuracy on the device and only synchronises when it prints.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from .. import launch
from ..data.cifar import get_cifar10
from ..data.loader import DeviceLoader, SyntheticImageNet
from ..models import build_model
from ..ops import functional as OF
from ..utils.trace import check_stream_budget, region, sync_debug_enabled
from ..parallel.comm import get_comm
from ..parallel.dp import DataParallel
from ..utils.checkpoint import load_resume, save_model, save_resume
from ..utils.logger import DeviceMeter, Logger
from .optim import FusedSGD


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def build_loaders(args, rank, world, dev, dtype, cpad):
    if args.stem == "imagenet":
        tr = SyntheticImageNet(int(args.batch_size / world), args.image_size, args.num_classes,
                               steps=args.max_steps or args.steps_per_epoch, device=dev,
                               dtype=dtype, cpad=cpad, seed=1234 + rank)
        te = SyntheticImageNet(int(args.batch_size / world), args.image_size, args.num_classes,
                               steps=args.eval_batches or 2, device=dev, dtype=dtype, cpad=cpad,
                               seed=99991 + rank, dataset_len=50000)
        return tr, te
    xtr, ytr = get_cifar10(args.data_root, True, args.synthetic, args.train_samples)
    xte, yte = get_cifar10(args.data_root, False, args.synthetic,
                           None if args.train_samples is None else max(args.train_samples // 5, 1))
    tr = DeviceLoader(xtr, ytr, args.batch_size, world, rank, train=True, device=dev, dtype=dtype,
                      cpad=cpad, fixed_order=args.fixed_order, max_batches=args.max_steps)
    te = DeviceLoader(xte, yte, args.batch_size, world, rank, train=False, device=dev, dtype=dtype,
                      cpad=cpad, shuffle=False, max_batches=args.eval_batches)
    if rank == 0:
        print("-------------------Make loader-------------------")
        print("Train Dataset :", tr.dataset_len, "   Test Dataset :", te.dataset_len)
    return tr, te


def _first_step_tuning(args, rank, comm):
    """After the first step every conv shape has been met (and tuned): adopt rank
    0's kernel choices on every rank (cudnn.benchmark state made rank-consistent),
    and optionally persist them (ops/tuning.py)."""
    from ..ops import tuning
    if comm is not None:
        tuning.sync(comm.group)
    path = getattr(args, "save_tune_table", "")
    if path and rank == 0:
        tuning.save(path)


_SYNC_DEBUG = sync_debug_enabled()


def resolve_step_mode(mode, world, on_gpu, image_size, dtype):
    """The GPU step schedule (``--step_mode``).  A ResNet-50 step at 224x224 / batch 256 is
    device-bound: weight gradients on a side stream overlap the data-gradient chain
    (two_stream).  The reference's own CIFAR-10 ResNet18 step (32x32, batch 32 per GPU) is
    host-bound: ~1 ms of GPU work behind ~2 ms of launches, where the side stream's per-block
    fork/join events cost more than they overlap (one_stream: 1.40 vs 2.05 ms/step on one
    MI355X) and a captured HIP graph of the whole step removes the launch path altogether
    (graph: 0.99 ms/step, profiles/step_mode_r05.txt).  Graphs need one process (no
    collectives inside the capture) and bf16 (fp8 delayed scaling updates on the host)."""
    if not on_gpu:
        return "two_stream"
    if mode == "auto":
        small = image_size is not None and image_size <= 64
        if not small:
            return "two_stream"
        mode = "graph" if world == 1 else "one_stream"
    if mode == "graph" and (world != 1 or dtype == "fp8" or _SYNC_DEBUG):
        mode = "one_stream"
    return mode


class GraphedStep:
    """The whole training step (forward, loss, backward, fused SGD) captured ONCE as a HIP graph
    on the current stream and replayed for every later batch of the same shape: the inputs are
    copied into the captured buffers, the learning rate is device-resident
    (``FusedSGD.graph_safe``), and the BN running statistics, statistic slots and gradient
    arena are updated in place by the replay exactly as by an eager step."""

    def __init__(self, model, optimizer, inp, target):
        optimizer.graph_safe()
        self.opt = optimizer
        self.sx = inp.detach().clone()
        self.sy = target.detach().clone()
        self.shape = (tuple(inp.shape), tuple(target.shape))
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=torch.cuda.current_stream()):
            out = model(self.sx)
            loss = OF.cross_entropy(out, self.sy)
            optimizer.zero_grad()
            loss.backward(OF.loss_seed(loss))
            optimizer.step()
        optimizer.steps -= 1            # the capture recorded the step, it did not run it
        self.out, self.loss = out.detach(), loss.detach()

    def fits(self, inp, target):
        return (tuple(inp.shape), tuple(target.shape)) == self.shape

    def __call__(self, inp, target):
        self.sx.copy_(inp)
        self.sy.copy_(target)
        self.opt.sync_lr()
        self.graph.replay()
        self.opt.steps += 1
        return self.out, self.loss


def _graph_of(optimizer):
    """The optimizer's captured step (GraphedStep), or None.  Held BY the optimizer -- the
    object whose arenas, momentum and device LR the graph updates in place -- so a later model /
    optimizer in the same process never replays another's graph, and the graph and its memory
    pool are freed with them."""
    return getattr(optimizer, "_pmd_graph", None)


def train_epoch(loader, model, optimizer, epoch, logger, args, rank, dev, comm=None,
                step_offset=0):
    batch_time = DeviceMeter()
    data_time = DeviceMeter()
    losses = DeviceMeter()
    top1 = DeviceMeter()
    model.train()
    n = len(loader)
    end = time.time()
    t_epoch = time.time()
    images = 0
    graphed = getattr(args, "step_mode_resolved", "two_stream") == "graph"
    for i, (inp, target) in enumerate(loader):
        data_time.update(time.time() - end)
        launch.maybe_inject_fault(rank, step_offset + i)
        g = _graph_of(optimizer) if graphed else None
        if graphed and g is None and step_offset + i >= 2:
            # steps 0-1 ran eagerly: kernel choices tuned, lazy state initialised
            g = optimizer._pmd_graph = GraphedStep(model, optimizer, inp, target)
        if g is not None and g.fits(inp, target):
            with region("graph"):
                output, loss = g(inp, target)
        else:
            with region("fwd"):
                output = model(inp)
                loss = OF.cross_entropy(output, target)
            optimizer.zero_grad()
            with region("bwd"):
                loss.backward(OF.loss_seed(loss))
            with region("opt"):
                optimizer.step()
        if comm is not None:
            comm.raise_if_failed()      # xGMI SyncBN timeout of a finished step (no device sync)
        if _SYNC_DEBUG and dev.type == "cuda":
            check_stream_budget(comm, model)   # step work fits the hardware queues
        if step_offset + i == 0 and dev.type == "cuda":
            _first_step_tuning(args, rank, comm)
        if comm is not None and comm.order_check_every and (step_offset + i) % comm.order_check_every == 0:
            comm.verify_order(model.collective_signature())
        bsz = inp.size(0)
        images += bsz
        correct = OF.correct_count(output.detach(), target)
        losses.update(loss.detach(), bsz)
        top1.update(correct.float().squeeze(0) * (100.0 / bsz), bsz)
        if i % args.print_freq == 0 or i == n - 1:
            _sync(dev)
            if comm is not None:
                comm.raise_if_failed()
        batch_time.update(time.time() - end)
        end = time.time()
        if rank == 0 and i % args.print_freq == 0:
            print("Epoch: [{0}][{1}/{2}]\t"
                  "Time {batch_time.val:.3f} ({batch_time.avg:.3f})\t"
                  "Data {data_time.val:.3f} ({data_time.avg:.3f})\t"
                  "Loss {loss.val:.4f} ({loss.avg:.4f})\t"
                  "Prec {top1.val:.3f}% ({top1.avg:.3f}%)".format(
                      epoch, i, n, batch_time=batch_time, data_time=data_time, loss=losses,
                      top1=top1), flush=True)
    _sync(dev)
    if comm is not None:
        comm.raise_if_failed()          # everything of this epoch has completed now
    elapsed = time.time() - t_epoch
    world = comm.world_size if comm is not None else 1
    ips = images * world / max(elapsed, 1e-9)
    if rank == 0:
        logger.write([epoch, losses.avg, top1.avg])
        print(f"Epoch {epoch} throughput: {ips:.1f} images/sec (all ranks)", flush=True)
    return losses.avg, top1.avg, ips


@torch.no_grad()
def validate(loader, model, epoch, logger, args, rank, dev, comm=None, mode="test"):
    batch_time = DeviceMeter()
    losses = DeviceMeter()
    model.eval()
    total_correct = torch.zeros(1, dtype=torch.float64, device=dev)
    seen = torch.zeros(1, dtype=torch.float64, device=dev)
    end = time.time()
    n = len(loader)
    for i, (inp, target) in enumerate(loader):
        output = model(inp)
        loss = OF.cross_entropy(output, target)
        total_correct += OF.correct_count(output, target).double()
        seen += target.numel()
        losses.update(loss, inp.size(0))
        batch_time.update(time.time() - end)
        end = time.time()
        if rank == 0 and i % args.print_freq == 0:
            print(mode, ": [{0}/{1}]\t"
                  "Time {batch_time.val:.3f} ({batch_time.avg:.3f})\t"
                  "Loss {loss.val:.4f} ({loss.avg:.4f})".format(
                      i, n, batch_time=batch_time, loss=losses), flush=True)
    if args.compat_metrics or comm is None:
        # reference semantics (main.py:168): local correct / full dataset size
        denom = float(loader.dataset_len) if args.compat_metrics else float(seen.item())
        acc = 100.0 * total_correct.item() / max(denom, 1.0)
    else:
        buf = torch.cat([total_correct, seen])
        if dist.get_backend() == "gloo":
            buf = buf.cpu()
        comm.all_reduce_(buf)
        acc = 100.0 * float(buf[0]) / max(float(buf[1]), 1.0)
    if rank == 0:
        print("Accuracy {:.2f}".format(acc), flush=True)
        logger.write([epoch, losses.avg, float(acc)])
    return losses.avg, acc


def run_rank(rank, world_size, args):
    """Per-rank orchestrator (reference ``main(rank, world_size)``, main.py:32-84)."""
    dev = launch.init_process(rank, world_size, args.backend, args.device, args.master_addr,
                              args.master_port, args.timeout_min)
    try:
        _run(rank, world_size, args, dev)
    except BaseException:
        launch.abort()          # ncclCommAbort: peers blocked in a collective error out
        raise
    finally:
        launch.shutdown()


def setup_syncbn(comm, sync_bn="on", transport="auto", on_gpu=True):
    """Install the SyncBN communicator.  transport "xgmi" (or "auto" on GPU)
    maps the one-shot IPC all-reduce for the statistics vectors."""
    if comm is None or sync_bn != "on":
        OF.set_bn_sync(None)
        return None
    if transport == "xgmi" or (transport == "auto" and on_gpu and comm.backend == "nccl"):
        if not on_gpu:
            raise ValueError("--syncbn_comm xgmi needs GPU ranks")
        try:
            x = comm.enable_xgmi()
            # light -> strict memory ordering, picked by the interleaving stress self-test;
            # PMD_XGMI_ORDER=light|strict pins one (still stress-tested)
            pinned = os.environ.get("PMD_XGMI_ORDER", "")
            if pinned:
                x.set_ordering(pinned)
                if not (x.self_test() and x.stress_test()):
                    raise RuntimeError(f"xGMI stress self-test failed with the pinned {pinned} ordering")
            else:
                x.select_ordering()
        except Exception as e:  # noqa: BLE001
            if transport == "xgmi":
                raise
            # "auto": keep training on the RCCL transport, and say so
            comm.xgmi = None
            if comm.rank == 0:
                print(f"[pmd] one-shot xGMI SyncBN transport unavailable ({e}); using RCCL",
                      flush=True)
    OF.set_bn_sync(comm)
    return comm


def _run(rank, world_size, args, dev):
    on_gpu = dev.type == "cuda"
    dtype = torch.bfloat16 if (args.dtype in ("bf16", "fp8") or (args.dtype == "auto" and on_gpu)) \
        else torch.float32
    if on_gpu and dtype != torch.bfloat16:
        raise ValueError("the gfx950 kernels compute in bf16; use --dtype bf16 (or fp8) on GPU")
    if args.dtype == "fp8":
        if not on_gpu:
            raise ValueError("--dtype fp8 needs the gfx950 path (GPU)")
        from ..ops.fp8 import Fp8Scaling
        OF.set_fp8(Fp8Scaling(dev))
    cpad = 8 if on_gpu else 3
    train_loader, test_loader = build_loaders(args, rank, world_size, dev, dtype, cpad)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    if on_gpu:
        # deterministic kernel choices: the committed per-device table unless a
        # table (or 'online' step-0 autotuning) is asked for
        from ..ops import tuning
        tt = getattr(args, "tune_table", "")
        if tt and tt != "online":
            tuning.load(tt)
        elif not tt:
            tuning.load_default()
    model = build_model(args.model, num_classes=args.num_classes, stem=args.stem).to(dev)
    comm = get_comm()
    setup_syncbn(comm, args.sync_bn, getattr(args, "syncbn_comm", "auto"), on_gpu)
    args.step_mode_resolved = resolve_step_mode(getattr(args, "step_mode", "auto"), world_size, on_gpu,
                                                args.image_size, args.dtype)
    OF.set_wgrad_stream(args.step_mode_resolved == "two_stream")
    if on_gpu and args.step_mode_resolved == "two_stream" and isinstance(train_loader, SyntheticImageNet):
        # batches generated (and laid out for the stem) one step ahead
        train_loader.prefetch(OF._wgrad_stream(dev), transform=OF.s2d_input_prefetch(model))
    if rank == 0 and on_gpu:
        print(f"[pmd] step mode: {args.step_mode_resolved}", flush=True)
    model = DataParallel(model, comm, bucket_mb=args.bucket_mb, first_bucket_mb=args.first_bucket_mb,
                         broadcast_buffers=args.broadcast_buffers,
                         reducer=getattr(args, "reducer", "native"),
                         compress=getattr(args, "grad_compress", "none"),
                         transport=getattr(args, "comm", "auto") if on_gpu else "c10d",
                         last_bucket_mb=getattr(args, "last_bucket_mb", 2.0))
    if rank == 0 and comm is not None:
        print("[pmd] gradient buckets (MiB, launch order): "
              + " ".join(f"{m:.2f}" for m in model.bucket_sizes_mb())
              + f" via {model.transport}", flush=True)
    optimizer = FusedSGD(model, lr=args.lr, momentum=args.momentum, weight_decay=args.wd,
                         nesterov=True)
    scheduler = torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=args.milestone_list,
                                                     gamma=args.gamma)
    train_logger = Logger(os.path.join(args.save_path, "train.log"))
    test_logger = Logger(os.path.join(args.save_path, "test.log"))
    start_epoch = 1
    if args.resume:
        last, _ = load_resume(args.resume, model, optimizer, scheduler)
        start_epoch = last + 1
    step = 0
    import warnings
    for epoch in range(start_epoch, args.epochs + 1):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")   # "scheduler.step() before optimizer.step()"
            scheduler.step()                  # every rank, at epoch start (B4 fixed)
        train_loader.set_epoch(epoch)
        train_epoch(train_loader, model, optimizer, epoch, train_logger, args, rank, dev, comm,
                    step_offset=step)
        step += len(train_loader)
        validate(test_loader, model, epoch, test_logger, args, rank, dev, comm, "test")
        if rank == 0:
            if epoch == int(args.epochs):
                save_model(model, args.save_path, epoch)
            if args.resume_every and epoch % args.resume_every == 0:
                save_resume(os.path.join(args.save_path, "resume.pth"), model, optimizer, scheduler,
                            epoch)
    if comm is not None:
        comm.barrier()
    if rank == 0 and not args.no_plot:
        from ..utils.plot import draw_plot
        draw_plot(args.save_path)
    model.close()       # release the native reducer (it holds the process group) before shutdown
