"""Multi-rank safety of the production data-parallel path on the test box's ONE
MI355X (the driver owns 8-GPU runs; these rehearse every W>1 mechanism that
can run with two ranks sharing a device):

  * deferred side-stream weight gradients + the reducer: each bucket fires
    exactly once per step, the reducer counts exactly one iteration per step
    (the double-finalize bug), and the deferred schedule gives the same
    training trajectory as the non-deferred one;
  * the native RCCL communicator (single rank: the real ncclCommInitRank /
    ncclAllReduce / event-fence path) under the gradient reducer;
  * a straggling rank drives its peer's SyncBN exchange into the wall-clock
    timeout, and the training loop RAISES instead of training on garbage;
  * forward progress with a long burst of spinning cross-rank kernels on a
    second stream concurrent with the spinning SyncBN exchanges of a
    training step (the HW-queue sharing hazard);
  * ``bench.py --gpus 2 --backend gloo --same_device`` runs the exact W>1
    bench code path and prints its JSON record.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _join_all(ctx, timeout):
    """ProcessContext.join returns after the FIRST process exits: loop until all
    have (or the deadline passes).  True when every rank finished."""
    import time
    end = time.time() + timeout
    while time.time() < end:
        if ctx.join(timeout=max(end - time.time(), 0.1)):
            return True
    return False


def _data(n=8, hw=32, seed=11):
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    x, _ = C.synth_images(n, hw, hw, 8, 3, 10, seed, 0)
    y = torch.arange(n, device="cuda") % 10
    return x, y


# --------------------------------------------------------------- deferred wgrads
def _defer_worker(rank, world, port, out, defer):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    OF._WGRAD_STREAM["on"] = True
    OF._WGRAD_STREAM["defer"] = defer
    OF.set_deterministic(True)          # bit-exact oracle (kernels/det.hip)
    # the runs are separate processes: pin the kernel choices (no per-process timing, whose
    # noise could pick another split-K plan and so another summation order)
    os.environ["PMD_CONV_AUTOTUNE"] = "0"
    os.environ["PMD_WGRAD_AUTOTUNE"] = "0"
    comm = get_comm()
    comm.enable_xgmi(timeout_s=20.0)
    OF.set_bn_sync(comm)
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=10, stem="imagenet").cuda()
    dp = DataParallel(model, comm, bucket_mb=2.0, first_bucket_mb=0.5)
    # BN in eval mode: the reducer, the bucket rebuild and the deferred side-stream wgrads
    # run the same as in training; the deterministic statistics mode makes every run of
    # the step bit-reproducible, so the schedules are compared exactly.
    dp.module.eval()
    # lr=0: the weights stay fixed, so every step's averaged gradients must agree
    # between the deferred and the per-block join (a race on the last bucket, or
    # a double all-reduce, shows up in ANY of the three steps)
    opt = FusedSGD(dp, lr=0.0, momentum=0.9, nesterov=True)
    x, y = _data(8, 64)
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    launches, grads = [], []
    for _ in range(3):
        loss = OF.cross_entropy(dp(xs), ys)
        opt.zero_grad()
        loss.backward()
        opt.step()
        launches.append(list(dp.collective_signature()))
        grads.append({n: p.grad.detach().float().cpu() for n, p in dp.module.named_parameters()})
    torch.cuda.synchronize()
    comm.xgmi.check()
    if rank == 0:
        torch.save({"iters": dp.num_iterations, "nb": len(dp.buckets), "launches": launches,
                    "grads": grads, "loss": float(loss)}, out)
    OF.set_bn_sync(None)
    dp.close()                  # the native reducer holds the process group
    dist.destroy_process_group()


def test_deferred_wgrad_buckets_fire_once_and_match(tmp_path):
    """the side-stream wgrad flush must run BEFORE the
    reducer's final step -- else every step all-reduces twice and the last
    bucket races the wgrads still writing it."""
    res = {}
    for tag, defer in (("d1", 1), ("d1b", 1), ("d0", 0)):
        out = str(tmp_path / f"{tag}.pt")
        mp.spawn(_defer_worker, args=(2, _free_port(), out, defer), nprocs=2, join=True)
        res[tag] = torch.load(out, weights_only=True)
    for tag, r in res.items():
        assert r["iters"] == 3, (tag, r["iters"])
        # iteration 1 runs on the construction-time buckets, 2-3 on the ready-order rebuild
        for it, order in enumerate(r["launches"]):
            assert order == list(range(len(order))), (tag, it, order)  # each once, index order
            if it > 0:
                assert len(order) == r["nb"], (tag, it, order)

    # The same averaged gradients, bit for bit, at every step: the same schedule twice
    # (d1, d1b) and with / without the deferred join (d0).  A double all-reduce, a torn
    # bucket or a gradient read before its side-stream producer finished cannot hide in it.
    for step in range(3):
        for tag in ("d1b", "d0"):
            a, b = res[tag]["grads"][step], res["d1"]["grads"][step]
            bad = [k for k in b if not torch.equal(a[k], b[k])]
            assert not bad, (tag, step, bad[:5])


# ------------------------------------------------------------- native RCCL comm
def test_native_rccl_comm_single_rank_reducer():
    """ncclGetUniqueId -> ncclCommInitRank -> bucketed ncclAllReduce(avg) on
    the communicator's own stream, event-fenced, under the native reducer."""
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel import rccl
    from pytorch_multiprocessing_distributed_amd.parallel.comm import Comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    rc = rccl.create_single()
    t = torch.arange(1000, device="cuda", dtype=torch.float32)
    want = t.clone()
    rc.all_reduce_(t, 1)
    rc.broadcast_(t, 0)
    torch.cuda.synchronize()
    assert torch.equal(t, want) and rc.check() and rc.calls == 2
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=60),
                            device_id=torch.device("cuda", 0))
    try:
        comm = Comm()
        x, y = _data(8, 32)
        grads = {}
        for transport in ("rccl", None):
            torch.manual_seed(0)
            m = build_model("res").cuda()
            dp = DataParallel(m, comm if transport else None, bucket_mb=0.5, first_bucket_mb=0.1,
                              transport=transport or "c10d", timeline=True)
            # eval-mode BN and lr 0: the gradient is a deterministic function of the
            # weights (tests/test_model_oracle_gpu.py: training-mode BN at init is chaotic)
            dp.module.eval()
            opt = FusedSGD(dp, lr=0.0)
            for _ in range(2):
                loss = OF.cross_entropy(dp(x), y)
                opt.zero_grad()
                loss.backward()
                opt.step()
            torch.cuda.synchronize()
            grads[transport] = {n: p.grad.detach().clone() for n, p in dp.module.named_parameters()}
            if transport:
                assert dp.rccl is not None and dp.rccl.calls > 0
                assert dp.num_iterations == 2
                tl = dp.bucket_timeline()
                assert len(tl) == len(dp.buckets) and all(r[4] == r[4] for r in tl)   # device times set
                dp.shutdown()
        # same model, same kernels, deterministic split-K reduction: the single-rank
        # averaging all-reduce over the native communicator must not change a bit
        for n, g in grads[None].items():
            rel = ((grads["rccl"][n] - g).float().norm() / g.float().norm().clamp_min(1e-12)).item()
            assert rel < 1e-6, (n, rel)
    finally:
        dp.close()                  # the native reducer holds the process group
        dist.destroy_process_group()


def test_auto_transport_picks_native_rccl_with_selftest_and_error_check():
    """--comm auto (the default of main.py / bench.py) on a single-rank nccl group
    with SyncBN on the one-shot xGMI kernel: DataParallel takes the native
    RcclComm after its exact self-test, attaches it to the per-step health check,
    trains a step through it, and an aborted communicator makes
    ``Comm.raise_if_failed`` raise (ncclCommGetAsyncError folded in)."""
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel import rccl
    from pytorch_multiprocessing_distributed_amd.parallel.comm import Comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=60),
                            device_id=torch.device("cuda", 0))
    try:
        comm = Comm()
        comm.enable_xgmi(timeout_s=20.0)
        assert comm.xgmi.self_test()
        OF.set_bn_sync(comm)
        torch.manual_seed(0)
        dp = DataParallel(build_model("res").cuda(), comm, bucket_mb=0.5, first_bucket_mb=0.1)
        assert dp.transport == "rccl" and dp.rccl is not None
        assert comm.natives == [dp.rccl] and comm.in_step_c10d_forbidden
        assert rccl.self_test(dp.rccl, comm.group)
        opt = FusedSGD(dp, lr=0.05)
        x, y = _data(8, 32)
        calls0 = dp.rccl.calls
        for _ in range(2):
            loss = OF.cross_entropy(dp(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            comm.raise_if_failed()
        torch.cuda.synchronize()
        assert bool(torch.isfinite(loss).item()) and dp.rccl.calls > calls0
        dp.shutdown()                       # ncclCommAbort
        with pytest.raises(RuntimeError, match="native RCCL communicator failed"):
            comm.raise_if_failed()
    finally:
        OF.set_bn_sync(None)
        dp.close()                  # the native reducer holds the process group
        dist.destroy_process_group()


# ---------------------------------------------------------- straggler -> raise
def _straggler_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # rank 1 sleeps 4 s before step 2 (step 1 begins with the host-side broadcast of
    # the bucket rebuild order, which would re-align the ranks on the host)
    os.environ["PMD_FAULT_DELAY"] = "1:2:4"
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd import launch
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    comm = get_comm()
    comm.enable_xgmi(timeout_s=20.0)    # steps 0-1 (per-rank kernel autotuning) at a safe timeout
    OF.set_bn_sync(comm)
    torch.manual_seed(0)
    dp = DataParallel(build_model("res").cuda(), comm, bucket_mb=1.0)
    opt = FusedSGD(dp, lr=0.05)
    x, y = _data(8, 32)
    err = ""
    steps_done = 0
    finite = []
    try:
        for i in range(4):
            launch.maybe_inject_fault(rank, i)
            loss = OF.cross_entropy(dp(x[:4]), y[:4])
            opt.zero_grad()
            loss.backward()
            opt.step()
            torch.cuda.synchronize()
            finite.append(bool(torch.isfinite(loss).item())
                          and bool(torch.isfinite(dp.flat.param_arena).all().item()))
            comm.raise_if_failed()
            steps_done += 1
            if i == 1:
                comm.barrier()
                comm.xgmi.set_timeout(0.5)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"err": err, "steps": steps_done, "finite": finite}, f)
    OF.set_bn_sync(None)
    os._exit(0)          # do not wait in a collective on a peer that already left


def test_straggler_timeout_raises(tmp_path):
    out = str(tmp_path / "s")
    ctx = mp.spawn(_straggler_worker, args=(2, _free_port(), out), nprocs=2, join=False)
    assert _join_all(ctx, 180)
    r0 = json.load(open(f"{out}.0"))
    assert "timed out" in r0["err"], r0
    assert r0["steps"] == 2, r0      # steps 0-1 fine, step 2 detected, no step 3
    # the timed-out exchange poisoned its outputs: the failing step's loss /
    # updated weights are NaN, not silently wrong (kernels/xgmi.hip)
    assert r0["finite"] == [True, True, False], r0


# ------------------------------------------- spinning kernels on two streams
def _progress_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    from pytorch_multiprocessing_distributed_amd.parallel.xgmi import XgmiAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    comm = get_comm()
    comm.enable_xgmi(timeout_s=20.0)
    OF.set_bn_sync(comm)
    burst = XgmiAllReduce(timeout_s=20.0)      # a second, independent spinning collective
    side = torch.cuda.Stream()
    torch.manual_seed(0)
    dp = DataParallel(build_model("resnet50", num_classes=10, stem="imagenet").cuda(), comm,
                      bucket_mb=4.0)
    opt = FusedSGD(dp, lr=0.05)
    x, y = _data(4, 64)
    bufs = []
    for step in range(3):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for k in range(40):       # ~ms of back-to-back cross-rank spinning kernels
                t = torch.full((32768,), float(rank + 1 + k), device="cuda")
                burst.all_reduce_(t)
                bufs.append((t, 2 * k + 3.0))
        loss = OF.cross_entropy(dp(x[rank * 2:(rank + 1) * 2]), y[rank * 2:(rank + 1) * 2])
        opt.zero_grad()
        loss.backward()
        opt.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    ok = all(bool((t == v).all()) for t, v in bufs)
    comm.xgmi.check()
    burst.check()
    if rank == 0:
        torch.save({"ok": ok, "loss": float(loss)}, out)
    OF.set_bn_sync(None)
    dist.destroy_process_group()


def test_spinning_collectives_on_two_streams_make_progress(tmp_path):
    out = str(tmp_path / "p.pt")
    ctx = mp.spawn(_progress_worker, args=(2, _free_port(), out), nprocs=2, join=False)
    assert _join_all(ctx, 240), "ranks did not finish (deadlock?)"
    got = torch.load(out, weights_only=True)
    assert got["ok"] and got["loss"] == got["loss"]


# ------------------------------------------------------ bench W>1 rehearsal
def test_bench_two_ranks_gloo_same_device():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--same_device", "--syncbn_comm", "xgmi", "--steps", "3", "--warmup", "2",
           "--batch", "16", "--image", "64", "--bucket_mb", "4"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2-same-gpu-gloo"
    assert rec["config"]["syncbn_comm"] == "xgmi" and rec["value"] > 0


@pytest.mark.parametrize("comm", ["auto", "c10d"])
def test_bench_dp_rehearsal_production_step(comm):
    """bench.py --dp_rehearsal: the production W>1 per-rank step on one GPU (DataParallel
    over a single-rank RCCL group, native reducer, bucket all-reduces on the native RcclComm
    -- or c10d --, SyncBN through the xGMI kernel) runs, reports itself as such, and its
    loss is finite."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dp_rehearsal", "--comm", comm,
           "--steps", "3", "--warmup", "2", "--batch", "16", "--image", "64", "--bucket_mb", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    cfg = rec["config"]
    assert rec["n_gpus"] == 1 and cfg["parallelism"] == "dp1-rehearsal"
    assert cfg["sync_bn"] is True and cfg["syncbn_comm"] == "xgmi"
    assert cfg["grad_transport"] == ("rccl" if comm == "auto" else "c10d")
    assert len(cfg["grad_buckets_mb"]) >= 2
    assert rec["final_loss"] == rec["final_loss"] and rec["value"] > 0
    if comm == "auto":
        assert "exact self-test passed" in r.stdout
