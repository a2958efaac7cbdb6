"""Multi-process data parallelism on CPU/gloo (BASELINE config 1 plumbing).

Key invariant: with SyncBN, a W-rank step on per-rank batch
B/W equals a single-process step on the global batch B -- loss, averaged
gradients, updated parameters and BN running statistics.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_steps(model, x, y, steps, dp_comm=None, bucket_mb=0.05, reducer="native", compress="none"):
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dp = DataParallel(model, dp_comm, bucket_mb=bucket_mb, first_bucket_mb=0.01, reducer=reducer,
                      compress=compress)
    opt = FusedSGD(dp, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    losses = []
    for _ in range(steps):
        loss = OF.cross_entropy(dp(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    return dp, losses


def _data(seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(8, 16, 16, 3, generator=g, dtype=torch.float64)
    y = torch.randint(0, 10, (8,), generator=g)
    return x, y


def _grads(dp):
    # by name: the data-parallel arena is re-laid out in ready order after iteration 1
    return {n: p.grad.detach().clone() for n, p in dp.module.named_parameters()}


def _worker(rank, world, port, out_path, reducer="native", compress="none"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    OF.set_bn_sync(comm)
    torch.manual_seed(100 + rank)            # different init per rank: DP must broadcast rank 0's
    model = build_model("res").double()
    if rank == 0:
        torch.manual_seed(0)
        model = build_model("res").double()
    x, y = _data()
    per = x.shape[0] // world
    dp, losses = _run_steps(model, x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per],
                            2, comm, reducer=reducer, compress=compress)
    assert len(dp.buckets) > 1
    assert dp.num_iterations == 2
    gl = [torch.stack(losses)]
    comm.all_reduce_(gl[0])
    if rank == 0:
        torch.save({"state": dp.module.state_dict(), "loss": gl[0] / world,
                    "grad": _grads(dp), "order": dp.rebuilt_order}, out_path)
    OF.set_bn_sync(None)
    dp.close()                  # the native reducer holds the process group: release it first
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("reducer", ["native", "python"])
def test_two_rank_step_equals_single_process(tmp_path, reducer):
    """Both reducers (C++ ``_C.Reducer`` and the Python one) give the exact
    global-batch step."""
    from pytorch_multiprocessing_distributed_amd.models import build_model
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, reducer), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    ref_model = build_model("res").double()
    x, y = _data()
    dp, losses = _run_steps(ref_model, x, y, 2, None)
    ref = dp.module.state_dict()
    for k, v in ref.items():
        torch.testing.assert_close(got["state"][k], v, rtol=1e-7, atol=1e-9, msg=k)
    # per-rank mean loss averaged over ranks == global-batch loss
    torch.testing.assert_close(got["loss"], torch.stack(losses), rtol=1e-9, atol=1e-9)
    for n, g in _grads(dp).items():
        torch.testing.assert_close(got["grad"][n], g, rtol=1e-6, atol=1e-9, msg=n)
    # the arena was re-laid out in the observed gradient-ready order: the linear
    # layer (first node of backward) leads, the stem conv comes last
    assert got["order"] is not None and got["order"][0].startswith("linear")
    assert got["order"][-1] in ("conv1.weight", "bn1.weight", "bn1.bias")


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
def test_multi_rank_step_equals_single_process(tmp_path, world):
    """W=4 and W=8 (2 / 1 samples per rank, the dp8 rank count of the scaling
    bench): the native reducer + SyncBN over gloo still give the exact
    global-batch step (bucket launch order, rebuild and SyncBN statistics with
    more than two peers)."""
    from pytorch_multiprocessing_distributed_amd.models import build_model
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(world, _free_port(), out, "native"), nprocs=world, join=True)
    got = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    ref_model = build_model("res").double()
    x, y = _data()
    dp, losses = _run_steps(ref_model, x, y, 2, None)
    for k, v in dp.module.state_dict().items():
        torch.testing.assert_close(got["state"][k], v, rtol=1e-7, atol=1e-9, msg=k)
    torch.testing.assert_close(got["loss"], torch.stack(losses), rtol=1e-9, atol=1e-9)
    for n, g in _grads(dp).items():
        torch.testing.assert_close(got["grad"][n], g, rtol=1e-6, atol=1e-9, msg=n)


@pytest.mark.slow
def test_two_rank_bf16_wire_compression(tmp_path):
    """compress="bf16": buckets travel in bf16, the fp32/fp64 arena receives
    the average -- equal to the exact step up to bf16 rounding."""
    from pytorch_multiprocessing_distributed_amd.models import build_model
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, "native", "bf16"), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    ref_model = build_model("res").double()
    x, y = _data()
    dp, _ = _run_steps(ref_model, x, y, 2, None)
    g = torch.cat([got["grad"][n].flatten() for n, _ in dp.module.named_parameters()])
    r = torch.cat([p.grad.flatten() for _, p in dp.module.named_parameters()])
    assert ((g - r).norm() / r.norm()).item() < 5e-2   # 2 steps of bf16-rounded averages


def _no_sync_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    torch.manual_seed(0)
    dp = DataParallel(build_model("res").double(), comm, bucket_mb=0.05, first_bucket_mb=0.01)
    x, y = _data(seed=10 + rank)
    dp.zero_grad()
    with dp.no_sync():
        OF.cross_entropy(dp(x[:4]), y[:4]).backward()
    assert dp.num_iterations == 0                       # nothing was communicated
    local = dp.flat.grad_arena.clone()
    other = comm.all_gather(local)
    assert not torch.equal(other[0], other[1])          # grads still rank-local
    OF.cross_entropy(dp(x[4:]), y[4:]).backward()       # accumulates, then averages
    assert dp.num_iterations == 1
    allg = comm.all_gather(dp.flat.grad_arena.clone())
    assert torch.equal(allg[0], allg[1])
    dp.close()                  # the native reducer holds the process group
    dist.destroy_process_group()


@pytest.mark.slow
def test_no_sync_gradient_accumulation():
    mp.spawn(_no_sync_worker, args=(2, _free_port()), nprocs=2, join=True)


def _fault_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["PMD_FAULT_RANK"] = "1"
    os.environ["PMD_FAULT_STEP"] = "0"
    from pytorch_multiprocessing_distributed_amd.launch import maybe_inject_fault
    maybe_inject_fault(rank, 0)


@pytest.mark.slow
def test_spawn_fail_fast_propagates_rank_error():
    with pytest.raises(mp.ProcessRaisedException, match="injected fault on rank 1"):
        mp.spawn(_fault_worker, args=(2, _free_port()), nprocs=2, join=True)


@pytest.mark.slow
def test_main_py_end_to_end_cpu_gloo(tmp_path):
    """BASELINE config 1: `python main.py --world_size 2` on CPU produces every
    reference artefact (logs, plots, main.py snapshot, model_<epochs>.pth)."""
    save = str(tmp_path / "run")
    cmd = [sys.executable, os.path.join(ROOT, "main.py"), "--world_size", "2", "--epochs", "2",
           "--synthetic", "--train_samples", "128", "--batch_size", "32", "--save_path", save,
           "--print-freq", "2", "--master_port", str(_free_port()), "--resume_every", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "Epoch: [1][0/4]" in r.stdout and "Accuracy" in r.stdout
    for f in ("main.py", "train.log", "test.log", "test_accuracy.png", "loss.png", "model_2.pth",
              "resume.pth"):
        assert os.path.exists(os.path.join(save, f)), f
    lines = open(os.path.join(save, "train.log")).read().splitlines()
    assert len(lines) == 2 and lines[0].startswith("0001 ")
    # resume from the epoch-2 checkpoint for one more epoch
    cmd2 = cmd[:]
    cmd2[cmd2.index("--epochs") + 1] = "3"
    cmd2[cmd2.index("--master_port") + 1] = str(_free_port())
    cmd2 += ["--resume", os.path.join(save, "resume.pth")]
    r = subprocess.run(cmd2, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Epoch: [3][0/4]" in r.stdout and "Epoch: [1]" not in r.stdout
    assert os.path.exists(os.path.join(save, "model_3.pth"))
