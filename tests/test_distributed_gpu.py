"""Two ranks sharing the one MI355X of the test box.

RCCL refuses two ranks on one device, so the collectives here run on gloo
(which handles GPU tensors by host staging); everything else -- the gfx950
kernels, SyncBN statistics exchange, direct-to-arena gradients, bucket
readiness / async all-reduce ordering, rank-0 broadcast -- is the exact
production path.  Invariant: a 2-rank step on per-rank batch B/2 equals one
process on the global batch B (up to bf16 rounding of the split statistics).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    x, _ = C.synth_images(8, 32, 32, 8, 3, 10, 11, 0)
    y = torch.arange(8, device="cuda") % 10
    return x, y


def _steps(model, x, y, comm, n=2):
    from pytorch_multiprocessing_distributed_amd.engine.optim import FusedSGD
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    dp = DataParallel(model, comm, bucket_mb=1.0, first_bucket_mb=0.25)
    opt = FusedSGD(dp, lr=0.05, momentum=0.9, weight_decay=1e-4, nesterov=True)
    losses = []
    for _ in range(n):
        loss = OF.cross_entropy(dp(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    return dp, torch.stack(losses)


def _worker(rank, world, port, out, stats_comm="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    if stats_comm == "xgmi":
        comm.enable_xgmi(timeout_s=20.0)     # SyncBN statistics over the one-shot IPC kernel
    OF.set_bn_sync(comm)
    torch.manual_seed(0 if rank == 0 else 77)     # rank 1 starts different: broadcast must fix it
    model = build_model("res").cuda()
    x, y = _data()
    per = x.shape[0] // world
    dp, losses = _steps(model, x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per], comm,
                        n=1)
    comm.all_reduce_(losses)
    if comm.xgmi is not None:
        comm.xgmi.check()
        assert comm.xgmi.calls > 0
    if rank == 0:
        torch.save({"grads": {n: p.grad.detach().float().cpu() for n, p in
                              dp.module.named_parameters()},
                    "buffers": {k: v.cpu() for k, v in dp.module.state_dict().items()
                                if "running" in k or "num_batches" in k},
                    "loss": (losses / world).cpu()}, out)
    OF.set_bn_sync(None)
    dist.destroy_process_group()


@pytest.mark.parametrize("stats_comm", ["gloo", "xgmi"])
def test_two_ranks_on_one_gpu_match_single_process(tmp_path, stats_comm):
    from pytorch_multiprocessing_distributed_amd.models import build_model
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, stats_comm), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    torch.manual_seed(0)
    model = build_model("res").cuda()
    x, y = _data()
    dp, losses = _steps(model, x, y, None, n=1)
    torch.testing.assert_close(got["loss"], losses.cpu(), rtol=1e-2, atol=1e-2)
    # all-reduced (averaged) gradients of the 2-rank step == single-process gradients
    # Gradient agreement: bf16 rounding differences (two partial statistics sums vs
    # one) are amplified through BN backward (mean-subtraction cancellation) at
    # random init -- the same ~0.995 cosine seen between two single-GPU runs on
    # different kernels -- so deep params are checked by direction, the head
    # (no BN downstream) tightly.  Exact equality of the algorithm is pinned by
    # the fp64 gloo/CPU test (test_distributed_cpu.py).
    errs = {}
    for n, p in dp.module.named_parameters():
        g, v = got["grads"][n], p.grad.detach().float().cpu()
        cos = torch.nn.functional.cosine_similarity(g.flatten(), v.flatten(), dim=0).item()
        rel = ((g - v).norm() / v.norm().clamp_min(1e-12)).item()
        errs[n] = (cos, rel)
    bad = {n: e for n, e in errs.items() if e[0] < 0.98 or (n.startswith("linear") and e[1] > 2e-2)}
    assert not bad, f"grad mismatch {bad} (all: {errs})"
    # SyncBN running statistics are the global-batch ones
    for k, v in dp.module.state_dict().items():
        if k in got["buffers"]:
            g = got["buffers"][k].float()
            v = v.float().cpu()
            if k.endswith("num_batches_tracked"):
                assert torch.equal(g, v), k
            else:
                assert (g - v).abs().max() <= 1e-2 * v.abs().max().clamp_min(1e-3), k
