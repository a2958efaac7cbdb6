"""Two ranks sharing the one MI355X of the test box.

RCCL refuses two ranks on one device, so the collectives here run on gloo
(which handles GPU tensors by host staging); everything else -- the gfx950
kernels, SyncBN statistics exchange, direct-to-arena gradients, bucket
readiness / async all-reduce ordering, rank-0 broadcast -- is the exact
production path.  Invariant: a 2-rank step on per-rank batch B/2 equals one
process on the global batch B, held PER TENSOR against the fp32 oracle at 3x the
single-process step's own error (test_model_oracle_gpu.py's method).
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


class _NoWork:
    def wait(self):
        pass


def _worker(rank, world, port, out, stats_comm="gloo", fault="none", model_name="res", det=False, streams=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    from pytorch_multiprocessing_distributed_amd.parallel import dp as DP
    from pytorch_multiprocessing_distributed_amd.parallel.comm import get_comm
    torch.cuda.set_device(0)
    # the rank's step streams (main / weight gradients / collectives) created before the process
    # group, as launch.init_process does for every production rank
    if streams:
        OF.init_step_streams(torch.device("cuda", 0))
    if det:
        # the production kernel choices (committed tables, no per-process online tuning of 8
        # processes sharing the GPU) and the deterministic statistics mode
        from pytorch_multiprocessing_distributed_amd.ops import tuning
        tuning.load_default()
        OF.set_deterministic(True)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = get_comm()
    if stats_comm == "xgmi":
        comm.enable_xgmi(timeout_s=20.0)     # SyncBN statistics over the one-shot IPC kernel
        comm.xgmi.select_ordering(verbose=False)
    OF.set_bn_sync(comm)
    if fault == "overlap":
        # not a fault: the backward statistics exchange on the side stream from the event after
        # the dgrad that produced its slots (PMD_SYNCBN_OVERLAP=1; the hand-offs on the fork ring)
        comm.overlap_bn_bwd = True
    if fault == "stats_half" and rank == 1:
        # negative control: ONE SyncBN statistics site (the 4th forward exchange) contributes
        # half its partial sums on rank 1 -- a wrong statistic at a single site
        calls = {"n": 0}
        orig_fwd, orig_ar = comm.bn_stats_fwd, comm.all_reduce_stats_

        def bad_fwd(st, *a, **k):
            calls["n"] += 1
            if calls["n"] == 4:
                st.mul_(0.5)
            return orig_fwd(st, *a, **k)
        comm.bn_stats_fwd = bad_fwd
    reducer = "native"
    if fault == "skip_bucket":
        # negative control: one gradient bucket's all-reduce never runs (its gradients stay
        # rank-local); the python reducer exposes the launch to patch
        reducer = "python"
        orig_launch = DP.DataParallel._launch

        def launch(self, b):
            if b.index == len(self.buckets) // 2:
                b.fired += 1
                b.work = _NoWork()
                return
            orig_launch(self, b)
        DP.DataParallel._launch = launch
    torch.manual_seed(0 if rank == 0 else 77)     # rank 1 starts different: broadcast must fix it
    if model_name == "resnet50":
        # bottleneck blocks with the linear-BN backward on EVERY identity block (PMD_BNLIN=all)
        OF._BNLIN = "all"
        lin_calls = {"n": 0}
        orig_lin = OF._bnlin_final

        def counted(*a, **k):
            lin_calls["n"] += 1
            return orig_lin(*a, **k)
        OF._bnlin_final = counted
        torch.manual_seed(0)
        model = build_model("resnet50", num_classes=10, stem="imagenet").cuda()
        x, y = C.synth_images(16, 64, 64, 8, 3, 10, 7, 0)
    else:
        model = build_model("res", num_classes=10, stem="cifar").cuda()
        x, y = C.synth_images(64, 32, 32, 8, 3, 10, 7, 0)   # == test_model_oracle_gpu's batch
    per = x.shape[0] // world
    dp = DP.DataParallel(model, comm, bucket_mb=1.0, first_bucket_mb=0.25, reducer=reducer)
    dp.train()
    loss = OF.cross_entropy(dp(x[rank * per:(rank + 1) * per]), y[rank * per:(rank + 1) * per])
    loss.backward()
    torch.cuda.synchronize()
    losses = loss.detach().reshape(1).clone()
    comm.all_reduce_(losses)
    if comm.xgmi is not None:
        comm.xgmi.check()
        assert comm.xgmi.calls > 0
    if rank == 0:
        torch.save({"grads": {n: p.grad.detach().float().cpu() for n, p in
                              dp.module.named_parameters()},
                    "buffers": {k: v.cpu() for k, v in dp.module.state_dict().items()
                                if "running" in k or "num_batches" in k},
                    "loss": float(losses.item() / world),
                    "lin_calls": lin_calls["n"] if model_name == "resnet50" else 0,
                    "nbuckets": len(dp.buckets)}, out)
    OF.set_bn_sync(None)
    dp.close()                  # the native reducer holds the process group
    dist.destroy_process_group()


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _oracle_violations(got, ms, loss, grads):
    """Per-tensor bound (the test_model_oracle_gpu.py method): the 2-rank
    step's error against the fp32 single-process oracle on EVERY one of the 38 gradient
    tensors must stay within 3x the SINGLE-PROCESS gfx950 step's error on that same tensor
    (floored at half its median) + 1e-2; BN running statistics within the single-process
    bounds of test_resnet50_train_bn_step_vs_fp32_oracle."""
    bad = []
    e1 = {n: _rel(g.float().cpu(), grads["f32"][n].float().cpu()) for n, g in grads["hip"].items()}
    e2 = {n: _rel(g, grads["f32"][n].float().cpu()) for n, g in got["grads"].items()}
    assert len(e2) == 38 and set(e1) == set(e2)
    med = sorted(e1.values())[len(e1) // 2]
    floor = 0.5 * med
    for n in e2:
        if e2[n] > 3.0 * max(e1[n], floor) + 1e-2:
            bad.append((n, round(e2[n], 4), round(e1[n], 4)))
    if abs(got["loss"] - loss["f32"]) / loss["f32"] > 1e-2:
        bad.append(("loss", got["loss"], loss["f32"]))
    ref = {k: v for k, v in ms["f32"].state_dict().items()}
    for k, g in got["buffers"].items():
        r = ref[k].cpu()
        if not g.dtype.is_floating_point:
            if not torch.equal(g, r):
                bad.append((k, g.tolist(), r.tolist()))
        elif k.endswith("running_var"):
            if _rel(g, r) > 1e-2:
                bad.append((k, _rel(g, r)))
        elif k.endswith("running_mean"):
            std = ((ref[k[:-4] + "var"].cpu().double() - 0.9) / 0.1).clamp_min(0).sqrt()
            err = ((g - r).double().norm() / (0.1 * std).norm()).item()
            if err > 1e-2:
                bad.append((k, err))
    return bad, e1, e2


@pytest.mark.parametrize("stats_comm,fault", [("gloo", "none"), ("xgmi", "none"), ("xgmi", "stats_half"),
                                              ("xgmi", "skip_bucket"), ("xgmi", "overlap")])
def test_two_ranks_on_one_gpu_match_single_process_per_tensor(tmp_path, stats_comm, fault):
    """2 ranks x batch 32 of ResNet-18-ref through the production W>1 path (SyncBN over the
    xGMI kernel at the stress-selected ordering, native reducer) == one process on the
    global batch 64, per gradient tensor and running statistic.  Negative controls: a
    statistics site halved on rank 1, and one bucket's all-reduce skipped, must FAIL."""
    import test_model_oracle_gpu as oracle
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, stats_comm, fault), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    ms, loss, grads = oracle._runs(train=True, model="res")
    bad, e1, e2 = _oracle_violations(got, ms, loss, grads)
    worst = sorted(((e2[n] / max(e1[n], 1e-6), n) for n in e2), reverse=True)[:5]
    print(f"[{stats_comm}/{fault}] buckets {got['nbuckets']}, worst e2/e1: "
          + ", ".join(f"{n} {r:.2f}" for r, n in worst))
    if fault in ("none", "overlap"):
        assert not bad, bad
    else:
        assert bad, f"negative control {fault} passed the per-tensor oracle"


def _r50_single(monkeypatch):
    """Single-process ResNet-50 step on the global batch (linear-BN backward everywhere):
    gfx950 kernels and the fp32 torch-primitive oracle, same weights and batch."""
    import copy
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.ops.native import C
    monkeypatch.setattr(OF, "_BNLIN", "all")
    torch.manual_seed(0)
    m0 = build_model("resnet50", num_classes=10, stem="imagenet").cuda()
    x, y = C.synth_images(16, 64, 64, 8, 3, 10, 7, 0)
    m0.train()
    grads, loss = {}, {}
    for k in ("hip", "f32"):
        m = copy.deepcopy(m0)
        OF.force_torch_prims(k == "f32")
        try:
            lo = OF.cross_entropy(m(x.float() if k == "f32" else x), y)
            lo.backward()
        finally:
            OF.force_torch_prims(False)
        torch.cuda.synchronize()
        loss[k] = float(lo)
        grads[k] = {n: p.grad.detach().float().cpu() for n, p in m.named_parameters()}
    return loss, grads


def test_two_ranks_resnet50_linear_bn_match_single_process(tmp_path, monkeypatch):
    """The linear-BN backward under SyncBN: 2 ranks x 8 images of ResNet-50 (every identity
    block's final BN back-propagated through its conv3, statistics over the xGMI kernel) == one
    process on the global 16, per gradient tensor against the fp32 oracle (3x the single
    process's own error, floored at half its median, + 1e-2)."""
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, "xgmi", "none", "resnet50"), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert got["lin_calls"] == 11      # every identity block whose output feeds a fused dgrad
    loss, grads = _r50_single(monkeypatch)
    e1 = {n: _rel(g, grads["f32"][n]) for n, g in grads["hip"].items()}
    e2 = {n: _rel(g, grads["f32"][n]) for n, g in got["grads"].items()}
    assert set(e1) == set(e2) and len(e2) == 161
    floor = 0.5 * sorted(e1.values())[len(e1) // 2]
    bad = [(n, round(e2[n], 4), round(e1[n], 4)) for n in e2 if e2[n] > 3.0 * max(e1[n], floor) + 1e-2]
    # the loss, like every tensor: within 3x the single process's own error against fp32 (a
    # batch of 16 64x64 images leaves l4's BN 64 values per channel: bf16 itself is ~3% off)
    own = abs(loss["hip"] - loss["f32"])
    assert abs(got["loss"] - loss["f32"]) <= 3.0 * own + 1e-2 * loss["f32"], (got["loss"], loss)
    assert not bad, bad


def test_eight_ranks_on_one_gpu_match_single_process_per_tensor(tmp_path):
    """the W=8 path rehearsed on the one GPU -- 8 ranks x batch 8 of
    ResNet-18-ref through the production W>1 path (SyncBN over the xGMI kernel with 8-rank
    slot / flag tables at the stress-selected ordering, native reducer, rank-0 broadcast of
    7 differently initialised replicas) == one process on the global batch 64, per gradient
    tensor and running statistic, at the same bound as the 2-rank case.  The ranks run the
    committed kernel tables in the deterministic statistics mode: one of ~7 runs with 8
    processes tuning online on the shared GPU in the atomic mode broke the bound on one bucket
    (layer4.0 bn2 / conv2, ~15x); the same 8-rank step repeated 80 times per rank in this mode
    (bench/w8_race.py) and 22 fresh first steps in the atomic mode were bit-identical."""
    import test_model_oracle_gpu as oracle
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(8, _free_port(), out, "xgmi", "none", "res", True), nprocs=8, join=True)
    got = torch.load(out, weights_only=True)
    ms, loss, grads = oracle._runs(train=True, model="res")
    bad, e1, e2 = _oracle_violations(got, ms, loss, grads)
    worst = sorted(((e2[n] / max(e1[n], 1e-6), n) for n in e2), reverse=True)[:5]
    print(f"[8 ranks] buckets {got['nbuckets']}, worst e2/e1: "
          + ", ".join(f"{n} {r:.2f}" for r, n in worst))
    assert not bad, bad

