"""Multi-GPU readiness checks that run without a GPU:
native-communicator abort on a rank failure, the ``--comm`` transport flag,
the single-in-step-communicator rule of ``--comm rccl``, and the capped last
gradient bucket."""
import os
import socket

import pytest
import torch

from pytorch_multiprocessing_distributed_amd import config, launch
from pytorch_multiprocessing_distributed_amd.parallel import rccl


class _FakeComm:
    def __init__(self, fail=False):
        self.aborted = 0
        self.fail = fail

    def abort(self):
        self.aborted += 1
        if self.fail:
            raise RuntimeError("abort failed")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_abort_reaches_every_native_communicator():
    a, b, c = _FakeComm(), _FakeComm(fail=True), _FakeComm()
    for x in (a, b, c):
        rccl.register(x)
    launch.abort()                       # no process group: only the native comms
    assert (a.aborted, b.aborted, c.aborted) == (1, 1, 1)   # one failing abort never stops the rest
    assert rccl.live() == []
    launch.abort()                       # idempotent: nothing left to abort
    assert a.aborted == 1


def test_run_rank_failure_aborts_native_comm(monkeypatch):
    """engine.train.run_rank: an exception inside the rank's run aborts the
    framework's own RCCL communicator(s) before the process group is torn down
    (peers blocked in a bucket all-reduce unblock)."""
    from pytorch_multiprocessing_distributed_amd.engine import train
    fake = _FakeComm()

    def boom(rank, world, args, dev):
        rccl.register(fake)
        raise RuntimeError("rank failure")
    monkeypatch.setattr(train, "_run", boom)
    args = config.parse_args(["--world_size", "1", "--device", "cpu", "--backend", "gloo",
                              "--master_port", str(_free_port())])
    with pytest.raises(RuntimeError, match="rank failure"):
        train.run_rank(0, 1, args)
    assert fake.aborted == 1


def test_comm_flag():
    assert config.parse_args([]).comm == "auto"
    assert config.parse_args(["--comm", "rccl"]).comm == "rccl"
    assert config.parse_args(["--comm", "c10d"]).comm == "c10d"
    with pytest.raises(SystemExit):
        config.parse_args(["--comm", "mpi"])


class _SelComm:
    """Enough of parallel.comm.Comm for resolve_transport."""
    def __init__(self, backend="nccl"):
        self.backend, self.rank, self.world_size, self.group = backend, 0, 8, None


class _Native:
    def __init__(self):
        self.aborted = 0

    def abort(self):
        self.aborted += 1


class _Xgmi:
    def __init__(self, capacity):
        self.capacity = capacity


@pytest.fixture
def bn_sync_guard():
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    prev = OF.get_bn_sync()
    yield OF
    OF.set_bn_sync(prev)


def test_auto_transport_selection(monkeypatch, bn_sync_guard, capsys):
    """--comm auto: rccl exactly when the native communicator can be the only
    in-step communicator AND its self-test passes on every rank; c10d otherwise,
    with the reason printed.  Explicit rccl raises where auto falls back."""
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.parallel import dp as DP
    OF = bn_sync_guard
    m = build_model("resnet50", num_classes=10, stem="imagenet")
    made = []

    def create(group=None, priority=0, store=None, stream=0, stream_spec=None):
        if stream_spec is not None:
            priority, stream = stream_spec()     # resolved inside create
        c = _Native()
        made.append(c)
        return c
    result = {"ok": True}
    monkeypatch.setattr(rccl, "create", create)
    monkeypatch.setattr(rccl, "self_test", lambda c, group=None: result["ok"])

    class Sync:
        xgmi = _Xgmi(32768)
    # SyncBN on the xGMI kernel, self-test passes -> rccl
    OF.set_bn_sync(Sync())
    t, c = DP.resolve_transport(_SelComm(), m, "native", "auto")
    assert t == "rccl" and c is made[-1] and c.aborted == 0
    assert "rccl" in capsys.readouterr().out
    # self-test fails -> c10d, the communicator is torn down
    result["ok"] = False
    t, c = DP.resolve_transport(_SelComm(), m, "native", "auto")
    assert t == "c10d" and c is None and made[-1].aborted == 1
    assert "self-test failed" in capsys.readouterr().out
    with pytest.raises(RuntimeError, match="self-test"):
        DP.resolve_transport(_SelComm(), m, "native", "rccl")
    result["ok"] = True
    # SyncBN over the process group -> c10d (two communicators in the step)
    OF.set_bn_sync(type("S", (), {"xgmi": None})())
    n = len(made)
    assert DP.resolve_transport(_SelComm(), m, "native", "auto") == ("c10d", None)
    assert len(made) == n                      # no communicator was even created
    with pytest.raises(ValueError, match="two communicators"):
        DP.resolve_transport(_SelComm(), m, "native", "rccl")
    # a statistics message that does not fit the xGMI kernel (R50: 4*2048+1 floats)
    class Small:
        xgmi = _Xgmi(4096)
    OF.set_bn_sync(Small())
    assert DP.resolve_transport(_SelComm(), m, "native", "auto")[0] == "c10d"
    assert "capacity" in capsys.readouterr().out
    # SyncBN off, python reducer, gloo, no comm, explicit c10d
    OF.set_bn_sync(None)
    assert DP.resolve_transport(_SelComm(), m, "native", "auto")[0] == "rccl"
    assert DP.resolve_transport(_SelComm(), m, "python", "auto")[0] == "c10d"
    assert DP.resolve_transport(_SelComm("gloo"), m, "native", "auto") == ("c10d", None)
    assert DP.resolve_transport(None, m, "native", "auto") == ("c10d", None)
    assert DP.resolve_transport(_SelComm(), m, "native", "c10d") == ("c10d", None)


def test_native_comm_errors_raise_every_step_and_no_c10d_fallback():
    """Comm.raise_if_failed folds in ncclCommGetAsyncError of the attached native
    communicators; with the native transport a SyncBN message the xGMI kernel
    cannot take raises instead of falling back to a c10d collective."""
    from pytorch_multiprocessing_distributed_amd.parallel.comm import Comm

    class C:
        def __init__(self):
            self.ok = True

        def check(self):
            return self.ok
    comm = Comm.__new__(Comm)
    comm.xgmi, comm.rank, comm.natives, comm.in_step_c10d_forbidden = None, 0, [], False
    nat = C()
    comm.attach_native(nat)
    comm.attach_native(nat)
    assert comm.natives == [nat]
    comm.raise_if_failed()
    nat.ok = False
    with pytest.raises(RuntimeError, match="native RCCL communicator failed"):
        comm.raise_if_failed()
    comm.in_step_c10d_forbidden = True
    comm._seq = comm._ncoll = 0
    with pytest.raises(RuntimeError, match="two communicators"):
        comm.all_reduce_stats_(torch.zeros(8))


def test_rccl_transport_needs_single_in_step_communicator():
    from pytorch_multiprocessing_distributed_amd.ops import functional as OF
    from pytorch_multiprocessing_distributed_amd.parallel.dp import _check_single_in_step_communicator

    class Sync:
        xgmi = None
    prev = OF.get_bn_sync()
    try:
        OF.set_bn_sync(Sync())               # SyncBN over the process group: refused
        with pytest.raises(ValueError, match="two communicators"):
            _check_single_in_step_communicator(Sync())
        s = Sync()
        s.xgmi = _Xgmi(32768)                # one-shot xGMI exchange: allowed
        OF.set_bn_sync(s)
        _check_single_in_step_communicator(s)
        OF.set_bn_sync(None)                 # --sync_bn off: allowed
        _check_single_in_step_communicator(Sync())
    finally:
        OF.set_bn_sync(prev)


@pytest.mark.parametrize("last_mb", [2.0, 0.5])
def test_last_bucket_is_capped(last_mb):
    from pytorch_multiprocessing_distributed_amd.models import build_model
    from pytorch_multiprocessing_distributed_amd.parallel.dp import DataParallel
    m = build_model("resnet50", num_classes=1000, stem="imagenet")
    dp = DataParallel(m, None, bucket_mb=25.0, first_bucket_mb=1.0, last_bucket_mb=last_mb)
    sizes = dp.bucket_sizes_mb()
    total = sum(p.numel() for p in m.parameters()) * 4 / 2 ** 20
    assert abs(sum(sizes) - total) < 1e-6
    assert sizes[-1] <= last_mb
    assert all(s <= 25.0 + 16.0 for s in sizes[:-1])      # a bucket may end on one big tensor
    # buckets tile the arena in order, every parameter exactly once
    seen = [i for b in dp.buckets for i in b.params]
    assert seen == list(range(len(dp.flat.params)))
    # uncapped: the tail is whatever remains after the 25 MiB buckets
    dp2 = DataParallel(build_model("resnet50", num_classes=1000, stem="imagenet"), None,
                       last_bucket_mb=None)
    assert dp2.bucket_sizes_mb()[-1] > last_mb


class _FactoryComm:
    def __init__(self, uid, rank):
        self.uid, self.rank, self.aborted = uid, rank, 0

    def abort(self):
        self.aborted += 1


def _create_worker(rank, world, port, out, fault, peer_init_fails):
    import datetime
    import time
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    spec_fails = fault.startswith("spec:")     # stream_spec() raising on that rank
    if fault and not spec_fails:
        os.environ["PMD_FAULT_RCCL_CREATE"] = fault
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    made = []

    def factory(uid, rk, w, dev, prio, stream, timeout):
        # the native constructor's contract: a rank whose peer never completes the init
        # gives up after `timeout` (non-blocking init + deadline) instead of hanging
        if peer_init_fails and rk == 1:
            raise RuntimeError("ncclCommInitRankConfig failed: injected")
        if peer_init_fails:
            time.sleep(min(timeout, 1.0))
            raise RuntimeError("rccl: ncclCommInitRank did not complete (a peer rank never joined)")
        c = _FactoryComm(uid, rk)
        made.append(c)
        return c

    t0 = time.time()
    res = {"rank": rank}
    try:
        def stream_spec():
            if spec_fails and int(fault[5:]) == rank:
                raise ImportError("injected: the step streams could not be resolved")
            return 0, 0
        c = rccl.create(factory=factory, uid_fn=lambda: b"u" * 128, init_timeout_s=1.0,
                        stream_spec=stream_spec)
        res.update(ok=True, uid=c.uid == b"u" * 128)
    except RuntimeError as e:
        res.update(ok=False, err=str(e))
    res["secs"] = time.time() - t0
    res["aborted"] = [c.aborted for c in made]
    # the process group still works: nobody is stuck in a native collective
    x = torch.ones(1)
    dist.all_reduce(x)
    res["after"] = float(x)
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("fault,peer_init_fails", [("", False), ("1:init", False), ("0:uid", False),
                                                   ("", True), ("spec:1", False), ("spec:0", False)])
def test_rccl_create_is_all_or_nothing(tmp_path, fault, peer_init_fails):
    """a communicator-creation failure on ONE rank must not leave its peers stuck in
    ncclCommInitRank / the self-test.  Every rank agrees (c10d MIN) before the init and after
    it, so either all ranks get a communicator or all raise the same error -- quickly."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "res")
    mp.spawn(_create_worker, args=(2, _free_port(), out, fault, peer_init_fails), nprocs=2, join=True)
    res = [torch.load(f"{out}.{r}", weights_only=False) for r in range(2)]
    expect_ok = not fault and not peer_init_fails
    for r in res:
        assert r["ok"] is expect_ok, r
        assert r["after"] == 2.0 and r["secs"] < 30, r
        if expect_ok:
            assert r["uid"]
        else:
            assert "not created" in r["err"] or "init failed" in r["err"], r
