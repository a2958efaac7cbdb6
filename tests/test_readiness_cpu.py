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
    assert config.parse_args([]).comm == "c10d"
    assert config.parse_args(["--comm", "rccl"]).comm == "rccl"
    with pytest.raises(SystemExit):
        config.parse_args(["--comm", "mpi"])


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
        s.xgmi = object()                    # one-shot xGMI exchange: allowed
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
