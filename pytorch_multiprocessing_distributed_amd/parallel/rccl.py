"""Native RCCL communicator bootstrap (reference
main.py:190-193, where ``init_process_group('nccl')`` hides all of this).

``init_process_group`` has already created the c10d TCPStore on
``MASTER_ADDR:MASTER_PORT``; it is the only piece borrowed from c10d.  Rank 0
calls ``ncclGetUniqueId`` and publishes the 128-byte id under a fresh store
key; every rank reads it and calls ``ncclCommInitRank`` on its own HIP device
(csrc/runtime/rccl_comm.cpp).  The resulting communicator owns one HIP
stream of the requested priority; the gradient reducer launches its bucket
all-reduces there, fenced with HIP events (no host blocking).
"""
from __future__ import annotations

import itertools
import weakref

import torch
import torch.distributed as dist

_SEQ = itertools.count()
# every live native communicator of this process, so a failing rank can abort
# them all (launch.abort) and its peers' RCCL kernels error out instead of
# waiting for a rank that will never arrive
_LIVE: "weakref.WeakSet" = weakref.WeakSet()
_STRONG: list = []          # objects that cannot be weakly referenced


def register(comm):
    """Track ``comm`` (anything with ``abort()``) for :func:`abort_all`."""
    try:
        _LIVE.add(comm)
    except TypeError:
        _STRONG.append(comm)
    return comm


def live():
    return list(_LIVE) + list(_STRONG)


def abort_all() -> int:
    """``ncclCommAbort`` every live native communicator; returns how many.
    Best effort: one communicator failing to abort never stops the others."""
    n = 0
    for c in live():
        try:
            c.abort()
            n += 1
        except Exception:  # noqa: BLE001 -- already failing; never mask the original error
            pass
    _LIVE.clear()
    _STRONG.clear()
    return n


def _store():
    from torch.distributed import distributed_c10d as c10d
    return c10d._get_default_store()


def create(group=None, priority: int = 0, store=None, stream: int = 0):
    """Collective over ``group`` (every rank calls it).  Returns ``_C.RcclComm``.
    ``stream``: HIP handle of an existing stream to run on (0: the communicator creates one)."""
    from ..ops.native import C
    if not dist.is_initialized():
        raise RuntimeError("torch.distributed must be initialised first (it hosts the TCPStore)")
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    store = store if store is not None else _store()
    key = f"pmd_rccl_uid_{next(_SEQ)}"
    if rank == 0:
        store.set(key, C.RcclComm.unique_id())
    uid = store.get(key)                      # blocks until rank 0 published it
    dev = torch.cuda.current_device()
    comm = C.RcclComm(bytes(uid), rank, world, dev, priority, stream)
    return register(comm)


def create_single(device: int | None = None, priority: int = 0):
    """A one-rank communicator (no process group needed): exercises the real
    RCCL launch / stream / event path on one GPU (tests, W=1 benches)."""
    from ..ops.native import C
    dev = torch.cuda.current_device() if device is None else device
    return register(C.RcclComm(bytes(C.RcclComm.unique_id()), 0, 1, dev, priority))


def self_test(c, group=None, n: int = 4097, rounds: int = 2) -> bool:
    """Collective over ``group`` (every rank calls it; host-syncing, run once at
    setup, like ``XgmiAllReduce.self_test``): exact check of the native
    communicator on rank-dependent integers -- SUM all-reduce, AVG all-reduce
    (the reducer's op) and a broadcast from rank 0 -- plus its asynchronous error
    state.  The verdict is agreed on by all ranks (MIN over the process group),
    so every rank takes the same transport decision."""
    dev = torch.device("cuda", c.device)
    W, r0 = c.world, c.rank
    ok = True
    try:
        i = torch.arange(n, device=dev, dtype=torch.float32)
        for r in range(rounds):
            s = i + 1000.0 * r0 + r
            c.all_reduce_(s, 0)
            a = i * (r0 + 1)
            c.all_reduce_(a, 1)
            b = torch.full((n,), float(7 * r0 + 3 + r), device=dev)
            c.broadcast_(b, 0)
            torch.cuda.synchronize(dev)
            want_s = i * W + 1000.0 * (W * (W - 1) / 2) + r * W
            want_a = i * ((W + 1) / 2.0)
            ok = (ok and bool(torch.equal(s, want_s))
                  and bool(torch.allclose(a, want_a, rtol=1e-6, atol=0.0))
                  and bool(torch.all(b == float(3 + r)).item()) and bool(c.check()))
    except Exception:  # noqa: BLE001 -- a failing communicator is a failed test, agreed below
        ok = False
    if dist.is_initialized():
        flag = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        ok = bool(flag.item() == 1)
    return ok
