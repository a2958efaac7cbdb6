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
import os
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


def _agree(ok: bool, group=None) -> bool:
    """MIN of a 0/1 flag over the process group (c10d: gloo or ProcessGroupNCCL -- never a
    native communicator), so every rank takes the same branch."""
    if not dist.is_initialized():
        return ok
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    flag = torch.tensor([1 if ok else 0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item() == 1)


def _fault_here(stage: str) -> bool:
    """Fault injection for tests: PMD_FAULT_RCCL_CREATE=<rank>[:<stage>] makes that rank fail
    its communicator creation at ``stage`` ("uid" = before the unique-id exchange, "init" =
    right before ncclCommInitRank; default "init")."""
    spec = os.environ.get("PMD_FAULT_RCCL_CREATE", "")
    if not spec:
        return False
    r, _, st = spec.partition(":")
    return int(r) == dist.get_rank() and (st or "init") == stage


def create(group=None, priority: int = 0, store=None, stream: int = 0, init_timeout_s: float | None = None,
           factory=None, uid_fn=None, stream_spec=None):
    """Collective over ``group`` (every rank calls it).  Returns ``_C.RcclComm``, or raises
    the SAME RuntimeError on every rank: no rank ever enters a native collective
    that a peer will not join.

      1. rank 0 publishes the unique id -- or the reason it could not make one -- under a
         fresh store key; every rank reads it (bounded by the store timeout);
      2. every rank agrees (c10d MIN) that it holds a valid id before ANY rank calls
         ncclCommInitRank -- a rank that failed so far skips the init, and so do its peers;
      3. the init itself is non-blocking and bounded (``init_timeout_s``, env
         ``PMD_RCCL_INIT_TIMEOUT``, default 300 s), so a peer failing INSIDE its init cannot
         hang this rank;
      4. every rank agrees that its communicator exists before anything uses it; on any
         failure each rank aborts its own communicator and raises.

    ``factory(uid, rank, world, device, priority, stream, timeout)`` / ``uid_fn()``: test
    doubles for the native constructor / ncclGetUniqueId (tests/test_readiness_cpu.py).
    ``stream_spec()`` -> (priority, stream handle): resolved HERE, inside the agreement
    protocol, so a rank failing to produce them fails the creation on every rank
    instead of skipping ``create`` while its peers wait in its first agreement."""
    if not dist.is_initialized():
        raise RuntimeError("torch.distributed must be initialised first (it hosts the TCPStore)")
    if init_timeout_s is None:
        init_timeout_s = float(os.environ.get("PMD_RCCL_INIT_TIMEOUT", "300"))
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    store = store if store is not None else _store()
    key = f"pmd_rccl_uid_{next(_SEQ)}"
    err = ""
    try:
        if factory is None or uid_fn is None:
            from ..ops.native import C
            factory = factory or C.RcclComm
            uid_fn = uid_fn or C.RcclComm.unique_id
        if stream_spec is not None:
            priority, stream = stream_spec()
    except Exception as e:  # noqa: BLE001 -- agreed on below, with every peer
        err = f"rank {rank}: communicator prerequisites: {e}"
    if rank == 0 and err:
        store.set(key, b"ERR:" + err.encode()[:200])
    elif rank == 0:
        try:
            if _fault_here("uid"):
                raise RuntimeError("injected unique-id failure (PMD_FAULT_RCCL_CREATE)")
            store.set(key, b"OK:" + bytes(uid_fn()))
        except Exception as e:  # noqa: BLE001
            err = f"rank 0: ncclGetUniqueId: {e}"
            store.set(key, b"ERR:" + err.encode()[:200])
    uid = None
    try:
        v = bytes(store.get(key))                    # blocks until rank 0 published (store timeout)
        if v.startswith(b"OK:"):
            uid = v[3:]
        else:
            err = err or v[4:].decode(errors="replace")
    except Exception as e:  # noqa: BLE001
        err = err or f"rank {rank}: unique id not received: {e}"
    if uid is not None and _fault_here("init"):
        err, uid = f"rank {rank}: injected init failure (PMD_FAULT_RCCL_CREATE)", None
    if not _agree(uid is not None and not err, group):
        raise RuntimeError(f"native RCCL communicator not created: {err or 'a peer rank failed before init'}")
    comm = None
    try:
        dev = torch.cuda.current_device() if torch.cuda.is_available() else 0
        comm = factory(uid, rank, world, dev, priority, stream, init_timeout_s)
    except Exception as e:  # noqa: BLE001
        err = f"rank {rank}: {e}"
    if not _agree(comm is not None, group):
        if comm is not None:
            try:
                comm.abort()
            except Exception:  # noqa: BLE001
                pass
        raise RuntimeError(f"native RCCL communicator init failed: {err or 'on a peer rank'}")
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
