"""Tracing and debug instrumentation.

* ``region(name)`` -- a roctx range (native ``roctxRangePushA``/``Pop`` from
  the extension) around a phase of the step: ``fwd``, ``bwd``, ``opt``,
  ``comm``...  Recorded by ``rocprofv3 --marker-trace``; free when
  ``PMD_ROCTX`` is unset (the default).
* ``PMD_SYNC_DEBUG=1`` -- every gfx950 primitive is followed by a device
  synchronize and error check, so an asynchronous fault is reported at the
  op that caused it (the HIP analogue of CUDA_LAUNCH_BLOCKING; combine with
  ``AMD_SERIALIZE_KERNEL=3`` for the runtime's own serialisation).
"""
from __future__ import annotations

import contextlib
import functools
import os

_ROCTX = os.environ.get("PMD_ROCTX", "0") == "1"


def roctx_enabled() -> bool:
    return _ROCTX


def enable_roctx(flag: bool = True):
    global _ROCTX
    _ROCTX = bool(flag)


@contextlib.contextmanager
def region(name: str):
    if not _ROCTX:
        yield
        return
    from ..ops.native import C
    C.roctx_push(name)
    try:
        yield
    finally:
        C.roctx_pop()


def mark(name: str):
    if _ROCTX:
        from ..ops.native import C
        C.roctx_mark(name)


def sync_debug_enabled() -> bool:
    return os.environ.get("PMD_SYNC_DEBUG", "0") == "1"


# HIP streams that carried framework kernels (PMD_SYNC_DEBUG): see check_stream_budget
STEP_STREAMS: set = set()
HW_QUEUES = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)


def check_stream_budget(comm=None, model=None):
    """Debug check (PMD_SYNC_DEBUG=1, once per step): the rank's step work must fit the
    hardware queues one stream each (docs/ARCHITECTURE.md, "Streams -> hardware queues").
    Counts every HIP stream a framework kernel was launched on, the SyncBN exchange's side
    stream, and the gradient-bucket transport's stream (the native RcclComm's, or
    ProcessGroupNCCL's internal one); raises if they exceed GPU_MAX_HW_QUEUES (default 4),
    i.e. if two streams -- possibly both carrying cross-rank waits -- could share a queue."""
    streams = set(STEP_STREAMS)
    if comm is not None:
        side = getattr(comm, "_side", None)
        if side is not None:
            streams.add(int(side.cuda_stream))
    transport = getattr(model, "transport", None) if model is not None else None
    rc = getattr(model, "rccl", None) if model is not None else None
    if rc is not None:
        streams.add(int(rc.stream_handle))
    elif transport == "c10d" and comm is not None and getattr(comm, "backend", "") == "nccl":
        streams.add("c10d-processgroupnccl")
    if len(streams) > HW_QUEUES:
        raise RuntimeError(f"[PMD_SYNC_DEBUG] step work on {len(streams)} HIP streams > {HW_QUEUES} hardware "
                           f"queues (GPU_MAX_HW_QUEUES): two streams would share a queue ({sorted(map(str, streams))})")
    return len(streams)


def wrap_sync_debug(module_globals: dict, names):
    """Replace ``names`` in a module namespace by versions that synchronize
    the device after the call and re-raise any HIP error with the op name
    (and record the stream each ran on, for :func:`check_stream_budget`)."""
    import torch

    def make(fn, nm):
        @functools.wraps(fn)
        def wrapped(*a, **k):
            STEP_STREAMS.add(int(torch.cuda.current_stream().cuda_stream))
            out = fn(*a, **k)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:  # surface the failing primitive
                raise RuntimeError(f"[PMD_SYNC_DEBUG] device error after {nm}: {e}") from e
            return out
        return wrapped

    for nm in names:
        module_globals[nm] = make(module_globals[nm], nm)
