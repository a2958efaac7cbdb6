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


def wrap_sync_debug(module_globals: dict, names):
    """Replace ``names`` in a module namespace by versions that synchronize
    the device after the call and re-raise any HIP error with the op name."""
    import torch

    def make(fn, nm):
        @functools.wraps(fn)
        def wrapped(*a, **k):
            out = fn(*a, **k)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:  # surface the failing primitive
                raise RuntimeError(f"[PMD_SYNC_DEBUG] device error after {nm}: {e}") from e
            return out
        return wrapped

    for nm in names:
        module_globals[nm] = make(module_globals[nm], nm)
