"""Process launch and process-group bootstrap.

* :func:`run_model` -- the reference's launcher (main.py:180-188): create
  ``save_path``, snapshot the entry script into it, then
  ``torch.multiprocessing.spawn(fn, nprocs=W, join=True)`` (fail-fast join:
  the first rank to die terminates the others and re-raises its traceback).
* :func:`init_process` -- rendezvous on ``MASTER_ADDR:MASTER_PORT``
  (reference hard-codes 127.0.0.1:20080, main.py:190-193; here the
  environment or flags override), binds rank -> local GPU, and
  creates the process group: backend ``"nccl"`` (= RCCL on ROCm, over xGMI)
  with GPUs, ``"gloo"`` on CPU.
* optional fault injection for tests: ``PMD_FAULT_RANK`` / ``PMD_FAULT_STEP``.
* :func:`abort` -- communicator abort on a rank failure (peers unblock).
"""
from __future__ import annotations

import datetime
import os
import shutil

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

DEFAULT_ADDR = "127.0.0.1"
DEFAULT_PORT = 20080


def resolve_device(kind="auto"):
    if kind == "cpu":
        return "cpu"
    if kind == "cuda":
        return "cuda"
    return "cuda" if torch.cuda.is_available() else "cpu"


def init_process(rank, world_size, backend="auto", device="auto", master_addr=None,
                 master_port=None, timeout_min=30):
    os.environ["MASTER_ADDR"] = master_addr or os.environ.get("MASTER_ADDR", DEFAULT_ADDR)
    os.environ["MASTER_PORT"] = str(master_port or os.environ.get("MASTER_PORT", DEFAULT_PORT))
    # dmabuf IPC is the only mode the MI355X host driver supports for RCCL peer buffers
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev_kind = resolve_device(device)
    if backend in ("auto", None):
        backend = "nccl" if dev_kind == "cuda" else "gloo"
    if backend == "rccl":
        backend = "nccl"
    if dev_kind == "cuda":
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        # the step's own streams before the process group creates any (one hardware
        # queue each: ops/functional.py init_step_streams)
        from .ops import functional as OF
        OF.init_step_streams(dev)
    else:
        dev = torch.device("cpu")
    kw = dict(backend=backend, rank=rank, world_size=world_size,
              timeout=datetime.timedelta(minutes=timeout_min))
    if backend == "nccl":
        kw["device_id"] = dev
    dist.init_process_group(**kw)
    return dev


def shutdown():
    if dist.is_available() and dist.is_initialized():
        # unreachable DataParallel wrappers (kept in cycles by their gradient hooks) and the
        # native reducer that holds the process group go first, then the group itself
        import gc
        gc.collect()
        dist.destroy_process_group()


def abort():
    """Abort the communicators of this rank (RCCL: ``ncclCommAbort``) after a
    local failure, so peers blocked in a collective fail fast instead of
    waiting out the collective timeout.  Best effort.  Covers the
    framework's own communicators (``parallel.rccl``: the ``--comm rccl``
    gradient transport) as well as the c10d process group."""
    from .parallel import rccl
    rccl.abort_all()
    if not (dist.is_available() and dist.is_initialized()):
        return
    try:
        from torch.distributed.distributed_c10d import _abort_process_group
        _abort_process_group()
    except Exception:  # noqa: BLE001 -- already failing; never mask the original error
        pass


def run_model(main_fn, world_size, save_path=None, snapshot=None, args=()):
    if save_path:
        os.makedirs(save_path, exist_ok=True)
        if snapshot:
            shutil.copy(snapshot, os.path.join(save_path, "main.py"))
    os.environ.setdefault("PYTHONWARNINGS", "ignore:semaphore_tracker:UserWarning")
    mp.spawn(main_fn, args=(world_size, *args), nprocs=world_size, join=True)


def maybe_inject_fault(rank, step):
    """Test hooks: ``PMD_FAULT_RANK``/``PMD_FAULT_STEP`` raise on
    that rank at that step; ``PMD_FAULT_DELAY=rank:step:seconds`` makes that
    rank a straggler (host sleep before the step), which drives its peers'
    SyncBN exchanges into their timeout."""
    fr = os.environ.get("PMD_FAULT_RANK")
    fs = os.environ.get("PMD_FAULT_STEP")
    if fr is not None and fs is not None and int(fr) == rank and int(fs) == step:
        raise RuntimeError(f"injected fault on rank {rank} at step {step}")
    fd = os.environ.get("PMD_FAULT_DELAY")
    if fd:
        r, s, sec = fd.split(":")
        if int(r) == rank and int(s) == step:
            import time
            time.sleep(float(sec))
