"""Communicator used by the reducer, SyncBN and metric reduction.

On an MI355X node the process group backend is ``"nccl"``, which on
PyTorch-ROCm *is* RCCL: collectives run over xGMI on RCCL's own HIP stream
and are ordered against the caller's current stream with HIP events (no host
blocking).  On CPU the same interface runs on gloo (BASELINE config 1).

Reference touchpoints: C1 init_process_group (main.py:190-193),
C3 initial broadcast, C5/C6 SyncBN statistics, C7 bucketed gradient
all-reduce, C8 metric reduction (main.py:173-177, dead in the reference),
C9 teardown (main.py:84).
"""
from __future__ import annotations

import hashlib
import os
import zlib

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, group=None):
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        # RCCL implements ncclAvg; gloo does not -> pre-scale there
        self.supports_avg = self.backend == "nccl"
        self.xgmi = None   # one-shot xGMI path for SyncBN statistics (enable_xgmi)
        # collective-order checker: rolling hash of every collective
        # issued through this object; verify_order() compares it across ranks
        self.order_check_every = int(os.environ.get("PMD_CHECK_ORDER", "0"))
        self._seq = 0
        self._ncoll = 0
        # PMD_SYNCBN_OVERLAP=1: backward SyncBN exchanges on a high-priority side stream
        # (forked after the producing dgrad, joined before bn_bwd_elemt).  Off by default
        # since round 4: the main stream has nothing to run between the two (the weight
        # gradients already live on their own stream), so the fork/join only added two
        # cross-stream hops per BN site -- 21.14 vs 20.86 ms per ResNet-50 step in the
        # W=1 rehearsal (profiles/rehearsal_r04.txt)
        self.overlap_bn_bwd = os.environ.get("PMD_SYNCBN_OVERLAP", "0") == "1"
        self._side = None
        # native communicators carrying in-step traffic (the gradient reducer's
        # RcclComm): their asynchronous error state is part of raise_if_failed
        self.natives = []
        # set while a native communicator carries the gradient buckets: a c10d
        # collective inside the step would then run next to them on another
        # stream (cross-rank deadlock hazard), so the SyncBN path must never fall
        # back to the process group
        self.in_step_c10d_forbidden = False

    def side_stream(self):
        """High-priority HIP stream for latency-bound SyncBN exchanges (GPU only)."""
        if self._side is None:
            import torch
            self._side = torch.cuda.Stream(priority=-1)
        return self._side

    def _record(self, op, t):
        if not self.order_check_every:          # checker off: no per-collective hashing
            self._ncoll += 1
            return
        key = f"{op}:{t.numel()}:{t.dtype}".encode()
        self._seq = (self._seq * 1000003 + zlib.crc32(key)) & 0x7FFFFFFFFFFFFFF
        self._ncoll += 1

    def verify_order(self, extra=()):
        """Collective: raise if ranks issued different collective sequences since
        construction (op, size, dtype, in order) -- the classic silent-hang /
        wrong-result bug of data-parallel code.  ``extra`` folds in sequences
        issued outside this object (the native reducer's bucket launch order)."""
        text = f"{self._seq}:{self._ncoll}:{list(extra)}"
        self.check_same(text, "collective sequence")

    def raise_if_failed(self):
        """Cheap per-step health check (no device sync): xGMI exchange timeouts
        (host-mapped error word) and the asynchronous error state of every
        attached native RCCL communicator (``ncclCommGetAsyncError``)."""
        if self.xgmi is not None:
            self.xgmi.raise_if_failed()
        for c in self.natives:
            if not c.check():
                raise RuntimeError(f"native RCCL communicator failed or was aborted (rank {self.rank}): "
                                   "gradient all-reduces of this step are invalid")

    def attach_native(self, c):
        """Fold a native communicator into :meth:`raise_if_failed`."""
        if c is not None and c not in self.natives:
            self.natives.append(c)
        return c

    def enable_xgmi(self, timeout_s: float | None = None):
        """Route small fp32 GPU all-reduces (SyncBN statistics) through the
        one-shot xGMI kernel (parallel/xgmi.py).  Collective: every rank calls it."""
        from .xgmi import XgmiAllReduce
        if timeout_s is None:
            timeout_s = float(os.environ.get("PMD_XGMI_TIMEOUT", "60"))
        self.xgmi = XgmiAllReduce(self.group, timeout_s)
        return self.xgmi

    # ------------------------------------------------------------ blocking
    def all_reduce_(self, t, op=dist.ReduceOp.SUM):
        self._record("all_reduce", t)
        dist.all_reduce(t, op=op, group=self.group)
        return t

    def all_reduce_stats_(self, t):
        """SUM all-reduce of a small statistics vector (SyncBN).  One-shot xGMI
        kernel when enabled and the message fits, RCCL/gloo otherwise."""
        x = self.xgmi
        if x is not None and x.accepts(t):
            self._record("xgmi_all_reduce", t)
            return x.all_reduce_(t)
        if self.in_step_c10d_forbidden:
            raise RuntimeError(
                f"SyncBN statistics message of {t.numel()} floats does not fit the xGMI kernel "
                f"(capacity {x.capacity if x is not None else 0}) and the gradient buckets run on a "
                "native RCCL communicator: a c10d fallback would put two communicators' collectives "
                "in flight at once; use --comm c10d")
        return self.all_reduce_(t)

    def fused_bn_ok(self, t):
        """Can the fused SyncBN statistics kernel handle these slot buffers?"""
        return self.xgmi is not None and t.is_cuda and t.dim() == 3 and t.shape[0] == 64

    def bn_stats_fwd(self, slots_a, slots_b, count, bn_a, bn_b, params_a, params_b, count_out,
                     shift_a=None, shift_b=None):
        self._record("xgmi_bn_fwd", slots_a)
        self.xgmi.bn_fwd(slots_a, slots_b, count, bn_a, bn_b, params_a, params_b, count_out,
                         shift_a, shift_b)

    def bn_stats_bwd(self, slots_a, slots_b, acc_a, acc_b, out_a, out_b):
        self._record("xgmi_bn_bwd", slots_a)
        self.xgmi.bn_bwd(slots_a, slots_b, acc_a, acc_b, out_a, out_b)

    def broadcast_(self, t, src=0):
        self._record("broadcast", t)
        dist.broadcast(t, src=src, group=self.group)
        return t

    def all_gather(self, t):
        self._record("all_gather", t)
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t, group=self.group)
        return out

    def barrier(self):
        if self.backend == "nccl" and torch.cuda.is_available():
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    # --------------------------------------------------------------- async
    def all_reduce_mean_async(self, t):
        """Average ``t`` in place across ranks; returns a Work handle."""
        self._record("all_reduce_mean", t)
        if self.supports_avg:
            return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        t.mul_(1.0 / self.world_size)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    # --------------------------------------------------------------- utils
    def reduce_mean(self, t):
        """Reference ``reduce_tensor`` (main.py:173-177): clone, SUM, /W."""
        rt = t.clone()
        self.all_reduce_(rt)
        rt /= self.world_size
        return rt

    def check_same(self, text: str, what="value"):
        """Verify a host string is identical on all ranks (param-shape check,
        collective-order check).  Raises on mismatch."""
        h = int(hashlib.sha1(text.encode()).hexdigest()[:15], 16)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else "cpu"
        t = torch.tensor([h, -h], dtype=torch.int64, device=dev)
        mx = t.clone()
        self.all_reduce_(mx, op=dist.ReduceOp.MAX)
        if int(mx[0]) != h or int(mx[1]) != -h:
            raise RuntimeError(f"{what} differs across ranks (rank {self.rank})")


def get_comm(group=None):
    if not dist.is_available() or not dist.is_initialized():
        return None
    if dist.get_world_size(group) == 1:
        return None
    return Comm(group)
