"""One-shot xGMI all-reduce for SyncBN statistics.

SyncBN's per-layer collectives are tiny (2C+1 floats forward, 2C backward;
<= 16 KiB) and sit on the critical path 2x53 times per ResNet-50 step
(reference main.py:43 -> torch:nn/modules/_functions.py:65-83, 155-165).
For those, a ring all-reduce is latency-bound: 2(W-1) dependent link hops
plus RCCL's launch/proxy overhead.  ``XgmiAllReduce`` instead peer-maps one
receive buffer per rank (HIP IPC; handles exchanged through the c10d
store) and runs a single kernel that pushes the vector to every peer over
the point-to-point xGMI links, signals, waits and sums locally in rank
order (kernels/xgmi.hip).  Large messages (gradient buckets) stay on RCCL,
which is bandwidth-optimal for them.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class XgmiAllReduce:
    def __init__(self, group=None, timeout_s: float = 60.0):
        from ..ops.native import C
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        dev = torch.cuda.current_device()
        # every step is agreed on by all ranks, so a local failure (e.g. IPC not
        # permitted) raises on EVERY rank instead of leaving peers in a barrier
        err = ""
        handle = b""
        try:
            self._c = C.XgmiComm(self.rank, self.world_size, dev, timeout_s)
            handle = self._c.handle()
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        handles = [None] * self.world_size
        dist.all_gather_object(handles, handle, group=group)
        if not err:
            try:
                self._c.open(handles)
            except Exception as e:  # noqa: BLE001
                err = f"rank {self.rank}: {e}"
        torch.cuda.synchronize()
        flag = torch.tensor([0 if err else 1], device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if flag.item() != 1:
            raise RuntimeError(f"xGMI transport setup failed ({err or 'on a peer rank'})")
        # nobody may write into a peer buffer before every rank mapped its peers
        dist.barrier(group=group)
        self.capacity = self._c.capacity

    def self_test(self, n: int = 4097, rounds: int = 3) -> bool:
        """Collective: exact check of the kernel against the known sum of
        rank-dependent integers (run once at setup; host-syncing)."""
        ok = True
        for r in range(rounds):
            t = torch.arange(n, device="cuda", dtype=torch.float32) + 1000.0 * self.rank + r
            self._c.all_reduce_(t)
            W = self.world_size
            want = (torch.arange(n, device="cuda", dtype=torch.float32) * W
                    + 1000.0 * (W * (W - 1) / 2) + r * W)
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(t, want)) and self._c.check()
        flag = torch.tensor([1 if ok else 0], device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item() == 1)

    def accepts(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                and t.numel() <= self.capacity)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM across ranks on the current stream (no host sync)."""
        return self._c.all_reduce_(t)

    def check(self):
        """Host-blocking health check: raises if any call timed out on a peer."""
        if not self._c.check():
            raise RuntimeError(f"xGMI all-reduce timed out waiting for a peer (rank {self.rank})")

    def raise_if_failed(self):
        """Non-blocking health check (host-mapped error word, no device sync):
        raises if any exchange that has COMPLETED so far timed out on a peer.
        The training loop calls it after every step; a timed-out exchange has
        produced wrong statistics, so training must not continue."""
        if self._c.failed():
            raise RuntimeError(f"xGMI SyncBN exchange timed out waiting for a peer (rank {self.rank}, "
                               f"timeout {self._c.timeout:.3g} s): statistics of that step are invalid")

    def set_timeout(self, seconds: float):
        self._c.set_timeout(float(seconds))

    @property
    def calls(self):
        return self._c.calls

    # ------------------------------------------------------------ SyncBN fused
    def _site(self, bn):
        """Native site id of a BN module: its Parameter / buffer objects registered once
        (XgmiComm.add_site), so a step's exchange passes only its per-step tensors."""
        key = getattr(bn, "_pmd_xgmi_site", None)
        if key is None or key[0] != id(self):
            sid = self._c.add_site(bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                   bn.num_batches_tracked, float(bn.eps), float(bn.momentum))
            key = (id(self), sid)
            bn._pmd_xgmi_site = key
        return key[1]

    def bn_fwd(self, slots_a, slots_b, count, bn_a, bn_b, params_a, params_b, count_out,
               shift_a=None, shift_b=None):
        """Collapse the conv-epilogue statistic slots, exchange, finalize: ONE
        kernel per BN site (see xgmi_bn_kernel).  Slots are cleared.  ``shift_*``:
        the statistics shifts the slots were accumulated about (identical on every
        rank), overwritten with the global batch means."""
        self._c.bn_fwd(slots_a, slots_b, float(count), self._site(bn_a),
                       -1 if bn_b is None else self._site(bn_b), params_a, params_b, count_out,
                       shift_a, shift_b)

    def bn_bwd(self, slots_a, slots_b, acc_a, acc_b, out_a, out_b):
        """Collapse the BN-backward reduce slots (+= local sums into the gamma/beta
        gradient arena), exchange, write global [2][C] sums."""
        aa = acc_a or (None, None)
        ab = acc_b or (None, None)
        self._c.bn_bwd(slots_a, slots_b, aa[0], aa[1], ab[0], ab[1], out_a, out_b)
