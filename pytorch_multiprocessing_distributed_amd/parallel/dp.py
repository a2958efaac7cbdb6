"""Synchronous data parallelism: the framework's replacement for
``torch.nn.parallel.DistributedDataParallel`` (reference main.py:44).

What it does:
  * construction: verifies parameter names/shapes agree on every rank (C2),
    re-homes parameters/grads into flat arenas (:mod:`.flat`), then
    broadcasts the parameter arena and all buffers from rank 0 in one
    collective per dtype (C3) -- replicas start identical (README.md:6);
  * backward: gradients accumulate straight into the grad arena; a hook
    counts readiness per bucket and buckets are launched as asynchronous
    in-place *average* all-reduces strictly in bucket-index order (a
    cursor, like DDP's ``next_bucket``: every rank issues the identical
    collective sequence), overlapping the rest of backward.  Buckets are
    contiguous arena slices with a small first bucket (DDP: 1 MiB first /
    25 MiB rest; sized here for xGMI rings, see ``bucket_mb``);
  * after the first iteration the arena is re-laid out in the OBSERVED
    gradient-ready order (rank 0's order, broadcast) and the buckets are
    rebuilt over it -- torch's Reducer does the same
    (torch:nn/parallel/distributed.py:1551, ``_rebuild_buckets``);
  * end of backward (autograd engine callback): joins the side-stream weight
    gradients still pending (``functional.flush_pending_wgrads``, BEFORE any
    bucket is force-launched), waits on every bucket (stream-side, no host
    block) and checks each bucket fired exactly once;
  * transport: ``"c10d"`` -- the torch process group (RCCL via
    ProcessGroupNCCL on GPU, gloo on CPU) -- or ``"rccl"`` -- the framework's
    own RCCL communicator (csrc/runtime/rccl_comm.cpp: uniqueId over the
    TCPStore, its own HIP stream, hipEvent fences, exact startup self-test,
    async-error check every step); ``"auto"`` (default) picks ``rccl`` whenever
    it can be the only in-step communicator (:func:`resolve_transport`);
  * the bucket bookkeeping + collective launch runs in the native C++
    ``_C.Reducer`` (csrc/runtime/reducer.cpp); ``reducer="python"`` keeps an
    equivalent pure-Python implementation for debugging / cross-checking;
  * ``compress="bf16"`` sends gradients over the wire in bf16 (half the xGMI
    bytes, fp32 arena kept);
  * ``no_sync()`` skips communication for gradient accumulation;
  * ``broadcast_buffers=True`` re-broadcasts BN buffers from rank 0 before
    each training forward (reference DDP default, C4); off by default since
    SyncBN keeps them identical;
  * ``timeline=True`` (or ``PMD_REDUCER_TIMELINE=1``) records each bucket's
    launch time and, on the RCCL transport, its device start/end relative to
    the end of backward (``bucket_timeline()``).

``state_dict()`` carries the ``module.`` prefix exactly like the reference's
DDP checkpoint (main.py:77).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from .comm import Comm
from .flat import flatten_module


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "work", "fired")

    def __init__(self, index, start, end, params):
        self.index = index
        self.start = start
        self.end = end
        self.params = params
        self.pending = len(params)
        self.work = None
        self.fired = 0


def _max_bn_stats_floats(module):
    """Largest SyncBN statistics message the model can send through
    ``Comm.all_reduce_stats_``: a projection block exchanges both of its BNs'
    [sum | sum^2] in one vector (+1 count), so 4 * max(C) + 1 bounds it."""
    cs = [int(m.num_features) for m in module.modules()
          if hasattr(m, "num_features") and hasattr(m, "running_mean")]   # ours and nn.BatchNorm*
    return 4 * max(cs) + 1 if cs else 0


def _check_single_in_step_communicator(comm, module=None):
    """``transport='rccl'`` puts the bucket all-reduces on a SECOND communicator
    (the native ``RcclComm``, its own HIP stream).  Two communicators with
    blocking collective kernels in flight at once on different streams can
    deadlock across ranks, so the only other in-step traffic allowed next to it
    is the one-shot xGMI SyncBN exchange (a kernel of ours with a wall-clock
    bounded spin, not a c10d collective).  SyncBN statistics over c10d (gloo or
    ProcessGroupNCCL) inside the step would be concurrent with the bucket
    all-reduces: refused.  (The once-per-run c10d traffic -- the bucket-rebuild
    order broadcast and the tuning-table broadcast -- is issued from the
    forward / after the step, i.e. after the finalize made the compute stream
    wait on every bucket, and c10d fences its stream on the compute stream, so
    it is serialised behind the native collectives.)"""
    from ..ops import functional as OF
    sync = OF.get_bn_sync()
    if sync is not None and getattr(sync, "xgmi", None) is None:
        raise ValueError("transport='rccl' (--comm rccl) with SyncBN over the process group would run "
                         "collectives of two communicators concurrently; use --syncbn_comm xgmi, "
                         "--sync_bn off, or --comm c10d")
    if sync is not None and module is not None:
        need = _max_bn_stats_floats(module)
        if need > sync.xgmi.capacity:
            raise ValueError(f"transport='rccl': a SyncBN statistics message of up to {need} floats exceeds "
                             f"the xGMI kernel's capacity ({sync.xgmi.capacity}) and would fall back to a "
                             "c10d collective inside the step; use --comm c10d")


def resolve_transport(comm, module, reducer="native", transport="auto", verbose=True):
    """Pick the gradient-bucket transport.  ``"auto"`` (the default of main.py and
    bench.py) takes the native RCCL communicator when it can be the ONLY
    communicator with collectives inside the step -- native reducer, GPU ranks,
    SyncBN off or on the one-shot xGMI kernel with room for every statistics
    message -- and its exact startup self-test passes on every rank; otherwise
    torch's ProcessGroupNCCL (c10d).  Returns ``(transport, RcclComm or None)``;
    rank 0 prints the choice and the reason."""
    if comm is None:
        return "c10d", None
    if transport not in ("auto", "c10d", "rccl"):
        raise ValueError(f"bad transport {transport!r}")
    if transport == "c10d":
        return "c10d", None
    reason = ""
    if comm.backend != "nccl" and transport == "auto":
        return "c10d", None                 # CPU / gloo ranks: the process group is the transport
    if reducer != "native" or comm.backend != "nccl":
        reason = "needs the native reducer on GPU (nccl) ranks"
    else:
        try:
            _check_single_in_step_communicator(comm, module)
        except ValueError as e:
            reason = str(e)
    if reason:
        if transport == "rccl":
            raise ValueError(f"transport='rccl': {reason}")
        if verbose and comm.rank == 0:
            print(f"[pmd] gradient transport: c10d ({reason})", flush=True)
        return "c10d", None
    from . import rccl
    c, err = None, ""

    def stream_spec():
        from ..ops.functional import STREAM_PRIO, comm_stream_handle
        return STREAM_PRIO, comm_stream_handle()

    try:
        # collective and all-or-nothing: raises on EVERY rank when any rank failed -- also in
        # resolving the stream, which happens inside the agreement -- before
        # any native collective runs, so the self-test below runs on all or none
        c = rccl.create(comm.group, stream_spec=stream_spec)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    ok = rccl.self_test(c, comm.group) if c is not None else False
    if not ok:
        if c is not None:
            c.abort()
        msg = f"native RCCL communicator self-test failed{': ' + err if err else ''}"
        if transport == "rccl":
            raise RuntimeError(msg)
        if verbose and comm.rank == 0:
            print(f"[pmd] gradient transport: c10d ({msg})", flush=True)
        return "c10d", None
    if verbose and comm.rank == 0:
        print("[pmd] gradient transport: rccl (native RcclComm, exact self-test passed on "
              f"{comm.world_size} rank(s))", flush=True)
    return "rccl", c


def _flush_wgrads():
    from ..ops.functional import flush_pending_wgrads
    flush_pending_wgrads()


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, comm: Comm | None = None, bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, broadcast_buffers: bool = False,
                 check_collectives: bool = True, reducer: str = "native", compress: str = "none",
                 transport: str = "auto", rebuild_buckets: bool = True, timeline: bool | None = None,
                 last_bucket_mb: float | None = 2.0, post_hooks: str = "auto"):
        super().__init__()
        if post_hooks not in ("auto", "always"):
            raise ValueError(f"bad post_hooks {post_hooks!r}")
        # "auto": the fused model (ops/functional.py) writes EVERY parameter's gradient
        # straight into the arena and marks it itself (functional._ready), so the per-
        # parameter AccumulateGrad post-hooks -- which autograd runs for every parameter of
        # every step even when its node returned no gradient -- are pure host overhead
        # there (161 Python calls per ResNet-50 step, 467 for ResNet-152); an unmarked
        # gradient would still be all-reduced by the finalize, just without overlap
        self.post_hooks = post_hooks
        self.last_bucket_mb = last_bucket_mb
        self.module = module
        self.comm = comm
        self.world_size = comm.world_size if comm is not None else 1
        self.broadcast_buffers = broadcast_buffers
        self.check_collectives = check_collectives
        self.bucket_mb, self.first_bucket_mb = bucket_mb, first_bucket_mb
        if reducer not in ("native", "python") or compress not in ("none", "bf16") \
                or transport not in ("auto", "c10d", "rccl"):
            raise ValueError(f"bad reducer/compress/transport: {reducer!r}/{compress!r}/{transport!r}")
        if comm is not None:
            desc = ";".join(f"{n}:{tuple(p.shape)}" for n, p in module.named_parameters())
            comm.check_same(desc, "parameter names/shapes")
        self.flat = flatten_module(module)
        self._build_buckets()
        self.rccl = None
        transport, self.rccl = resolve_transport(comm, module, reducer, transport)
        if self.rccl is not None:
            comm.attach_native(self.rccl)          # per-step ncclCommGetAsyncError check
            comm.in_step_c10d_forbidden = True     # SyncBN may never fall back to c10d now
        if comm is not None:
            self._sync_module_states()
        self._sync_enabled = True
        self._callback_queued = False
        self._marked = [False] * len(self.flat.params)
        self._marks, self._last_marks, self._next = [], [], 0   # python reducer state
        self._hooks = []
        self.reducer_kind = reducer if comm is not None else None
        self.compress = compress
        self.transport = transport if comm is not None else None
        self.timeline = (os.environ.get("PMD_REDUCER_TIMELINE", "0") == "1") if timeline is None \
            else bool(timeline)
        self._native = None
        self._rebuild_pending = bool(rebuild_buckets) and comm is not None
        self.rebuilt_order = None
        if comm is not None and reducer == "native":
            from ..ops.native import C
            pg = None
            if self.rccl is None:
                pg = comm.group if comm.group is not None else dist.group.WORLD
            bounds, pbucket = self._bounds()
            self._native = C.Reducer(pg, self.rccl, self.flat.grad_arena, bounds, pbucket,
                                     comm.supports_avg, compress == "bf16", _flush_wgrads,
                                     self.timeline)
        elif comm is not None and compress != "none":
            raise ValueError("compress requires the native reducer")
        if comm is not None:
            self._install_hooks()
        self.iteration = 0

    # ------------------------------------------------------------ buckets
    def _build_buckets(self):
        """Contiguous arena slices in arena (= expected gradient-ready) order: a
        small first bucket so the first all-reduce starts early, ``bucket_mb``
        after that, and a small LAST bucket.  The last-ready parameters (stem and
        first stage) only get their gradients at the very end of backward, so
        their all-reduce cannot overlap anything; capping that tail bounds the
        exposed collective (at W=8 a ring all-reduce moves 2(W-1)/W of the bucket
        over each xGMI link: 2 MiB fp32 -> 3.7 MB at ~150 GB/s ~ 25 us + launch
        latency, vs ~9 MB / 60 us for the uncapped R50 tail)."""
        fp = self.flat
        n = len(fp.params)
        nb = [p.numel() * p.element_size() for p in fp.params]
        tail_start = n
        if self.last_bucket_mb and n > 1:
            cap, acc = int(self.last_bucket_mb * 2 ** 20), 0
            while tail_start > 1 and acc + nb[tail_start - 1] <= cap:
                tail_start -= 1
                acc += nb[tail_start]
            if tail_start == n:          # the last parameter alone exceeds the cap
                tail_start = n - 1
        groups, cur, nbytes = [], [], 0
        cap = int(self.first_bucket_mb * 2 ** 20)
        for i in range(tail_start):
            cur.append(i)
            nbytes += nb[i]
            if nbytes >= cap:
                groups.append(cur)
                cur, nbytes = [], 0
                cap = int(self.bucket_mb * 2 ** 20)
        if cur:
            groups.append(cur)
        if tail_start < n:
            groups.append(list(range(tail_start, n)))
        # bucket = contiguous arena slice from its first param to the next bucket's start
        starts = [fp.offsets[g[0]] for g in groups] + [fp.numel]
        self.buckets = [_Bucket(j, starts[j], starts[j + 1], g) for j, g in enumerate(groups)]
        self._param_bucket = [None] * len(fp.params)
        for b in self.buckets:
            for i in b.params:
                self._param_bucket[i] = b

    def _bounds(self):
        bounds = [b.start for b in self.buckets] + [self.flat.numel]
        pbucket = [self._param_bucket[i].index for i in range(len(self.flat.params))]
        return bounds, pbucket

    def bucket_sizes_mb(self):
        return [(b.end - b.start) * 4 / 2 ** 20 for b in self.buckets]

    def _direct_only(self):
        return self.post_hooks == "auto" and getattr(self.module, "impl", None) == "fused"

    def close(self):
        """Release the native reducer (which holds the process group) and the gradient hooks
        now, before the process group is destroyed: the hooks' closures keep this object in
        a reference cycle, which Python may otherwise collect only at interpreter exit --
        destroying a gloo process group there, after the rest of the runtime, could abort the
        process.  The wrapped module keeps its parameters and gradients."""
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self._native = None

    def _install_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        direct_only = self._direct_only()
        for i, p in enumerate(self.flat.params):
            h = self._make_native_hook(i) if self._native is not None else self._make_hook(i)
            # AccumulateGrad path (params whose grad is returned to autograd) ...
            if not direct_only:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._post_hook(h)))
            # ... and the direct path (fused ops that wrote into the arena call this)
            p._pmd_ready = h

    @staticmethod
    def _post_hook(h):
        # autograd fires post-accumulate hooks even for a None gradient; a param
        # whose arena gradient is still being written on a side stream is
        # claimed (ops.functional._claim) and is marked by its writer's _ready
        def post(p):
            if not getattr(p, "_pmd_claim", False):
                h(p)
        return post

    def _maybe_rebuild(self):
        """Once, before the second iteration: re-lay the arena out in the order
        gradients became ready in iteration 1 (rank 0's observation, broadcast so
        every rank builds the identical layout) and rebuild the buckets."""
        self._rebuild_pending = False
        if self._native is not None:
            seen = list(self._native.last_mark_order())
        else:
            seen = list(self._last_marks)
        n = len(self.flat.params)
        order = seen + [i for i in range(n) if i not in set(seen)]   # unused params last
        t = torch.tensor(order, dtype=torch.int64,
                         device=self.flat.device if self.comm.backend == "nccl" else "cpu")
        self.comm.broadcast_(t, 0)
        order = [int(v) for v in t.tolist()]
        self.rebuilt_order = [self.flat.names[i] for i in order]
        if order == list(range(n)):
            return
        self.flat.relayout(order)
        self._build_buckets()
        if self._native is not None:
            self._native.rebuild(*self._bounds())
        self._marked = [False] * n
        self._install_hooks()

    # --------------------------------------------------------- state sync
    @torch.no_grad()
    def _sync_module_states(self):
        if self.rccl is not None:
            self.rccl.broadcast_(self.flat.param_arena, 0)
        else:
            self.comm.broadcast_(self.flat.param_arena, 0)
        self._broadcast_buffers()

    @torch.no_grad()
    def _broadcast_buffers(self):
        by_dtype = {}
        for b in self.module.buffers():
            by_dtype.setdefault(b.dtype, []).append(b)
        for bufs in by_dtype.values():
            flat = torch.cat([b.reshape(-1) for b in bufs])
            # in-step: on the gradient transport's own communicator (the native one never
            # shares the step with a c10d collective, Comm.in_step_c10d_forbidden)
            if self.rccl is not None:
                self.rccl.broadcast_(flat, 0)
            else:
                self.comm.broadcast_(flat, 0)
            off = 0
            for b in bufs:
                n = b.numel()
                b.copy_(flat[off: off + n].view_as(b))
                off += n

    # --------------------------------------------------------------- hooks
    def _make_hook(self, i):
        # Called by the AccumulateGrad post-hook and/or by fused ops that wrote the
        # gradient into the arena directly (autograd may still run the post-hook
        # for those with an undefined grad) -> idempotent per iteration.
        def hook(_p):
            if not self._sync_enabled or self._marked[i]:
                return
            self._marked[i] = True
            self._marks.append(i)
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            b = self._param_bucket[i]
            b.pending -= 1
            while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
                self._launch(self.buckets[self._next])
                self._next += 1
        return hook

    def _make_native_hook(self, i):
        mark = self._native.mark

        def hook(_p):
            mark(i)
        return hook

    def _launch(self, b):
        if b.work is not None:
            raise RuntimeError(f"bucket {b.index} launched twice in one iteration")
        b.fired += 1
        b.work = self.comm.all_reduce_mean_async(self.flat.grad_arena[b.start: b.end])

    def _finalize(self):
        _flush_wgrads()          # deferred side-stream weight grads are marked first
        # params that received no gradient this iteration (unused): launch their bucket anyway
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        for b in self.buckets:
            b.work.wait()
        if self.check_collectives:
            bad = [b.index for b in self.buckets if b.fired != 1]
            if bad:
                raise RuntimeError(f"buckets {bad} fired != 1 times this iteration")
        for b in self.buckets:
            b.work = None
            b.fired = 0
            b.pending = len(b.params)
        self._marked = [False] * len(self.flat.params)
        self._last_marks = self._marks
        self._marks = []
        self._next = 0
        self._callback_queued = False
        self.iteration += 1

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync_enabled
        self._set_sync(False)
        try:
            yield
        finally:
            self._set_sync(old)

    def _set_sync(self, on):
        self._sync_enabled = on
        if self._native is not None:
            self._native.set_enabled(on)

    def collective_signature(self):
        """Bucket launch order of the last iteration (for Comm.verify_order)."""
        if self._native is not None:
            return self._native.last_launch_order()
        return []

    def bucket_timeline(self):
        """Last iteration: [(bucket, host launch us after first mark, host finalize us,
        device start ms, device end ms)], device times relative to the end of the
        backward's compute work (negative = overlapped), NaN where unavailable."""
        if self._native is None:
            return []
        return [tuple(r) for r in self._native.timeline()]

    @property
    def num_iterations(self):
        return self._native.iteration if self._native is not None else self.iteration

    # ------------------------------------------------------------- forward
    def forward(self, *args, **kwargs):
        if self.comm is not None and torch.is_grad_enabled():
            # like DDP: buckets are rebuilt after the first iteration that produced
            # gradients, whatever the BN mode of the module
            if self._rebuild_pending and self.num_iterations >= 1:
                self._maybe_rebuild()
            if self.broadcast_buffers and self.module.training:
                self._broadcast_buffers()
        return self.module(*args, **kwargs)

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def shutdown(self):
        """Abort the native communicator (peers blocked in a collective error out)."""
        if self.rccl is not None:
            self.rccl.abort()
            if self.comm is not None:
                self.comm.in_step_c10d_forbidden = False
