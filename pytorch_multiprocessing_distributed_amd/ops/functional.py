"""Fused, autograd-aware ResNet ops over NHWC activations.

Every op is a ``torch.autograd.Function`` whose forward/backward are written
in terms of *primitives* (:mod:`.torch_prims` on CPU, :mod:`.hip_prims` =
hand-written gfx950 kernels on an MI355X).  The graph is what the reference
gets from ``nn.Conv2d`` + ``nn.SyncBatchNorm`` + ``F.relu`` + the in-place
residual add (reference model/resnet.py:35-39, 65-70; main.py:43), re-cut so
memory-bound work is fused and every residual block is ONE autograd node:

forward, per conv->BN(->ReLU) stage
  conv        implicit-GEMM conv; its epilogue also accumulates per-channel
              (sum, sum^2) BN statistics
  stats       SyncBN: one all-reduce of [sum | sum^2 | count] per BN site (the
              two BNs of a projection block share one); single replica: a
              single collapse+finalize kernel
  apply       one elementwise pass: normalise, add the (BN'd) shortcut, ReLU
backward, per stage
  reduce      one pass: sum(dz*mask), sum(dz*mask*xhat) -> [all-reduce] ->
              gamma/beta grads written straight into the reducer's arena
  elemt       one pass -> dy
  dgrad       implicit-GEMM; the block's input gradient from the residual /
              projection path is added in the epilogue (no separate add pass)
  wgrad       split-K MFMA kernel accumulating straight into the arena view
              of ``weight.grad``

Gradients of parameters that live in the flat arena (:mod:`..parallel.flat`)
are written in place and the data-parallel reducer is notified directly
(``param._pmd_ready``), so AccumulateGrad never runs for them.

SyncBN semantics follow torch.nn.SyncBatchNorm (torch:nn/modules/
_functions.py:39-207): global statistics in forward, globally reduced
``sum_dy``/``sum_dy_xmu`` in backward, *local* gamma/beta gradients (the
reducer averages them).  Unlike torch there is no device->host sync (B13).
"""
from __future__ import annotations

import os
import weakref

import torch

from . import torch_prims

_NAN_CHECK = os.environ.get("PMD_NAN_CHECK", "0") == "1"   # debug: finite-check block backward

_state = {"bn_sync": None, "force_torch": os.environ.get("PMD_PRIMS", "") == "torch",
          # fuse each BN-backward reduce into the dgrad epilogue that produces its input
          "fuse_bnred": os.environ.get("PMD_FUSE_BNRED", "1") != "0",
          "fused_site_hits": 0,
          "fused_site_misses": 0,
          "fused_stem": os.environ.get("PMD_FUSED_STEM", "1") != "0",
          "fp8": None,          # Fp8Scaling when the block convs run in fp8 (config 5)
          "wimg": None,         # WeightImageSet of the running forward (grouped weight prep)
          "det": os.environ.get("PMD_DET_STATS", "0") == "1"}   # set_deterministic


def set_deterministic(flag: bool):
    """Deterministic BN-statistics mode (test / debug; kernels/det.hip): every statistics
    producer adds into private per-row-block slots that are folded in a fixed order, the loss
    sum likewise, and the linear-BN backward (LDS atomics) is off, so two identical steps --
    or one step with its stream hand-offs on different event mechanisms, or a HIP-graph replay
    and the eager step it captured -- give bit-identical gradients, parameters and statistics.
    Slower (one extra fold launch per statistics producer); never on in production.
    ``PMD_DET_STATS=1`` turns it on at import."""
    _state["det"] = bool(flag)
    from .native import C
    C.det_stats_set(bool(flag))


def deterministic() -> bool:
    return _state.get("det", False)


def set_bn_sync(comm):
    """Install the communicator used for SyncBN statistics (None = local BN)."""
    _state["bn_sync"] = comm


def get_bn_sync():
    return _state["bn_sync"]


class WeightImageSet:
    """bf16 weight images of every conv of a model, refreshed by ONE grouped
    kernel per forward (native ``_C.WeightImages``) instead of one prep launch
    per conv.  ``entries``: [(conv module, padded input channels, want dgrad image)]."""

    def __init__(self, entries):
        from .native import C
        self.entries = list(entries)
        self.index = {(id(m.weight), cp, wt): i for i, (m, cp, wt) in enumerate(self.entries)}
        self._dev = self.entries[0][0].weight.device
        self._c = C.WeightImages([m.weight for m, _, _ in self.entries],
                                 [cp for _, cp, _ in self.entries], [wt for _, _, wt in self.entries])

    def refresh(self, need_bwd=True):
        """Forward images (and, when a backward follows, the dgrad images) in ONE launch on the
        current stream.  (The dgrad images on the idle side stream during the forward measured
        step-neutral, 12,699 / 12,684 vs 12,704 / 12,712 img/s in round 4.)"""
        self._c.refresh(3 if need_bwd else 1)
        if self.fp8 is not None:
            self.fp8.refresh()

    fp8 = None   # Fp8WeightSet of the same model when fp8 (config 5) is active

    def lookup(self, w, cin, want_t):
        i = self.index.get((id(w), cin, want_t))
        if i is None and not want_t:
            i = self.index.get((id(w), cin, True))   # a superset of what was asked
        return None if i is None else tuple(self._c.get(i))


class Fp8WeightSet:
    """e4m3 images of the block convs' weights, quantised with their delayed-
    scaling sites by ONE grouped launch per step (native ``_C.Fp8WeightImages``)
    instead of one ``quant_weight_fp8`` launch per conv.  ``entries``:
    [(conv module, input channels)]."""

    def __init__(self, entries, f8):
        from .native import C
        self.f8 = f8
        self.index = {id(m): i for i, (m, _) in enumerate(entries)}
        sites = [f8.site(("w", id(m)), init_from=m.weight) for m, _ in entries]
        # + the transposed [Cp][R][S][K] images of the fp8 dgrads (same scale sites)
        self._c = C.Fp8WeightImages([m.weight for m, _ in entries], [cp for _, cp in entries],
                                    [sc for sc, _ in sites], [am for _, am in sites],
                                    [FP8_DGRAD] * len(entries))

    def refresh(self):
        self._c.refresh()

    def lookup(self, conv_m, cin):
        i = self.index.get(id(conv_m))
        return None if i is None else self._c.get(i)

    def lookup_t(self, conv_m):
        """The fp8 dgrad's e4m3 [Cp][R][S][K] image (None: not kept for this conv)."""
        i = self.index.get(id(conv_m))
        return None if i is None else self._c.get_t(i)


def _weight_images(P, w, dtype, cin, want_t):
    wi = _state["wimg"]
    if wi is not None:
        r = wi.lookup(w, cin, want_t)
        if r is not None:
            return r
    return P.conv_weight(w, dtype, cin, want_t)


def _conv_weight(P, conv_m, dtype, cin, want_t):
    return _weight_images(P, conv_m.weight, dtype, cin, want_t)


class weight_images:
    """Context manager: install ``wset`` (refreshed) for the duration of a forward."""

    def __init__(self, wset):
        self.wset = wset

    def __enter__(self):
        if self.wset is not None:
            self.wset.refresh(need_bwd=torch.is_grad_enabled())
        self.prev = _state["wimg"]
        _state["wimg"] = self.wset
        return self.wset

    def __exit__(self, *exc):
        _state["wimg"] = self.prev
        return False


def set_fp8(scaling):
    """Install an :class:`ops.fp8.Fp8Scaling` (block convolutions' forward in fp8
    on the gfx950 path) or ``None`` for bf16."""
    _state["fp8"] = scaling


def get_fp8():
    return _state["fp8"]


def _fp8_for(P):
    f = _state["fp8"]
    return f if (f is not None and getattr(P, "SUPPORTS_FP8", False)) else None


# Which convs run their forward in fp8 (the BN-apply feeding a bf16 conv skips its
# e4m3 copy).  The fp8 gain of a conv has to pay for that copy (1 B per input element):
#   PMD_FP8_CONVS=spatial (default with PMD_FP8_WGRAD=0): the R x S > 1 convs (3x3), which run 1.2-1.4x
#     faster in fp8 (790-1,144 vs 600-856 TFLOP/s) and read a 64-512-channel input;
#     the 1x1 convs save less than their e4m3 input copy costs (conv_bench per-layer
#     table in profiles/fp8_ring_depth_r02_rejected.txt);
#   PMD_FP8_CONVS=all (default): every block conv whose reduction Kg = R*S*Cin >= PMD_FP8_MIN_KG
#     (default 0 = every block conv with the fp8 gradients, else 128 = a full e4m3 K-tile).
# fp8 weight gradients (e5m2 dY x e4m3 X) for every conv whose forward ran in fp8; the
# bf16 copy of a stage activation is then not written at all (PMD_FP8_WGRAD=0: bf16 wgrads)
FP8_WGRAD = os.environ.get("PMD_FP8_WGRAD", "1") != "0"
# With fp8 weight gradients the e4m3 input copy also halves the wgrad's activation bytes and
# runs it at the fp8 MFMA rate, so every eligible block conv pays ("all": 13,217 / 13,193 vs
# "spatial" 12,961 / 13,007 vs bf16 12,578 / 12,609 img/s, one lease, round 3); without them
# only the 3x3 convs do (round 2: profiles/fp8_policy_ab_r02.txt).
FP8_CONVS = os.environ.get("PMD_FP8_CONVS", "all" if FP8_WGRAD else "spatial")
# fp8 data gradients (e5m2 dY x e4m3 transposed weight image, the bf16 dgrad's fused
# epilogue) for the same convs (PMD_FP8_DGRAD=0: bf16 dgrads); needs the fp8 wgrads' dY copy
FP8_DGRAD = FP8_WGRAD and os.environ.get("PMD_FP8_DGRAD", "1") != "0"
# Minimum forward reduction R*S*Cin of an fp8 conv.  A 64-deep reduction half-fills the
# 128-deep e4m3 K-tile, but with fp8 data AND weight gradients the l1 convs still pay
# through their e5m2-only dY and e4m3-only activations: 0 = every block conv (13,976 /
# 13,998 vs 13,791 / 13,784 img/s at 128, same lease); 128 without the fp8 gradients.
FP8_MIN_KG = int(os.environ.get("PMD_FP8_MIN_KG", "0" if FP8_DGRAD else "128"))


def fp8_eligible(conv_m, cin) -> bool:
    rs = conv_m.weight.shape[2] * conv_m.weight.shape[3]
    if FP8_CONVS == "spatial" and rs == 1:
        return False
    return int(cin) * rs >= FP8_MIN_KG


def _conv_fwd_any(P, f8, h, hq, wp, conv_m, want_stats):
    """bf16 conv, or the fp8 one when ``hq = (e4m3 input, scale)`` is given."""
    if f8 is None or hq is None:
        return P.conv_fwd(h, wp, conv_m.stride, conv_m.padding, want_stats)
    sw, aw = f8.site(("w", id(conv_m)), init_from=conv_m.weight)
    wi = _state["wimg"]
    wq = wi.fp8.lookup(conv_m, h.shape[-1]) if (wi is not None and wi.fp8 is not None
                                                 and wi.fp8.f8 is f8) else None
    if wq is None or wq.shape[-1] != h.shape[-1]:
        wq = P.quant_weight_fp8(conv_m.weight, h.shape[-1], sw, aw)
    return P.conv_fp8_fwd(hq[0], wq, hq[1], sw, conv_m.stride, conv_m.padding, want_stats)


def set_fuse_bn_reduce(flag: bool):
    """Fuse BN-backward reduces into the producing dgrad epilogues (default on)."""
    _state["fuse_bnred"] = bool(flag)


def force_torch_prims(flag: bool):
    _state["force_torch"] = bool(flag)


def prims_for(t):
    if t.is_cuda and not _state["force_torch"]:
        from . import hip_prims
        return hip_prims
    return torch_prims


_EMPTY = {}


def _empty(dev):
    e = _EMPTY.get(dev)
    if e is None:
        e = _EMPTY[dev] = torch.empty(0, device=dev)
    return e


# ------------------------------------------------------------- grad routing
def _grad_target(p):
    """Arena view to accumulate ``p``'s gradient into directly, or None."""
    if p is not None and p.requires_grad and getattr(p, "_pmd_direct", False) and p.grad is not None:
        return p.grad
    return None


def _ready(*ps):
    """Tell the gradient reducer these parameters' arena gradients are final
    (on the current stream).  Clears a pending-writer claim (:func:`_claim`)."""
    for p in ps:
        if getattr(p, "_pmd_claim", False):
            p._pmd_claim = False
        h = getattr(p, "_pmd_ready", None)
        if h is not None:
            h(p)


def _claim(p):
    """A writer on ANOTHER stream owns ``p``'s arena gradient until it calls
    :func:`_ready`.  autograd runs a parameter's post-accumulate-grad hook even
    when the node returned None for it (no gradient to accumulate), i.e. right
    when the block backward returns -- before a deferred side-stream wgrad has
    been joined.  The reducer's post-hook skips claimed parameters, so a bucket
    can never be all-reduced while a side-stream kernel still writes into it."""
    p._pmd_claim = True


def _conv_wgrad_any(P, dy, x, xq, wk_shape, stride, pad, out=None):
    """bf16 weight gradient, or the fp8 one (e5m2 dY x e4m3 X) when the conv input's
    e4m3 copy ``xq = (q, scale)`` was saved and dY carries its e5m2 copy."""
    dq = getattr(dy, "_pmd_q8", None)
    if xq is not None and dq is not None:
        return P.conv_wgrad_fp8(dq[0], dq[1], xq[0], xq[1], wk_shape, stride, pad, out=out)
    if x.dtype == torch.uint8:
        raise RuntimeError("fp8-only activation (no bf16 copy) but dY has no e5m2 copy: "
                           "the fp8 weight gradient must run for this conv")
    return P.conv_wgrad(dy, x, wk_shape, stride, pad, out=out)


def _wgrad(P, dy, x, wpack, stride, pad, w, xq=None):
    """Weight gradient: accumulated into the arena (returns None) or returned."""
    if not w.requires_grad:
        return None
    cx = wpack[0].shape[-1]
    tgt = _grad_target(w)
    if tgt is not None and cx == w.shape[1]:
        _conv_wgrad_any(P, dy, x, xq, tuple(wpack[0].shape), stride, pad, out=tgt.permute(0, 2, 3, 1))
        _ready(w)
        return None
    dwk = _conv_wgrad_any(P, dy, x, xq, tuple(wpack[0].shape), stride, pad)   # fp32 [K,R,S,Cx]
    if cx != w.shape[1]:
        dwk = dwk[..., : w.shape[1]].contiguous()
    return dwk.permute(0, 3, 1, 2)                                   # [K,C,R,S] channels_last


# PMD_SIDE_SHORTCUT=0: the projection-shortcut convs of the forward stay on the main stream
_SIDE_SHORTCUT = os.environ.get("PMD_SIDE_SHORTCUT", "1") != "0"

# the split-K reductions of one block's side-stream weight gradients as ONE grouped launch
# (kernels/conv_wgrad.hip wgrad_flush) instead of one per weight gradient; PMD_WS_GROUP=0: per wgrad
_WS_GROUP = os.environ.get("PMD_WS_GROUP", "1") != "0"
_WGRAD_STREAM = {"on": os.environ.get("PMD_WGRAD_STREAM", "1") != "0", "streams": {},
                 "defer": int(os.environ.get("PMD_WGRAD_DEFER", "1") or 0)}  # join lag in blocks


# Priority of the step's own HIP streams (default high, -1; PMD_STREAM_PRIO=0: normal).
# HIP keeps one pool of hardware queues per priority (GPU_MAX_HW_QUEUES each) and hands a
# new stream the least shared queue of its pool; RCCL / c10d create several long-lived streams of their own in
# the normal pool, so a normal-priority side stream can land on the SAME hardware queue as
# the main stream and lose all its overlap (bench/queue_map.py, profiles/queues_r04.txt).
# With the step's streams (main, weight gradients, SyncBN exchange, gradient buckets) all in
# the high-priority pool they get one queue each (see docs/ARCHITECTURE.md, "Streams ->
# hardware queues").
STREAM_PRIO = 0 if os.environ.get("PMD_STREAM_PRIO", "1") == "0" else -1


# Cross-stream fork / join points between the main and the weight-gradient stream (~60 per
# ResNet-50 step).  torch.cuda.Event records a marker with a SYSTEM-scope release, which the
# main stream pays between its two kernels (6.1 us per fork, bench/event_fence.py);
# PMD_FORK_EVENTS=0/1/2 uses the native event ring (csrc/runtime/events.cpp) with the default /
# no system fence (default: 3.5 us per fork, +0.35% on the ResNet-50 step,
# profiles/fork_events_r05.txt) / a device-scope release instead -- both streams are on one
# device, where the producing kernel's own release covers the consumer.  -1: torch events.
# Host- and peer-visible sync points keep torch's events.
_FORK_EV = int(os.environ.get("PMD_FORK_EVENTS", "1") or 1)
_RINGS: dict = {}


def _fork_ring(dev):
    if _FORK_EV < 0 or torch.cuda.is_current_stream_capturing():
        return None
    r = _RINGS.get(dev)
    if r is None:
        from .native import C
        r = _RINGS[dev] = C.StreamEvents(1024, _FORK_EV, dev.index)
    return r


def _stream_wait(waiter, producer):
    """``waiter`` waits for everything issued so far on ``producer`` (same device)."""
    ring = _fork_ring(producer.device)
    if ring is None:
        waiter.wait_stream(producer)
    else:
        ring.fork(producer.cuda_stream, waiter.cuda_stream)


# test hook (negative controls of the hand-off tests): the fork whose running count reaches 0 is
# SKIPPED -- the side stream then runs without waiting for the main stream's producer
_DROP_FORK = [-1]


def _fork(side, main):
    """The side stream forks from the main stream: it waits for everything issued on main."""
    if _DROP_FORK[0] >= 0:
        _DROP_FORK[0] -= 1
        if _DROP_FORK[0] < 0:
            return
    _stream_wait(side, main)


class _RingEvent:
    __slots__ = ("ring", "slot")

    def __init__(self, ring, stream):
        self.ring = ring
        self.slot = ring.record(stream.cuda_stream)


def _record_on(stream):
    """An event recorded on ``stream`` now (a ring slot, or a torch event)."""
    ring = _fork_ring(stream.device)
    if ring is None:
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev
    return _RingEvent(ring, stream)


def _wait_on(stream, ev):
    if isinstance(ev, _RingEvent):
        ev.ring.wait(stream.cuda_stream, ev.slot)
    else:
        stream.wait_event(ev)


def _wgrad_stream(dev):
    st = _WGRAD_STREAM["streams"].get(dev)
    if st is None:
        st = _WGRAD_STREAM["streams"][dev] = torch.cuda.Stream(device=dev, priority=STREAM_PRIO)
    return st


_STEP_STREAMS: dict = {}


def _new_stream(dev, prio=None, cu_mask=None):
    # a NEW HIP stream: torch.cuda.Stream(priority=...) hands out streams of torch's fixed
    # per-priority pool (32 streams created together and spread round-robin over the hardware
    # queues, shared with whatever else -- gloo, c10d -- draws from the pool), so two of the
    # step's streams could land on one queue depending on the pool cursor
    from .native import C
    return torch.cuda.ExternalStream(C.create_stream(dev.index, STREAM_PRIO if prio is None else prio,
                                                     list(cu_mask or [])), device=dev)


def init_step_streams(dev):
    """Create the rank's step streams -- main (made current), weight gradients, gradient
    collectives (RcclComm) -- as new HIP streams at STREAM_PRIO, in that order, BEFORE any
    communicator or torch stream pool exists: HIP hands a new stream the least-used hardware
    queue of its priority pool, so the three take three different queues whatever is created
    later (profiles/queues_r04.txt).  Idempotent per device.  Returns the main stream."""
    if dev in _STEP_STREAMS:
        torch.cuda.set_stream(_STEP_STREAMS[dev]["main"])
        return _STEP_STREAMS[dev]["main"]
    main = _new_stream(dev)
    main.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.set_stream(main)
    side = _new_stream(dev)
    _WGRAD_STREAM["streams"][dev] = side
    comm = _new_stream(dev)
    _STEP_STREAMS[dev] = {"main": main, "wgrad": side, "comm": comm}
    return main


def comm_stream_handle(dev=None) -> int:
    """HIP handle of the pre-created gradient-collective stream of ``dev`` (default: the
    current device; 0: none was created)."""
    if not _STEP_STREAMS:
        return 0
    if dev is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    e = _STEP_STREAMS.get(torch.device(dev) if not isinstance(dev, torch.device) else dev)
    return int(e["comm"].cuda_stream) if e else 0


def set_wgrad_stream(flag: bool):
    """Run the block weight gradients on a side HIP stream (default on)."""
    _WGRAD_STREAM["on"] = bool(flag)


class _WgradSide:
    """Weight gradients of one block backward on a side HIP stream.

    A wgrad only needs dY and the saved conv input, and nothing in the block
    backward consumes its result, so it can run concurrently with the main
    stream's BN-backward elementwise pass and the next dgrad (memory- / epilogue-
    bound work next to the MFMA-heavy wgrad).  The side stream forks from the
    main stream before each wgrad (dY is final), and the main stream joins it
    once at the end of the block backward; only THEN are the weights marked
    ready for the gradient all-reduce, so a bucket never launches on a
    gradient still being written.  ``record_stream`` keeps dY / X alive for
    the side stream in the caching allocator."""

    def __init__(self, t):
        self.on = _WGRAD_STREAM["on"] and t.is_cuda and not _state["force_torch"]
        self.ready = []
        self.deferred = False
        if self.on:
            from .native import C
            self.C = C
            dev = t.device
            self.side = _wgrad_stream(dev)
            self.main = torch.cuda.current_stream(dev)

    def wgrad(self, P, dy, x, wpack, stride, pad, w, xq=None):
        if not self.on or _grad_target(w) is None:
            return _wgrad(P, dy, x, wpack, stride, pad, w, xq)
        _claim(w)
        # one fork per weight gradient, issued as soon as dY is final: batching two behind one
        # fork saves a marker but delays the first, -0.5% / -1.1% for 2 / 3 (fork_events_r05)
        _fork(self.side, self.main)
        with torch.cuda.stream(self.side):
            tgt = _grad_target(w)
            if _WS_GROUP:
                # split-K reductions queued; join() launches them as ONE grouped kernel
                self.C.wgrad_set_defer(True)
                self.deferred = True
            try:
                _conv_wgrad_any(P, dy, x, xq, tuple(wpack[0].shape), stride, pad, out=tgt.permute(0, 2, 3, 1))
            finally:
                if _WS_GROUP:
                    self.C.wgrad_set_defer(False)
        dy.record_stream(self.side)
        x.record_stream(self.side)
        dq = getattr(dy, "_pmd_q8", None)
        if dq is not None:
            dq[0].record_stream(self.side)
        if xq is not None:
            xq[0].record_stream(self.side)
        self.ready.append(w)
        return None

    def fork(self, fn, keep=()):
        """``fn()`` on the side stream after everything issued so far on the main stream;
        returns (its result, the event the main stream must wait on before using it; None
        when it ran here)."""
        if not self.on:
            return fn(), None
        _fork(self.side, self.main)
        with torch.cuda.stream(self.side):
            r = fn()
        for t in keep:
            if t is not None and t.is_cuda:
                t.record_stream(self.side)
        return r, _record_on(self.side)

    def run(self, w, fn, keep=()):
        """Like :meth:`wgrad` for a weight gradient computed by ``fn(target)`` (target = the
        arena view [K,R,S,C] fp32 it must ADD into); ``keep``: tensors made on the main stream
        that ``fn`` reads.  Without an arena target (or the side stream) ``fn`` runs here on a
        zeroed tensor, which is returned for autograd ([K,C,R,S] channels_last); else None."""
        tgt = _grad_target(w)
        if tgt is None:
            out = torch.zeros(w.shape[0], w.shape[2], w.shape[3], w.shape[1], dtype=torch.float32,
                              device=w.device)
            fn(out)
            return out.permute(0, 3, 1, 2)
        if not self.on:
            fn(tgt.permute(0, 2, 3, 1))
            _ready(w)
            return None
        _claim(w)
        _fork(self.side, self.main)
        with torch.cuda.stream(self.side):
            fn(tgt.permute(0, 2, 3, 1))
        for t in keep:
            if t is not None and t.is_cuda:
                t.record_stream(self.side)
        self.ready.append(w)
        return None

    def join(self):
        """End of the block backward: the join is DEFERRED by one block -- the
        main stream waits for the PREVIOUS block's side work (whose wgrads have
        overlapped this block's backward) and marks those weights ready; this
        block's side work is joined by the next block, or by the end-of-backward
        engine callback queued with the first deferral (queued before the
        reducer's own finalize callback, so every weight is ready before any
        bucket is force-launched)."""
        if not (self.on and self.ready):
            return
        if self.deferred:
            with torch.cuda.stream(self.side):
                self.C.wgrad_flush()        # the block's split reductions: one launch
            self.deferred = False
        if not _WGRAD_STREAM["defer"]:
            _stream_wait(self.main, self.side)
            for w in self.ready:
                _ready(w)
            self.ready = []
            return
        ev = _record_on(self.side)
        pend = _WGRAD_STREAM.get("pending")
        if pend is None:
            pend = _WGRAD_STREAM["pending"] = []
            torch.autograd.Variable._execution_engine.queue_callback(_wgrad_flush)
        pend.append((self.main, ev, self.ready))
        while len(pend) > _WGRAD_STREAM["defer"]:
            _join_pending(pend.pop(0))
        self.ready = []


def _join_pending(pend):
    main, ev, ws = pend
    _wait_on(main, ev)
    for w in ws:
        _ready(w)


def _wgrad_flush():
    for pend in _WGRAD_STREAM.pop("pending", None) or []:
        _join_pending(pend)


def flush_pending_wgrads():
    """Join every side-stream weight gradient still deferred and mark those
    weights ready.  The data-parallel reducer calls this at the START of its
    end-of-backward finalize (before it force-launches any bucket), so no
    bucket is ever all-reduced while its gradients are still being written and
    every deferred weight is marked inside the iteration it belongs to."""
    _wgrad_flush()


def _bn_acc(bn):
    """(d_beta, d_gamma) arena targets for a BN module, or None."""
    tb, tg = _grad_target(bn.bias), _grad_target(bn.weight)
    if tb is None or tg is None:
        return None
    return (tb, tg)


def bn_stat_shift(bn):
    """Per-BN-site statistics shift K (fp32 [C], on the BN's device): the conv
    epilogue accumulates (sum (y-K), sum (y-K)^2) and every finalize overwrites K
    with the batch mean, so the next step's sums are taken about (nearly) the
    mean and E[y^2] - E[y]^2 cannot cancel catastrophically (common.h
    bn_moments).  Starts at the running mean (0 for a fresh model).  A plain
    attribute -- not a buffer: not in state_dict, not broadcast; under SyncBN it
    stays identical on every rank because it is set from the global mean."""
    ref = bn.running_mean if bn.running_mean is not None else bn.weight
    k = getattr(bn, "_pmd_shift", None)
    if k is None or k.device != ref.device or k.numel() != ref.numel():
        k = (bn.running_mean.detach().float().clone() if bn.running_mean is not None
             else torch.zeros(ref.numel(), dtype=torch.float32, device=ref.device))
        bn._pmd_shift = k
    return k


_BN_SHIFT = os.environ.get("PMD_BN_SHIFT", "1") != "0"
# Linear-BN backward for a block's final BN (PMD_BNLIN: "auto" = the large 1x1 stride-1 conv3
# outputs of the l1 / l2 stages, "all" = every eligible identity block, "0" = off): the BN
# backward is folded through the 1x1 conv that produced its input (y = z W^T), so neither the
# BN-backward elementwise pass nor the producer's statistics epilogue ever reads y, and dy is
# never materialised -- see _bnlin_final.
_BNLIN = os.environ.get("PMD_BNLIN", "auto")
_BNLIN_MIN = int(os.environ.get("PMD_BNLIN_MIN", str(200704 * 512)))   # M * K of the BN input


def _bnlin_eligible(conv_m, yf, x, training, fuse, shortcut, f8):
    if (_BNLIN == "0" or not (training and fuse) or shortcut is not None or f8 is not None
            or _state.get("det")):   # its reductions are LDS-atomic (not in the deterministic mode)
        return False
    ks = conv_m.kernel_size if isinstance(conv_m.kernel_size, tuple) else (conv_m.kernel_size,) * 2
    st = conv_m.stride if isinstance(conv_m.stride, tuple) else (conv_m.stride,) * 2
    if ks != (1, 1) or st != (1, 1):
        return False
    return _BNLIN == "all" or yf.numel() >= _BNLIN_MIN


# a BN site whose reduce a dgrad epilogue fused receives dz already gated by its ReLU mask:
# the elementwise pass and the identity-path addend skip re-reading the mask (PMD_PREMASKED=0: re-read)
_PREMASKED = os.environ.get("PMD_PREMASKED", "1") != "0"


def _shift_of(bn):
    return bn_stat_shift(bn) if (_BN_SHIFT and bn is not None) else None


def _stats_req(bn, training):
    """``want_stats`` for the conv feeding ``bn``: its statistics shift (True when
    shifting is off, PMD_BN_SHIFT=0), or False."""
    if not training:
        return False
    k = _shift_of(bn)
    return True if k is None else k


class _Pre(list):
    """BN-backward reduce slot buffers produced by a fused dgrad epilogue, plus
    the HIP event recorded right after that dgrad (None on CPU)."""
    __slots__ = ("event",)

    def __init__(self, bufs, event=None):
        super().__init__(bufs)
        self.event = event


def _after_dgrad_event(t, sync):
    if sync is None or not t.is_cuda or not getattr(sync, "overlap_bn_bwd", False) \
            or getattr(sync, "xgmi", None) is None:
        return None
    return _record_on(torch.cuda.current_stream(t.device))


# ---------------------------------------------------------------- BN pieces
_UNSET = object()
# stats object returned by the public conv() -> the shift its sums were taken about
_SHIFT_USED: dict = {}


def _pop_shift(st):
    e = _SHIFT_USED.pop(id(st), None) if st is not None else None
    return e[1] if (e is not None and e[0]() is st) else _UNSET


def _bn_forward_params(P, y, st, bn, training, sync, y2=None, st2=None, bn2=None,
                       k1=_UNSET, k2=_UNSET):
    """-> (p1, p2, count); count is a host float (local) or device scalar (SyncBN).
    ``k1``/``k2``: the shift the statistics were accumulated about (default: the
    BN's own -- what every fused path requests from its producing conv)."""
    if not training:
        p1 = P.bn_eval_params(bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.eps)
        p2 = None
        if bn2 is not None:
            p2 = P.bn_eval_params(bn2.running_mean, bn2.running_var, bn2.weight, bn2.bias, bn2.eps)
        return p1, p2, None
    c1 = y.shape[-1]
    m_local = y.numel() // c1
    k1 = _shift_of(bn) if k1 is _UNSET else k1
    k2 = _shift_of(bn2) if k2 is _UNSET else k2
    if sync is None:
        p1 = P.stats_finalize_local(st, float(m_local), bn.weight, bn.bias, bn.eps,
                                    bn.running_mean, bn.running_var, bn.momentum,
                                    bn.num_batches_tracked, k1)
        p2 = None
        if bn2 is not None:
            p2 = P.stats_finalize_local(st2, float(m_local), bn2.weight, bn2.bias, bn2.eps,
                                        bn2.running_mean, bn2.running_var, bn2.momentum,
                                        bn2.num_batches_tracked, k2)
        return p1, p2, float(m_local)
    fused = getattr(sync, "fused_bn_ok", None)
    if fused is not None and fused(st) and hasattr(P, "_release"):
        # collapse + one-shot xGMI exchange + finalize in ONE kernel
        dev = y.device
        p1 = torch.empty(4, c1, dtype=torch.float32, device=dev)
        p2 = torch.empty(4, y2.shape[-1], dtype=torch.float32, device=dev) if bn2 is not None else None
        count = torch.empty(1, dtype=torch.float32, device=dev)
        sync.bn_stats_fwd(st, st2, float(m_local), bn, bn2, p1, p2, count, k1, k2)
        P._release(st, st2)
        return p1, p2, count
    buf = P.stats_collapse(st, st2, float(m_local))
    sync.all_reduce_stats_(buf)
    count = buf[-1:]
    p1 = P.bn_finalize(buf[: 2 * c1].view(2, c1), count, bn.weight, bn.bias, bn.eps,
                       bn.running_mean, bn.running_var, bn.momentum, bn.num_batches_tracked, k1)
    p2 = None
    if bn2 is not None:
        c2 = y2.shape[-1]
        p2 = P.bn_finalize(buf[2 * c1: 2 * c1 + 2 * c2].view(2, c2), count, bn2.weight, bn2.bias,
                           bn2.eps, bn2.running_mean, bn2.running_var, bn2.momentum,
                           bn2.num_batches_tracked, k2)
    return p1, p2, count


def _elemt(P, dout, mask, y, p, gamma, red, count, relu, want_dzm=False, q8=None):
    if q8 is not None and not want_dzm:
        # + the e5m2 copy of dY for the fp8 weight / data gradients (dy._pmd_q8); q8[2]: it
        # is the only copy (both consumers of this dY run in fp8)
        return P.bn_bwd_elemt(dout, mask, y, p, gamma, red, count, relu, q8=q8[:2],
                              q8_only=len(q8) > 2 and q8[2])
    return P.bn_bwd_elemt(dout, mask, y, p, gamma, red, count, relu, want_dzm=want_dzm)


def _bn_backward(P, dout, mask, relu, training, sync, count, y1, p1, bn1, y2=None, p2=None,
                 bn2=None, want_dzm=False, pre=None, elemt_fn=None, q8=(None, None)):
    """BN(+second BN)(+ReLU) backward. Returns (dy1, dy2, dzm, grads) with
    grads = [d_g1, d_b1, d_g2, d_b2] for params that were NOT written directly.
    ``pre``: the reduce results already produced by the dgrad that computed
    ``dout`` (fused epilogue), in the order (bn1[, bn2]).  ``elemt_fn(red, count)``
    replaces the elementwise pass of BN 1 (fused stem: it re-derives dz itself;
    red/count are None in eval mode).  ``q8[i]``:
    (scale, amax) of an e5m2 copy of dY of BN i for an fp8 weight gradient."""
    if pre is not None:
        r1 = pre[0]
        r2 = pre[1] if y2 is not None else None
        # the dgrad that fused this reduce stored dz * mask (kernels/conv_igemm.hip epilogue):
        # dout is already gated by the ReLU mask, so the elementwise pass skips the mask bytes
        if _PREMASKED:
            relu = False
    else:
        r1 = P.bn_bwd_reduce(dout, mask, y1, p1, relu)
        r2 = P.bn_bwd_reduce(dout, mask, y2, p2, relu) if y2 is not None else None
    acc1 = _bn_acc(bn1)
    acc2 = _bn_acc(bn2) if bn2 is not None else None
    c1 = y1.shape[-1]
    fused = getattr(sync, "fused_bn_ok", None) if training else None
    if (fused is not None and fused(r1) and hasattr(P, "_release") and acc1 is not None
            and (bn2 is None or acc2 is not None)):
        # collapse (+= local gamma/beta grads) + one-shot exchange in ONE kernel
        c2 = y2.shape[-1] if y2 is not None else 0
        red = torch.empty(2 * c1 + 2 * c2, dtype=torch.float32, device=dout.device)
        ev = getattr(pre, "event", None) if pre is not None else None
        if ev is not None and getattr(sync, "overlap_bn_bwd", False):
            # the reduce slots were complete right after the dgrad that produced them
            # (event); run the exchange on the side stream from there, so it overlaps
            # the weight-gradient kernel(s) issued since, and join before bn_bwd_elemt
            # (and before the gamma/beta grads are marked ready for the reducer)
            side = sync.side_stream()
            _wait_on(side, ev)
            with torch.cuda.stream(side):
                sync.bn_stats_bwd(r1, r2, acc1, acc2, red[:2 * c1], red[2 * c1:] if c2 else None)
            _wait_on(torch.cuda.current_stream(), _record_on(side))
        else:
            sync.bn_stats_bwd(r1, r2, acc1, acc2, red[:2 * c1], red[2 * c1:] if c2 else None)
        P._release(r1, r2)
        _ready(bn1.bias, bn1.weight)
        if bn2 is not None:
            _ready(bn2.bias, bn2.weight)
        if elemt_fn is not None:
            dy1, dzm = elemt_fn(red[:2 * c1].view(2, c1), count), None
        else:
            dy1, dzm = _elemt(P, dout, mask, y1, p1, bn1.weight, red[:2 * c1].view(2, c1), count,
                              relu, want_dzm=want_dzm, q8=q8[0])
        dy2 = None
        if y2 is not None:
            dy2, _ = _elemt(P, dout, mask, y2, p2, bn2.weight, red[2 * c1:].view(2, -1), count,
                            relu, q8=q8[1])
        return dy1, dy2, dzm, [None, None, None, None]
    red = P.stats_collapse(r1, r2, None, acc1, acc2)     # local sums; gamma/beta grads += local
    grads = [None, None, None, None]
    if acc1 is None:
        grads[0], grads[1] = red[c1:2 * c1], red[:c1]
    else:
        _ready(bn1.bias, bn1.weight)
    if y2 is not None:
        c2 = y2.shape[-1]
        if acc2 is None:
            grads[2], grads[3] = red[2 * c1 + c2:], red[2 * c1:2 * c1 + c2]
        else:
            _ready(bn2.bias, bn2.weight)
    if training:
        if sync is not None:
            red = red.clone()
            sync.all_reduce_stats_(red)
        if elemt_fn is not None:
            dy1, dzm = elemt_fn(red[:2 * c1].view(2, c1), count), None
        else:
            dy1, dzm = _elemt(P, dout, mask, y1, p1, bn1.weight, red[:2 * c1].view(2, c1),
                              count, relu, want_dzm=want_dzm, q8=q8[0])
        dy2 = None
        if y2 is not None:
            dy2, _ = _elemt(P, dout, mask, y2, p2, bn2.weight, red[2 * c1:].view(2, -1), count,
                            relu, q8=q8[1])
    elif elemt_fn is not None:
        dy1, dy2, dzm = elemt_fn(None, None), None, None
    else:
        dy1, dzm = P.bn_bwd_elemt_eval(dout, mask, p1, relu, want_dzm=want_dzm)
        dy2 = P.bn_bwd_elemt_eval(dout, mask, p2, relu)[0] if y2 is not None else None
    return dy1, dy2, dzm, grads


# ---------------------------------------------------------------------- conv
class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, want_stats):
        # want_stats: False / True / the BN statistics shift tensor (bn_stat_shift)
        P = prims_for(x)
        wpack = _weight_images(P, w, x.dtype, x.shape[-1], x.requires_grad)
        y, stats = P.conv_fwd(x, wpack, stride, pad, want_stats)
        ctx.save_for_backward(x, *wpack)
        ctx.conf = (stride, pad, w)
        if stats is None:
            stats = _empty(x.device)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)   # no zeros_like(stats) fill for the unused grad
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None, None, None
        x, *wpack = ctx.saved_tensors
        stride, pad, w = ctx.conf
        P = prims_for(x)
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = P.conv_dgrad(dy, wpack, tuple(x.shape), stride, pad)
        dw = _wgrad(P, dy, x, wpack, stride, pad, w) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None, None


class _StemS2DConvFn(torch.autograd.Function):
    """ImageNet stem conv (7x7/s2/pad 3 over 3 channels, reference
    model/resnet.py:79 with the ImageNet stem) as a space-to-depth 4x4/s1 conv
    over 16 channels on the gfx950 kernels (csrc/kernels/stem.hip): 256-deep
    reduction instead of 392 (of which 62% was channel padding).  Same output,
    same BN statistics contract; the weight gradient is folded back to 7x7x3."""

    @staticmethod
    def forward(ctx, x, w, want_stats):
        from . import hip_prims as HP
        from .native import C
        xs = getattr(x, "_pmd_s2d_in", None)           # made by the data prefetch (s2d_input_prefetch)
        if xs is not None:
            x._pmd_s2d_in = None
        if xs is None or tuple(xs.shape) != (x.shape[0], x.shape[1] // 2, x.shape[2] // 2, 16):
            xs = C.stem_s2d_input(x)                   # [N, H/2, W/2, 16]
        ws = C.stem_s2d_weight(w.detach())             # [K, 4, 4, 16] bf16
        oh, ow = x.shape[1] // 2, x.shape[2] // 2
        want, shift = HP._TP.stats_request(want_stats)
        buf = HP._acquire(w.shape[0], x.device) if want else None
        out = C.conv_fwd_hw(xs, ws, 1, 2, oh, ow, want, buf, shift)
        y = out[0]
        y._pmd_s2d = True       # its gradient may arrive lazily from the fused stem tail
        stats = out[1] if want else _empty(x.device)
        ctx.save_for_backward(xs)
        ctx.w = w
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)   # no zeros_like(stats) fill for the unused grad
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        from .native import C
        (xs,) = ctx.saved_tensors
        w = ctx.w
        if dy is None or not ctx.needs_input_grad[1] or not w.requires_grad:
            return None, None, None
        lazy = getattr(dy, "_pmd_stem", None)
        dws = None
        if lazy is not None:
            # the fused stem tail handed over its backward elementwise pass (_StemPoolFn): the
            # weight gradient produces dy itself, which is never written
            from . import hip_prims as HP
            dws = HP.stem_wgrad_fused(*lazy, xs, 2)
            if dws is None:                                          # outside the fused plan
                dy = HP.stem_pool_bwd_elemt(*lazy[:7])
        if dws is None:
            dws = C.conv_wgrad(dy.contiguous(), xs, 4, 4, 1, 2, None)   # fp32 [K, 4, 4, 16]
        tgt = _grad_target(w)
        if tgt is not None:
            C.stem_s2d_wgrad_fold(dws, w.shape[1], tgt.permute(0, 2, 3, 1))
            _ready(w)
            return None, None, None
        dw = C.stem_s2d_wgrad_fold(dws, w.shape[1], None)            # [K, 7, 7, C]
        return None, dw.permute(0, 3, 1, 2), None


_S2D_STEM = os.environ.get("PMD_STEM_S2D", "1") != "0"


def set_s2d_stem(flag: bool):
    global _S2D_STEM
    _S2D_STEM = bool(flag)


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def s2d_input_prefetch(model):
    """The space-to-depth stem's input transform as a data-prefetch step (data/loader.py
    SyntheticImageNet.prefetch ``transform``), or None when ``model`` has no such stem: the
    prefetching stream lays each batch out for the 4x4 stem conv one step ahead
    (``x._pmd_s2d_in``), so the step's first main-stream kernel is the stem conv itself."""
    m = getattr(model, "module", model)
    c = getattr(m, "conv1", None)
    if (not _S2D_STEM or os.environ.get("PMD_S2D_PREFETCH", "1") == "0" or c is None or getattr(c, "weight", None) is None or tuple(c.weight.shape[2:]) != (7, 7)
            or _pair(c.stride) != (2, 2) or _pair(c.padding) != (3, 3)):
        return None

    def transform(x):
        if x.is_cuda and x.dim() == 4 and x.shape[-1] == 8 and x.shape[1] % 2 == 0 and x.shape[2] % 2 == 0:
            from .native import C
            x._pmd_s2d_in = C.stem_s2d_input(x)
        return x
    return transform


def _s2d_stem_ok(x, conv_mod):
    w = conv_mod.weight
    return (_S2D_STEM and x.is_cuda and not _state["force_torch"] and x.dim() == 4 and x.shape[-1] == 8
            and x.shape[1] % 2 == 0 and x.shape[2] % 2 == 0 and tuple(w.shape[2:]) == (7, 7)
            and w.shape[1] <= 4 and _pair(conv_mod.stride) == (2, 2) and _pair(conv_mod.padding) == (3, 3)
            and not x.requires_grad)


def conv(x, conv_mod, want_stats=None, bn=None):
    """Returns ``(y, stats)``; ``stats`` = per-channel (sum, sum^2) of y in the
    backend's layout (consumed by :func:`bn_add_act`), taken about ``bn``'s
    statistics shift when the consuming BN module is given."""
    if want_stats is None:
        want_stats = conv_mod.training
    req = _stats_req(bn, True) if (bn is not None and want_stats) else bool(want_stats)
    if _s2d_stem_ok(x, conv_mod):
        y, st = _StemS2DConvFn.apply(x, conv_mod.weight, req)
    else:
        y, st = _ConvFn.apply(x, conv_mod.weight, conv_mod.stride, conv_mod.padding, req)
    # the shift the sums were taken about travels with them (keyed by the stats
    # object this call returned; bn_add_act pops it): a BN finalize must use
    # exactly this K (None: plain sums), not re-derive it from its module
    if want_stats:
        _SHIFT_USED[id(st)] = (weakref.ref(st), req if torch.is_tensor(req) else None)
    return y, st


# ------------------------------------------------------------------------ BN
class _BNActFn(torch.autograd.Function):
    """out = act( BN1(y1) + [BN2(y2) | res | 0] )."""

    @staticmethod
    def forward(ctx, cfg, y1, s1, g1, b1, res, y2, s2, g2, b2):
        bn1, bn2, relu, training, k1, k2 = cfg
        P = prims_for(y1)
        sync = _state["bn_sync"] if training else None
        two = y2 is not None
        p1, p2, count = _bn_forward_params(P, y1, s1, bn1, training, sync, y2, s2,
                                           bn2 if two else None, k1=k1, k2=k2)
        out, mask = P.bn_apply(y1, p1, res, y2, p2, relu)
        ctx.cfg = (bn1, bn2 if two else None, relu, training, res is not None, sync, count)
        ctx.save_for_backward(y1, mask if relu else _empty(y1.device), p1,
                              *([y2, p2] if two else []))
        return out

    @staticmethod
    def backward(ctx, dout):
        bn1, bn2, relu, training, has_res, sync, count = ctx.cfg
        sv = ctx.saved_tensors
        y1, mask, p1 = sv[:3]
        y2, p2 = (sv[3], sv[4]) if bn2 is not None else (None, None)
        P = prims_for(y1)
        dy1, dy2, dzm, g = _bn_backward(P, dout.contiguous(), mask, relu, training, sync, count,
                                        y1, p1, bn1, y2, p2, bn2, want_dzm=has_res)
        return None, dy1, None, g[0], g[1], (dzm if has_res else None), dy2, None, g[2], g[3]


def bn_add_act(y, stats, bn, residual=None, res_y=None, res_stats=None, res_bn=None, relu=True):
    k1, k2 = _pop_shift(stats), _pop_shift(res_stats)
    cfg = (bn, res_bn, relu, bn.training, k1, k2)
    if res_y is not None:
        return _BNActFn.apply(cfg, y, stats, bn.weight, bn.bias, None,
                              res_y, res_stats, res_bn.weight, res_bn.bias)
    return _BNActFn.apply(cfg, y, stats, bn.weight, bn.bias, residual, None, None, None, None)


def conv_bn_act(x, conv_mod, bn, relu=True):
    y, s = conv(x, conv_mod, want_stats=bn.training, bn=bn)
    return bn_add_act(y, s, bn, relu=relu)


# ------------------------------------------------------------- stem tail
class _StemPoolFn(torch.autograd.Function):
    """ImageNet stem tail as one node: out = maxpool3x3s2(relu(BN(y))), y = conv1(x)
    (reference resnet.py:97 + the ImageNet max-pool).  On the gfx950 path the
    activation is never materialised: one kernel forward (kernels/stem.hip),
    and the backward recomputes dz = pool-gradient * ReLU-mask from y in its
    reduce and elementwise passes."""

    @staticmethod
    def forward(ctx, cfg, y, st, g, b):
        bn, training, k1 = cfg
        P = prims_for(y)
        sync = _state["bn_sync"] if training else None
        p, _, count = _bn_forward_params(P, y, st, bn, training, sync, k1=k1)
        out, arg = P.stem_pool_fwd(y, p)
        # the producer is the space-to-depth stem conv (its only consumer is this node): the
        # backward may hand it the elementwise pass instead of a materialised dy
        ctx.lazy = bool(getattr(y, "_pmd_s2d", False)) and training and _STEM_LAZY
        ctx.cfg = (bn, training, sync, count)
        ctx.arg = arg
        ctx.save_for_backward(y, p)
        return out

    @staticmethod
    def backward(ctx, dout):
        bn, training, sync, count = ctx.cfg
        y, p = ctx.saved_tensors
        arg = ctx.arg
        P = prims_for(y)
        dout = dout.contiguous()
        red = P.stem_pool_bwd_reduce(dout, arg, y, p)

        def elemt(r, cnt):
            if ctx.lazy and r is not None:
                # dy for the stem conv's weight gradient, produced inside that kernel
                # (_StemS2DConvFn.backward -> stem_wgrad_fused): a stand-in of y's shape without
                # storage, carrying the elementwise pass's operands
                lz = torch.empty((), dtype=y.dtype, device=y.device).expand(y.shape)
                lz._pmd_stem = (dout, arg, y, p, bn.weight, r.contiguous(), cnt)
                return lz
            return P.stem_pool_bwd_elemt(dout, arg, y, p, bn.weight, r, cnt, eval_mode=not training)
        dy, _, _, g = _bn_backward(P, dout, None, True, training, sync, count, y, p, bn, pre=[red],
                                   elemt_fn=elemt)
        ctx.arg = None
        return None, dy, None, g[0], g[1]


# PMD_STEM_LAZY=1: the stem's backward elementwise pass inside the stem conv's weight gradient
# (kernels/conv_wgrad.hip stem_wgrad_fused_kernel: dy [N,112,112,64] never written nor re-read, -0.8 GB
# per step; bit-identical to the two passes, tests/test_stem_s2d_gpu.py).  Measured step-neutral
# (18.587 vs 18.567 ms, 3 interleaved rounds, profiles/stem_fused_r06.txt): the end of the backward is
# bounded by the side stream's layer-1 weight gradients, not by the stem -- off by default.
_STEM_LAZY = os.environ.get("PMD_STEM_LAZY", "0") == "1"


def fused_stem_enabled():
    return _state["fused_stem"]


def set_fused_stem(flag: bool):
    """ImageNet stem tail as one fused node (default) or conv_bn_act + max-pool."""
    _state["fused_stem"] = bool(flag)


def bn_relu_maxpool(y, stats, bn):
    """maxpool3x3s2(relu(BN(y))) for the ImageNet stem (fused on the gfx950 path).
    Consumes the statistics shift :func:`conv` registered for ``stats`` (like
    :func:`bn_add_act`), so no registry entry outlives the step."""
    return _StemPoolFn.apply((bn, bn.training, _pop_shift(stats)), y, stats, bn.weight, bn.bias)


# ------------------------------------------------- linear-BN backward (final BN)
def _bnlin_prep(P, bn, p, wpack, z):
    """Forward-time part of the linear-BN backward (see _bnlin_final), on the weight-gradient
    side stream while the forward continues: the diag(gamma * invstd)-scaled dgrad image of the
    conv3 weights and the z statistics the weight gradient needs (z^T z, colsum z).  Returns
    (dgrad pack, Gz, colsum, event or None)."""
    c = z.shape[-1]
    wk = wpack[0]

    def work():
        return (P.bnlin_dimg(bn.weight, p, wk, c), P.conv_wgrad(z, z, (c, 1, 1, c), 1, 0), P.colsum(z))
    if not (z.is_cuda and _WGRAD_STREAM["on"] and not _state["force_torch"]):
        return (*work(), None)
    side = _wgrad_stream(z.device)
    main = torch.cuda.current_stream(z.device)
    _stream_wait(side, main)
    with torch.cuda.stream(side):
        dpack, gz, cs = work()
    z.record_stream(side)
    p.record_stream(side)
    for t in dpack:
        if t is not None:
            t.record_stream(main)
    return dpack, gz, cs, _record_on(side)


def _bnlin_final(P, dz, pre, training, sync, count, z, wpack, conv_m, bn, p, rec_prev, side, put, prep):
    """Backward of ``out = relu(BN(y) + x)`` with ``y = z W^T`` (a 1x1 stride-1 conv) that never
    materialises ``dy`` (the BN passes are the step's bytes): no BN-backward
    elementwise pass.  ``dz = dout * relu_mask`` arrives from the next block's dgrad together
    with its fused statistics (slots ``pre[0]``: sum dz, sum dz*xhat).  With
    dy = A dz + B y + Cc per channel k (A = gamma*invstd from the forward; B, Cc from the
    global sums after the collapse / SyncBN exchange, which run exactly as at every site):

      D      = dz (diag(A) W)       plain dgrad on the forward-prepared scaled image
      dz_in  = D + z (W^T diag(B) W) + Cc W     one small GEMM of z (reduction = C) with D as
                                                its addend, the bias and the previous BN's fused
                                                reduce in its epilogue  (B y W = z W^T B W)
      dW     = diag(A) T + diag(B) W (z^T z) + Cc (x) colsum(z),   T = dz^T z   (side stream:
               T is the conv's own weight-gradient GEMM; z^T z, colsum z from the forward)

    W is the bf16 compute image the forward used, so y = z W^T is the forward's product before
    its bf16 rounding -- the one difference from the elementwise path.  Returns (dz_in, the
    fused reduce of ``rec_prev``'s BN, [d_gamma, d_beta] for params not in the arena)."""
    wk = wpack[0]
    c = z.shape[-1]
    dpack, gz, cs, ev = prep
    T, _ = side.fork(lambda: P.conv_wgrad(dz, z, tuple(wk.shape), 1, 0), keep=(dz, z))
    if ev is not None:
        _wait_on(torch.cuda.current_stream(dz.device), ev)
    dmain = P.conv_dgrad(dz, dpack, tuple(z.shape), 1, 0)             # dz diag(A) W
    state = {}

    def lin(red, cnt):
        gpack, bias, abc = P.bnlin_coeff(red, cnt, bn.weight, p, wk, c)
        _hin, _wp, y_, p_, z_ = rec_prev
        dx, red_ = P.conv_dgrad(z, gpack, tuple(z.shape), 1, 0, dmain, bnred=(z_, [(y_, p_)]),
                                addend_bias=bias)
        state["pre"] = _Pre(red_, _after_dgrad_event(dx, sync if training else None))
        state["abc"] = abc
        return dx

    dx, _, _, g = _bn_backward(P, dz, None, False, training, sync, count, dz, p, bn,
                               pre=pre, elemt_fn=lin)
    abc = state["abc"]

    def wgrad(out):
        P.bnlin_wgrad_(out, abc, T, wk, gz, cs)
    put(conv_m.weight, side.run(conv_m.weight, wgrad, keep=(abc, wk)))
    return dx, state["pre"], g


# ------------------------------------------------------------ residual block
class _BnSite:
    """Hand-off between two consecutive residual blocks for the fused BN reduce:
    block i (forward) records its final BN(s) (ReLU mask, [(y, params)]); block
    i+1 (backward) computes d(out_i) with the reduce fused into the same dgrad
    epilogue and deposits the partial sums; block i (backward) takes them iff
    the gradient it received IS that tensor (otherwise -- e.g. the output had
    another consumer and autograd summed gradients -- it recomputes)."""

    __slots__ = ("mask", "sets", "red", "dx_ptr", "dx_shape")

    def __init__(self, mask, sets):
        self.mask = mask
        self.sets = sets
        self.red = None
        self.dx_ptr = None
        self.dx_shape = None

    def put(self, dx, red):
        self.red = red
        self.dx_ptr = dx.data_ptr()
        self.dx_shape = tuple(dx.shape)

    def take(self, dout, P):
        red, self.red = self.red, None
        if red is None:
            return None
        if dout.data_ptr() == self.dx_ptr and tuple(dout.shape) == self.dx_shape:
            _state["fused_site_hits"] += 1
            return red
        _state["fused_site_misses"] += 1
        rel = getattr(P, "_release", None)
        if rel is not None:
            for b in red:          # the pool hands out zeroed slot buffers only
                b.zero_()
            rel(*red)
        return None


class _ResidualBlockFn(torch.autograd.Function):
    """A whole ResNet block as one autograd node.

    stages   : [(conv, bn)]*  conv -> BN -> ReLU  (Bottleneck: 1x1, 3x3; Basic: 3x3)
    final    : (conv, bn)     conv -> BN, then + shortcut, ReLU
    shortcut : None (identity) or (conv, bn) projection on the block input
    """

    @staticmethod
    def forward(ctx, cfg, x, *params):
        stages, final, shortcut, training = cfg
        P = prims_for(x)
        sync = _state["bn_sync"] if training else None
        f8 = _fp8_for(P)
        hq = None
        if f8 is not None:
            # e4m3 copy of the block input: written by the previous block's BN-apply,
            # else quantised here (first block: the max-pool output)
            hq = getattr(x, "_pmd_q8", None)
            if hq is not None:
                x._pmd_q8 = None                # consumed: do not keep it alive with x
            elif (fp8_eligible(stages[0][0], x.shape[-1])
                  or (shortcut is not None and fp8_eligible(shortcut[0], x.shape[-1]))):
                sx, ax = f8.site(("in", id(stages[0][0])))
                hq = (P.quant_bf16_fp8(x, sx, ax), sx)
        xq = hq
        # fp8 weight gradients: a conv whose forward read an e4m3 input keeps that input
        # (+ its scale) for an e5m2 x e4m3 wgrad, and a stage activation consumed only by
        # such a conv is written in e4m3 alone (no bf16 copy: h is then the uint8 tensor,
        # used for its shape)
        # (grad mode is off inside Function.forward: ask the node whether a backward follows)
        f8w = f8 is not None and training and FP8_WGRAD and any(ctx.needs_input_grad)

        def used_q(conv_m, hq_, h_):
            return hq_ if (hq_ is not None and fp8_eligible(conv_m, h_.shape[-1])) else None
        # projection shortcut of a two-stream step: its conv (+ BN statistics) on the side stream,
        # which is idle during the forward, concurrent with the main path's convs; joined before
        # the final BN-apply that adds it
        sc_pre = None
        if shortcut is not None and _SIDE_SHORTCUT and x.is_cuda and _WGRAD_STREAM["on"] \
                and not _state["force_torch"] and not torch.cuda.is_current_stream_capturing():
            sconv, sbn = shortcut
            wps = _conv_weight(P, sconv, x.dtype, x.shape[-1], x.requires_grad)
            xq_s = used_q(sconv, xq, x)
            main = torch.cuda.current_stream(x.device)
            side = _wgrad_stream(x.device)
            _stream_wait(side, main)
            with torch.cuda.stream(side):
                ys, sts = _conv_fwd_any(P, f8, x, xq_s, wps, sconv, _stats_req(sbn, training))
            x.record_stream(side)
            if xq_s is not None:
                xq_s[0].record_stream(side)
            sc_pre = (wps, xq_s, ys, sts, _record_on(side), main)
        h = x
        recs, qins = [], []
        nxt_convs = [c for c, _ in stages[1:]] + [final[0]]
        for si, (conv_m, bn) in enumerate(stages):
            wp = _conv_weight(P, conv_m, x.dtype, h.shape[-1], True)
            hq_in = used_q(conv_m, hq, h)
            y, st = _conv_fwd_any(P, f8, h, hq_in, wp, conv_m, _stats_req(bn, training))
            p, _, count = _bn_forward_params(P, y, st, bn, training, sync)
            if f8 is not None and fp8_eligible(nxt_convs[si], y.shape[-1]):
                site = f8.site(("a", id(bn)))
                z, zmask, zq = P.bn_apply(y, p, relu=True, fp8=site, fp8_only=f8w)
                hq = (zq, site[0])
                if z is None:
                    z = zq
            else:
                z, zmask = P.bn_apply(y, p, relu=True)
                hq = None
            recs.append((h, wp, y, p, zmask, count))
            qins.append(hq_in if f8w else None)
            h = z
        fconv, fbn = final
        wpf = _conv_weight(P, fconv, x.dtype, h.shape[-1], True)
        hq_f = used_q(fconv, hq, h)
        fuse = _state["fuse_bnred"] and training
        yf, stf = _conv_fwd_any(P, f8, h, hq_f, wpf, fconv, _stats_req(fbn, training))
        qins.append(hq_f if f8w else None)
        # e4m3 copy of the block output only if its consumer -- the next block's first
        # conv, which has this block's first-conv kernel shape -- runs in fp8
        osite = (f8.site(("a", id(fbn))) if f8 is not None and fp8_eligible(stages[0][0], yf.shape[-1])
                 else None)
        if shortcut is not None:
            sconv, sbn = shortcut
            if sc_pre is not None:
                wps, xq_s, ys, sts, ev, main = sc_pre
                _wait_on(main, ev)
                ys.record_stream(main)               # allocated on the side stream, used here
                if sts is not None:
                    sts.record_stream(main)
            else:
                wps = _conv_weight(P, sconv, x.dtype, x.shape[-1], x.requires_grad)
                xq_s = used_q(sconv, xq, x)
                ys, sts = _conv_fwd_any(P, f8, x, xq_s, wps, sconv, _stats_req(sbn, training))
            qins.append(xq_s if f8w else None)
            pf, ps, countf = _bn_forward_params(P, yf, stf, fbn, training, sync, ys, sts, sbn)
            r = P.bn_apply(yf, pf, None, ys, ps, relu=True, **({"fp8": osite} if osite else {}))
        else:
            wps = None
            pf, _, countf = _bn_forward_params(P, yf, stf, fbn, training, sync)
            r = P.bn_apply(yf, pf, x, relu=True, **({"fp8": osite} if osite else {}))
        out, omask = r[0], r[1]
        if osite is not None:
            out._pmd_q8 = (r[2], osite[0])      # the next block's fp8 conv input
        ctx.cfg = (cfg, sync, [r[5] for r in recs], countf, len(wpf),
                   0 if wps is None else len(wps), [len(r[1]) for r in recs])
        # e4m3 conv inputs for the fp8 wgrads: (q, scale) per stage conv, final conv,
        # projection conv; the scales are views of the Fp8Scaling buffer, which the next
        # update() rewrites only after this backward (stream order)
        ctx.qins = qins if any(q is not None for q in qins) else None
        ctx.f8 = f8 if f8w else None
        wi = _state["wimg"]
        ctx.f8img = (wi.fp8 if (f8w and FP8_DGRAD and wi is not None and wi.fp8 is not None
                                and wi.fp8.f8 is f8) else None)
        # cross-block fusion: the NEXT block's first dgrad computes d(out) and can
        # reduce this block's final BN(s) in its epilogue.  The site carries what
        # it needs; the input's site (previous block) is remembered likewise.
        ctx.in_site = getattr(x, "_pmd_bnsite", None) if fuse else None
        ctx.out_site = None
        # linear-BN backward of the final BN (no elementwise pass, see _bnlin_final)
        ctx.bnlin = (_bnlin_eligible(fconv, yf, x, training, fuse, shortcut, f8)
                     and h.shape[-1] == wpf[0].shape[-1])
        ctx.bnlin_prep = _bnlin_prep(P, fbn, pf, wpf, h) if ctx.bnlin else None
        if fuse:
            ctx.out_site = _BnSite(omask, [(yf, pf)] + ([(ys, ps)] if shortcut is not None else []))
            out._pmd_bnsite = ctx.out_site
        # saved: the ReLU bitmasks (not the activations they came from) + conv inputs
        flat = [x, omask, yf, pf, h, *wpf]
        for (hin, wp, y, p, zmask, _) in recs:
            flat += [hin, y, p, zmask, *wp]
        if shortcut is not None:
            flat += [ys, ps, *wps]
        ctx.save_for_backward(*flat)
        return out

    @staticmethod
    def backward(ctx, dout):
        cfg, sync, counts, countf, nwf, nws, nwst = ctx.cfg
        stages, final, shortcut, training = cfg
        nst = len(stages)
        sv = list(ctx.saved_tensors)
        x, omask, yf, pf, hlast = sv[:5]
        i = 5
        wpf = tuple(sv[i:i + nwf])
        i += nwf
        recs = []
        for k in range(nst):
            hin, y, p, z = sv[i:i + 4]
            i += 4
            recs.append((hin, tuple(sv[i:i + nwst[k]]), y, p, z))
            i += nwst[k]
        P = prims_for(x)
        dout = dout.contiguous()
        fconv, fbn = final
        grads = {}
        nan_check = _NAN_CHECK

        def chk(name, t):
            if nan_check and t is not None:
                q8 = getattr(t, "_pmd_q8", None)
                if t.dtype == torch.uint8 and q8 is not None:
                    # an e5m2-only dY (fp8 gradients): the raw bytes are always "finite"
                    # as floats, so check the dequantised values
                    from .native import C
                    t = C.dequant_fp8(t, 1.0 / q8[1], bf8=True)
                if not torch.isfinite(t.float()).all():
                    raise FloatingPointError(f"non-finite {name} in block backward ({fconv.weight.shape})")
        chk("dout", dout)

        def put(p, g):
            if g is not None:
                grads[id(p)] = g

        qins = ctx.qins or [None] * (nst + 2)

        convs = [c for c, _ in stages] + [final[0]] + ([shortcut[0]] if shortcut is not None else [])

        def gsite(i, bn_):
            # e5m2 scale/amax site of the dY that feeds conv i's fp8 weight gradient, and
            # whether that copy is the only one (conv i's dgrad runs in fp8 as well)
            if ctx.f8 is None or i >= len(qins) or qins[i] is None:
                return None
            sc, am = ctx.f8.grads.site(("dy", id(bn_)))
            only = ctx.f8img is not None and ctx.f8img.lookup_t(convs[i]) is not None
            return sc, am, only
        # reduce of the final BN(s), if the next block's dgrad already produced it
        pre = ctx.out_site.take(dout, P) if ctx.out_site is not None else None
        # --- final BN (+ projection BN) and the residual ReLU
        if shortcut is not None:
            sconv, sbn = shortcut
            ys, ps = sv[i], sv[i + 1]
            wps = tuple(sv[i + 2:i + 2 + nws])
            dyf, dys, _, g = _bn_backward(P, dout, omask, True, training, sync, countf,
                                          yf, pf, fbn, ys, ps, sbn, pre=pre,
                                          q8=(gsite(nst, fbn), gsite(nst + 1, sbn)))
            put(sbn.weight, g[2])
            put(sbn.bias, g[3])
            dres = None
        else:
            # the identity-path gradient dout * relu_mask is NOT materialised: the first
            # stage's dgrad epilogue adds dout gated by the mask bits
            if not (ctx.bnlin and pre is not None):
                dyf, _, _, g = _bn_backward(P, dout, omask, True, training, sync, countf,
                                            yf, pf, fbn, pre=pre,
                                            q8=(gsite(nst, fbn), None))
            # dout pre-masked by the fused reduce (see _bn_backward): no addend mask either
            dres = (dout, None if (pre is not None and _PREMASKED) else omask)
        lin = shortcut is None and ctx.bnlin and pre is not None
        if not lin:
            put(fbn.weight, g[0])
            put(fbn.bias, g[1])
        fuse = _state["fuse_bnred"] and training

        f8img = ctx.f8img

        def dgrad(dy_, wp_, conv_m_, shape, addend=None, bnred=None, addend_mask=None):
            # fp8 data gradient when dY carries its e5m2 copy and the conv keeps an e4m3
            # transposed weight image; else the bf16 kernel (same epilogue options)
            dq = getattr(dy_, "_pmd_q8", None)
            if dq is not None and f8img is not None:
                wtq = f8img.lookup_t(conv_m_)
                if wtq is not None:
                    sw = ctx.f8.site(("w", id(conv_m_)))[0]
                    return P.conv_dgrad_fp8(dq[0], dq[1], wtq, sw, shape, conv_m_.stride, conv_m_.padding,
                                            addend, bnred=bnred, addend_mask=addend_mask)
            return P.conv_dgrad(dy_, wp_, shape, conv_m_.stride, conv_m_.padding, addend, bnred=bnred,
                                addend_mask=addend_mask)

        def dgrad_fused(dy_, wp_, conv_m_, shape, rec, addend=None):
            # dgrad whose output feeds stage rec's BN+ReLU backward: fuse its reduce
            if not fuse:
                return dgrad(dy_, wp_, conv_m_, shape, addend), None
            _hin, _wp, y_, p_, z_ = rec
            dx_, red_ = dgrad(dy_, wp_, conv_m_, shape, addend, bnred=(z_, [(y_, p_)]))
            return dx_, _Pre(red_, _after_dgrad_event(dx_, sync if training else None))
        side = _WgradSide(dout)
        if lin:
            # linear-BN backward of the final BN through the 1x1 conv3 (no y, no dy)
            dh, pre_k, g = _bnlin_final(P, dout, pre, training, sync, countf, hlast, wpf, fconv,
                                        fbn, pf, recs[-1], side, put, ctx.bnlin_prep)
            ctx.bnlin_prep = None
            put(fbn.weight, g[0])
            put(fbn.bias, g[1])
        else:
            chk("dyf", dyf)
            # --- final conv (its wgrad forks to the side stream first: it overlaps the dgrad)
            put(fconv.weight, side.wgrad(P, dyf, hlast, wpf, fconv.stride, fconv.padding, fconv.weight,
                                         qins[nst]))
            dh, pre_k = dgrad_fused(dyf, wpf, fconv, tuple(hlast.shape), recs[-1])
        chk("dh(final)", dh)
        dx = None
        # --- conv->BN->ReLU stages in reverse; the block-input gradient of the
        #     residual/projection path is added in the first stage's dgrad epilogue
        for k in range(nst - 1, -1, -1):
            conv_m, bn = stages[k]
            hin, wp, y, p, zmask = recs[k]
            dy, _, _, g = _bn_backward(P, dh, zmask, True, training, sync, counts[k], y, p, bn,
                                       pre=pre_k, q8=(gsite(k, bn), None))
            put(bn.weight, g[0])
            put(bn.bias, g[1])
            chk(f"dy(stage {k})", dy)
            put(conv_m.weight, side.wgrad(P, dy, hin, wp, conv_m.stride, conv_m.padding,
                                          conv_m.weight, qins[k]))
            if k > 0:
                dh, pre_k = dgrad_fused(dy, wp, conv_m, tuple(hin.shape), recs[k - 1])
            elif ctx.needs_input_grad[1]:
                if shortcut is not None:
                    addend = dgrad(dys, wps, sconv, tuple(x.shape))
                    amask = None
                else:
                    addend, amask = dres
                site = ctx.in_site
                if site is not None:
                    # d(x) is the previous block's d(out): reduce ITS final BN(s) here
                    dx, site_red = dgrad(dy, wp, conv_m, tuple(x.shape), addend,
                                         bnred=(site.mask, site.sets), addend_mask=amask)
                    site.put(dx, _Pre(site_red, _after_dgrad_event(dx, sync if training else None)))
                else:
                    dx = dgrad(dy, wp, conv_m, tuple(x.shape), addend, addend_mask=amask)
        if shortcut is not None:
            put(sconv.weight, side.wgrad(P, dys, x, wps, sconv.stride, sconv.padding, sconv.weight,
                                         qins[nst + 1]))
        side.join()
        return (None, dx, *[grads.get(id(p)) for p in _block_params(stages, final, shortcut)])


def _block_params(stages, final, shortcut):
    ps = []
    for conv_m, bn in [*stages, final] + ([shortcut] if shortcut is not None else []):
        ps += [conv_m.weight, bn.weight, bn.bias]
    return ps


def residual_block(x, stages, final, shortcut, training):
    """Run a ResNet block (see :class:`_ResidualBlockFn`) as one autograd node."""
    cfg = (tuple(stages), final, shortcut, training)
    return _ResidualBlockFn.apply(cfg, x, *_block_params(stages, final, shortcut))


# --------------------------------------------------------------------- pools
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        P = prims_for(x)
        out, idx = P.maxpool_fwd(x)
        ctx.save_for_backward(idx)
        ctx.xshape = tuple(x.shape)
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        return prims_for(dout).maxpool_bwd(dout.contiguous(), idx, ctx.xshape)


def max_pool3x3s2(x):
    return _MaxPoolFn.apply(x)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.xshape = tuple(x.shape)
        ctx.dtype = x.dtype
        return prims_for(x).avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dout):
        return prims_for(dout).avgpool_bwd(dout.contiguous(), ctx.xshape, ctx.dtype)


def global_avg_pool(x):
    """[N,H,W,C] -> [N,C] (fp32 accumulation)."""
    return _AvgPoolFn.apply(x)


class _LinearFn(torch.autograd.Function):
    """Classifier head (reference model/resnet.py:86,104) on the gfx950 MFMA GEMMs
    (kernels/linear.hip): forward with the bias fused, dgrad, and the weight /
    bias gradients written straight into the gradient arena (no AccumulateGrad
    pass, no library GEMM or reduction kernels on the step)."""

    @staticmethod
    def forward(ctx, x, w, b):
        P = prims_for(x)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.b = b
        return P.linear_fwd(x, w, b)

    @staticmethod
    def backward(ctx, dout):
        x, w = ctx.saved_tensors
        b = ctx.b
        P = prims_for(dout)
        dout = dout.contiguous()
        dx = P.linear_dgrad(dout, w).to(x.dtype) if ctx.needs_input_grad[0] else None
        tw = _grad_target(w)
        tb = _grad_target(b) if b is not None else None
        dw = db = None
        if tw is not None and (b is None or tb is not None):
            P.linear_wgrad(dout, x, tw, tb, True)
            _ready(w, *([b] if b is not None else []))
        else:
            if ctx.needs_input_grad[1]:
                dw = torch.empty_like(w, dtype=torch.float32)
                db = torch.empty_like(b, dtype=torch.float32) if (b is not None and ctx.needs_input_grad[2]) else None
                P.linear_wgrad(dout, x, dw, db, False)
            elif b is not None and ctx.needs_input_grad[2]:
                db = dout.float().sum(0)
        return dx, dw, db


def linear(x, lin):
    return _LinearFn.apply(x, lin.weight, lin.bias)


# ---------------------------------------------------------------------- loss
class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        P = prims_for(logits)
        loss, lse = P.xent_fwd(logits.contiguous(), target)
        ctx.save_for_backward(logits, target, lse)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, gloss):
        logits, target, lse = ctx.saved_tensors
        P = prims_for(logits)
        return P.xent_bwd(gloss.reshape(1).to(logits.dtype), logits, target, lse), None


def cross_entropy(logits, target):
    """Mean softmax cross-entropy (== nn.CrossEntropyLoss(), reference main.py:48)."""
    return _XentFn.apply(logits, target)


_SEEDS: dict = {}


def loss_seed(loss):
    """d(loss)/d(loss) = 1 as a cached device scalar: ``loss.backward(loss_seed(loss))``
    is ``loss.backward()`` without the ATen fill autograd launches for its
    implicit ones_like seed every step (read-only: the loss backward only reads it)."""
    key = (loss.device, loss.dtype)
    t = _SEEDS.get(key)
    if t is None:
        t = _SEEDS[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
    return t


def correct_count(logits, target):
    """Device-side top-1 correct count (int64 [1]); no host sync."""
    return prims_for(logits).correct_count(logits, target)
