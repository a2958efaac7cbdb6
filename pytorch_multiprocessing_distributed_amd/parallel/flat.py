"""Flat parameter / gradient arenas.

All trainable parameters of a module are re-homed into ONE contiguous fp32
arena (and their ``.grad`` into a second one), laid out in *reverse
registration order* -- the order gradients become ready in backward, which is
also the order torch's DDP Reducer builds buckets in
(torch:nn/parallel/distributed.py:828-834).  Consequences:

  * a gradient bucket is a contiguous slice of the grad arena, so the
    all-reduce runs in place on it with zero copies (DDP's
    ``gradient_as_bucket_view`` without the bookkeeping);
  * the optimizer is one fused kernel over the whole arena (K16);
  * the initial rank-0 broadcast is a single collective (C3).

Parameter logical shapes/strides are preserved (conv weights keep their
channels-last strides), so state_dict keys/shapes are unchanged.

:meth:`FlatParams.relayout` re-orders the arenas in place (same storage) once
the data-parallel wrapper has OBSERVED the order gradients become ready in
(torch's Reducer rebuilds its buckets after the first iteration the same way,
torch:nn/parallel/distributed.py:1551); optimizer state arenas registered as
``companions`` are permuted with them.
"""
from __future__ import annotations

import torch

_ALIGN = 4  # elements (16 B) -> every parameter view starts 16-B aligned


def _phys_shape_and_perm(p):
    """Dense physical shape + permutation back to the logical view."""
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
        k, c, r, s = p.shape
        return (k, r, s, c), (0, 3, 1, 2)
    return tuple(p.shape), None


class FlatParams:
    def __init__(self, module: torch.nn.Module, dtype=None):
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if not named:
            raise ValueError("module has no trainable parameters")
        self.names = [n for n, _ in reversed(named)]
        self.params = [p for _, p in reversed(named)]
        dev = self.params[0].device
        dtype = dtype or self.params[0].dtype
        for p in self.params:
            if p.dtype != dtype:
                raise TypeError(f"flat arena expects {dtype} master params, got {p.dtype}")
            if p.device != dev:
                raise ValueError("all parameters must live on one device")
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        self.device = dev
        self.version = 0          # bumped by relayout(): parameter storage moved
        self.companions = []      # same-layout state arenas (optimizer momentum)
        self.param_arena = torch.zeros(off, dtype=dtype, device=dev)
        self.grad_arena = torch.zeros(off, dtype=dtype, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                pv = self._view(self.param_arena, p, o)
                pv.copy_(p.detach())
                p.data = pv
                p.grad = self._view(self.grad_arena, p, o)
                # fused ops may accumulate this param's gradient straight into the arena
                p._pmd_direct = True

    @staticmethod
    def _view(arena, p, off):
        phys, perm = _phys_shape_and_perm(p)
        v = arena[off: off + p.numel()].view(phys)
        return v.permute(*perm) if perm else v

    def slice_of(self, i):
        o = self.offsets[i]
        return o, o + self.params[i].numel()

    @torch.no_grad()
    def relayout(self, order):
        """Re-order the arenas so parameter ``order[k]`` (current index) comes
        k-th; contents move in place (no reallocation), ``p.data``/``p.grad``
        are re-pointed.  Returns nothing; ``self.params``/``names``/``offsets``
        follow the new order and ``version`` increments."""
        order = [int(i) for i in order]
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("relayout: order must be a permutation of the parameter indices")
        if order == list(range(len(self.params))):
            return
        new_params = [self.params[i] for i in order]
        new_offsets, off = [], 0
        for p in new_params:
            new_offsets.append(off)
            off += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        assert off == self.numel
        for arena in [self.param_arena, self.grad_arena, *self.companions]:
            tmp = arena.clone()
            for i, no in zip(order, new_offsets):
                oo, n = self.offsets[i], self.params[i].numel()
                arena[no: no + n].copy_(tmp[oo: oo + n])
        for p, o in zip(new_params, new_offsets):
            p.data = self._view(self.param_arena, p, o)
            p.grad = self._view(self.grad_arena, p, o)
        self.names = [self.names[i] for i in order]
        self.params = new_params
        self.offsets = new_offsets
        self.version += 1

    def zero_grad(self):
        if self.grad_arena.is_cuda:
            from ..ops.native import C
            C.zero_(self.grad_arena)       # the framework's fill kernel, not ATen's
        else:
            self.grad_arena.zero_()

    def rebind_grads(self):
        """Re-attach .grad views (e.g. after someone set them to None)."""
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad_arena[o:].data_ptr():
                p.grad = self._view(self.grad_arena, p, o)


def get_flat(module) -> "FlatParams | None":
    return getattr(module, "_pmd_flat", None)


def flatten_module(module) -> FlatParams:
    fp = get_flat(module)
    if fp is None:
        fp = FlatParams(module)
        object.__setattr__(module, "_pmd_flat", fp)
    return fp
