"""Fused SGD (momentum / Nesterov / weight decay) over the flat arena.

Math is exactly ``torch.optim.SGD`` (torch:optim/sgd.py:383-477) as used by
the reference (lr 0.1, momentum 0.9, wd 1e-4, nesterov; main.py:51-55):

    g   = g + wd * p
    buf = g                      (first step)   | m * buf + (1 - dampening) * g
    g   = g + m * buf            (nesterov)     | buf
    p   = p - lr * g

but the whole model is ONE kernel launch over the flat param/grad/momentum
arenas (K16) instead of ~5 multi-tensor launches.  It subclasses
``torch.optim.Optimizer`` so ``torch.optim.lr_scheduler.MultiStepLR`` (the
reference scheduler, main.py:57-59) drives ``param_groups[0]['lr']``.
"""
from __future__ import annotations

import torch

from ..ops.functional import prims_for
from ..parallel.flat import flatten_module, get_flat


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, module, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True,
                 dampening=0.0):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        inner = getattr(module, "module", module)
        self.flat = get_flat(inner) or flatten_module(inner)
        defaults = dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov,
                        dampening=dampening)
        super().__init__(self.flat.params, defaults)
        self.momentum_arena = torch.zeros_like(self.flat.param_arena)
        self.flat.companions.append(self.momentum_arena)   # follows arena relayouts
        self.steps = 0
        # device-resident learning rate: the SGD kernel reads it, so a captured
        # HIP graph of the step follows scheduler updates (see graph_safe())
        self.lr_dev = None
        self._lr_cached = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        P = prims_for(self.flat.param_arena)
        if self.lr_dev is not None and not torch.cuda.is_current_stream_capturing():
            self.sync_lr()
        P.sgd_nesterov_(self.flat.param_arena, self.flat.grad_arena, self.momentum_arena,
                        g["lr"], g["momentum"], g["weight_decay"], g["nesterov"],
                        self.steps == 0, g["dampening"], self.lr_dev)
        self.steps += 1
        return loss

    def graph_safe(self):
        """Switch to the device-resident LR (call before capturing a step)."""
        if self.lr_dev is None:
            self.lr_dev = torch.zeros(1, dtype=torch.float32, device=self.flat.device)
            self._lr_cached = None
            self.sync_lr()
        return self

    def sync_lr(self):
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_cached:
            self.lr_dev.fill_(lr)
            self._lr_cached = lr

    def zero_grad(self, set_to_none: bool = False):
        # grads are views into the arena: always zero in place
        self.flat.zero_grad()

    # ------------------------------------------------------ resume state
    def state_dict(self):
        # momentum per parameter name: independent of the arena layout (which the
        # data-parallel wrapper re-orders after its first iteration)
        mom = {n: self.momentum_arena[o: o + p.numel()].detach().cpu().clone()
               for n, p, o in zip(self.flat.names, self.flat.params, self.flat.offsets)}
        return {"steps": self.steps, "momentum": mom,
                "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                 for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.steps = int(sd["steps"])
        mom = sd["momentum"]
        if isinstance(mom, dict):
            for n, p, o in zip(self.flat.names, self.flat.params, self.flat.offsets):
                self.momentum_arena[o: o + p.numel()].copy_(mom[n].to(self.momentum_arena.device))
        else:   # flat arena in construction order (older resume files)
            self.momentum_arena.copy_(mom.to(self.momentum_arena.device))
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
