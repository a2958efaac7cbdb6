"""FP8 (OCP e4m3) training precision -- BASELINE config 5.

Recipe ("fp8 weights + activations" for the convolution GEMMs):
  * every block convolution's FORWARD runs on the CDNA4 scaled fp8 MFMA
    (``v_mfma_scale_f32_16x16x128_f8f6f4``, 2x the bf16 rate): its weight is
    quantised per step from the fp32 master into an e4m3 KRSC image, its input
    activation is the e4m3 copy that the producing BN-apply kernel writes next
    to the bf16 one (no extra pass);
  * per-tensor *delayed* scaling: each site (weight / activation) owns a scale
    and an amax in two flat device buffers; kernels accumulate amax while they
    quantise, and ``Fp8Scaling.update()`` (once per training step, one fused
    device op, no host sync) turns last step's amax into this step's scale
    ``448 / amax``;
  * the WEIGHT GRADIENT of every conv whose forward ran in fp8 runs on the same
    scaled MFMA (``conv_wgrad_fp8``: e5m2 dY x e4m3 X, 2x the bf16 rate, half the
    operand bytes): the BN-backward elementwise pass writes an e5m2 (bf8) copy of dY
    next to the bf16 one, with its own delayed scale (``Fp8Scaling.grads``, fmax
    57344), and the X operand is the e4m3 activation the forward already made --
    which is then the ONLY copy of a stage activation (BN-apply skips the bf16 one);
  * the stem conv, the classifier, BatchNorm, the loss and the data-gradient GEMMs
    stay in bf16 / fp32 (fp32 master weights, reference checkpoint format
    unchanged).
"""
from __future__ import annotations

import torch

E4M3_MAX = 448.0
E5M2_MAX = 57344.0
AMAX_SLOTS = 64     # == kAmaxSlots (csrc/kernels/common.h)
# first-step scale of a gradient (e5m2) site, before any amax was observed: values up
# to 57344 / 4096 = 14 representable, normals down to 2^-14 / 4096 ~ 1.5e-8
GRAD_INIT_SCALE = 4096.0


class Fp8Scaling:
    def __init__(self, device, capacity: int = 1024, margin: float = 1.0, fmax: float = E4M3_MAX,
                 init_scale: float = 1.0, grads: bool = True):
        self.device = torch.device(device)
        self.fmax = float(fmax)
        # [site][slot]: kernels atomicMax into slot (block % 64) -- no single-address contention
        self.amax = torch.zeros(capacity, AMAX_SLOTS, dtype=torch.float32, device=self.device)
        self.scale = torch.full((capacity,), float(init_scale), dtype=torch.float32, device=self.device)
        self.capacity = capacity
        self.margin = float(margin)
        self.sites: dict = {}
        self._views: dict = {}
        self.steps = 0
        # e5m2 sites of the backward (dY of the fp8 weight gradients); margin 2: a
        # gradient may grow between steps, saturating costs more than one bit of range
        self.grads = (Fp8Scaling(device, capacity, margin=2.0, fmax=E5M2_MAX, init_scale=GRAD_INIT_SCALE,
                                 grads=False) if grads else None)

    def site(self, key, init_from: torch.Tensor | None = None):
        """(scale [1], amax [64 slots]) views for ``key``; a new weight site takes
        its first scale from the tensor's current amax (device op, no sync)."""
        v = self._views.get(key)
        if v is not None:                   # hot path: no tensor slicing per call
            return v
        idx = self.sites.get(key)
        if idx is None:
            idx = len(self.sites)
            if idx >= self.capacity:
                raise RuntimeError("Fp8Scaling capacity exceeded")
            self.sites[key] = idx
            if init_from is not None:
                a = init_from.detach().abs().max().float().clamp_min(1e-12)
                self.scale[idx:idx + 1].copy_((self.fmax / self.margin) / a)
        v = self._views[key] = (self.scale[idx:idx + 1], self.amax[idx])
        return v

    @torch.no_grad()
    def update(self):
        """Delayed scaling: scale <- 448 / amax(previous step) where observed; amax <- 0.
        On the GPU one native launch (``fp8_update_scales``: a wave per site folds its
        64 amax slots); elsewhere the same in torch ops."""
        if self.grads is not None:
            self.grads.update()
        n = len(self.sites)
        if n == 0:
            return
        if self.device.type == "cuda":
            from .native import C
            C.fp8_update_scales(self.amax, self.scale, n, self.fmax / self.margin)
        else:
            a = self.amax[:n].amax(dim=1)
            s = self.scale[:n]
            torch.where(a > 0, (self.fmax / self.margin) / a.clamp_min(1e-12), s, out=s)
            self.amax[:n].zero_()
        self.steps += 1

    def amax_of(self, key):
        """Current-step amax of a site (max over its slots)."""
        return self.amax[self.sites[key]].max()

    def state_dict(self):
        return {"scale": self.scale.cpu(), "amax": self.amax.amax(dim=1).cpu(), "sites": len(self.sites)}
