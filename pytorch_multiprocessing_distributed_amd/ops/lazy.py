"""A BatchNorm-backward output that is never written to memory.

The reference's BN backward (``batch_norm_backward_elemt``, reached through
model/resnet.py:36-39 / 66-70 -> nn.SyncBatchNorm) produces dY and stores it
for the conv backward that consumes it.  Per channel that elementwise pass is
affine in its two inputs,

    dY = a * dzm + b * y + c        (dzm = dZ gated by the ReLU mask)

so when the consumer is a 1x1 convolution the gfx950 dgrad / wgrad kernels
apply it while reading their operand (kernels/conv_igemm.hip "TX",
kernels/conv_wgrad.hip): the dzm and y tiles are read side by side and
transformed in registers.  That removes a 3-tensor-pass kernel (read dZ, y,
mask; write dY) per BN site from the critical main stream in exchange for one
extra operand read in each consumer.  ``LazyDy`` carries the operands; the
coefficients come from one tiny kernel (bn_bwd_coef, the exact terms
bn_bwd_elemt uses).
"""
from __future__ import annotations


class LazyDy:
    __slots__ = ("dzm", "y", "coef", "_args")

    def __init__(self, dzm, y, coef, elemt_args):
        self.dzm = dzm          # bf16 [N,H,W,C]: dZ already gated by the ReLU mask
        self.y = y              # bf16 [N,H,W,C]: the BN input
        self.coef = coef        # fp32 [3, Cp]: a | b | c
        self._args = elemt_args  # (P, mask, p, gamma, red, count, relu): to materialise

    @property
    def shape(self):
        return self.dzm.shape

    @property
    def device(self):
        return self.dzm.device

    @property
    def dtype(self):
        return self.dzm.dtype

    def record_stream(self, stream):
        self.dzm.record_stream(stream)
        self.y.record_stream(stream)
        self.coef.record_stream(stream)

    def materialize(self):
        """The dY tensor itself (debug checks, consumers that cannot fuse)."""
        P, mask, p, gamma, red, count, relu = self._args
        return P.bn_bwd_elemt(self.dzm, mask, self.y, p, gamma, red, count, relu)[0]


def is_lazy(t) -> bool:
    return isinstance(t, LazyDy)
