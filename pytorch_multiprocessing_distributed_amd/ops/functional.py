"""Fused, autograd-aware ResNet ops over NHWC activations.

Every op is a ``torch.autograd.Function`` whose forward/backward are written
in terms of *primitives* (:mod:`.torch_prims` on CPU, :mod:`.hip_prims` =
hand-written gfx950 kernels on an MI355X).  The op graph is what the
reference gets from ``nn.Conv2d`` + ``nn.SyncBatchNorm`` + ``F.relu`` +
in-place residual add (reference model/resnet.py:35-39, 65-70; main.py:43),
re-cut so that memory-bound work is fused:

  conv            -> implicit-GEMM conv whose epilogue also emits the
                     per-channel (sum, sum^2) BN statistics
  bn_add_act      -> [SyncBN all-reduce of the statistics] -> finalize
                     (+ running-stat update) -> one elementwise pass that
                     normalises, adds the (optionally BN'd) residual and ReLUs
  backward        -> one reduce pass (sum dz, sum dz*xhat) -> [SyncBN
                     all-reduce] -> one elementwise pass

SyncBN semantics follow torch.nn.SyncBatchNorm (torch:nn/modules/
_functions.py:39-207): global statistics in forward, globally reduced
``sum_dy``/``sum_dy_xmu`` in backward, *local* gamma/beta gradients (DDP
averages them).  Unlike torch there is no device->host sync.
"""
from __future__ import annotations

import os

import torch

from . import torch_prims

_state = {"bn_sync": None, "force_torch": os.environ.get("PMD_PRIMS", "") == "torch"}


def set_bn_sync(comm):
    """Install the communicator used for SyncBN statistics (None = local BN)."""
    _state["bn_sync"] = comm


def get_bn_sync():
    return _state["bn_sync"]


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


# ---------------------------------------------------------------------- conv
class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pad, want_stats):
        P = prims_for(x)
        wpack = P.conv_weight(w, x.dtype, x.shape[-1], x.requires_grad)
        y, stats = P.conv_fwd(x, wpack, stride, pad, want_stats)
        ctx.save_for_backward(x, *wpack)
        ctx.conf = (stride, pad, tuple(w.shape))
        if stats is None:
            stats = _empty(x.device)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, *wpack = ctx.saved_tensors
        stride, pad, wshape = ctx.conf
        P = prims_for(x)
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = P.conv_dgrad(dy, wpack, tuple(x.shape), stride, pad)
        if ctx.needs_input_grad[1]:
            dwk = P.conv_wgrad(dy, x, tuple(wpack[0].shape), stride, pad)   # fp32 [K,R,S,Cx]
            c = wshape[1]
            if dwk.shape[-1] != c:
                dwk = dwk[..., :c].contiguous()
            dw = dwk.permute(0, 3, 1, 2)          # [K,C,R,S], channels_last strides
        return dx, dw, None, None, None


def conv(x, conv_mod, want_stats=None):
    """Returns ``(y, stats)``; ``stats`` = fp32 [2, K] (sum, sum^2) of y."""
    if want_stats is None:
        want_stats = torch.is_grad_enabled() or conv_mod.training
    return _ConvFn.apply(x, conv_mod.weight, conv_mod.stride, conv_mod.padding, bool(want_stats))


# ------------------------------------------------------------------------ BN
class _BNActFn(torch.autograd.Function):
    """out = act( BN1(y1) + [BN2(y2) | res | 0] )."""

    @staticmethod
    def forward(ctx, cfg, y1, s1, g1, b1, res, y2, s2, g2, b2):
        bn1, bn2, relu, training = cfg
        P = prims_for(y1)
        sync = _state["bn_sync"] if training else None
        c1 = y1.shape[-1]
        m_local = y1.numel() // c1
        two = y2 is not None
        if training:
            # local (sum, sum^2) of both branches + element count in ONE buffer
            # -> one all-reduce per BN site (both BNs of a projection block share it)
            buf = P.stats_collapse(s1, s2 if two else None, float(m_local))
            if sync is not None:
                sync.all_reduce_(buf)
            count = buf[-1:]
            gs1 = buf[: 2 * c1].view(2, c1)
            p1 = P.bn_finalize(gs1, count, g1, b1, bn1.eps, bn1.running_mean, bn1.running_var,
                               bn1.momentum, bn1.num_batches_tracked)
            if two:
                c2 = y2.shape[-1]
                gs2 = buf[2 * c1: 2 * c1 + 2 * c2].view(2, c2)
                p2 = P.bn_finalize(gs2, count, g2, b2, bn2.eps, bn2.running_mean,
                                   bn2.running_var, bn2.momentum, bn2.num_batches_tracked)
        else:
            count = None
            p1 = P.bn_eval_params(bn1.running_mean, bn1.running_var, g1, b1, bn1.eps)
            if two:
                p2 = P.bn_eval_params(bn2.running_mean, bn2.running_var, g2, b2, bn2.eps)
        out = P.bn_apply(y1, p1, res, y2, p2 if two else None, relu)
        ctx.cfg = (relu, training, two, res is not None, sync)
        saved = [y1, out, p1, g1]
        if two:
            saved += [y2, p2, g2]
        if count is not None:
            saved.append(count)
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        relu, training, two, has_res, sync = ctx.cfg
        sv = list(ctx.saved_tensors)
        y1, out, p1, g1 = sv[:4]
        if two:
            y2, p2, g2 = sv[4:7]
        count = sv[-1] if training else None
        P = prims_for(y1)
        dout = dout.contiguous()
        d_y1 = d_g1 = d_b1 = d_res = d_y2 = d_g2 = d_b2 = None
        r1 = P.bn_bwd_reduce(dout, out, y1, p1, relu)
        r2 = P.bn_bwd_reduce(dout, out, y2, p2, relu) if two else None
        red = P.stats_collapse(r1, r2, None)            # flat [2C1 (+2C2)], local sums
        c1 = y1.shape[-1]
        # gamma/beta grads use the LOCAL sums (DDP averages them), like torch SyncBN
        d_b1, d_g1 = red[:c1], red[c1:2 * c1]
        if two:
            c2 = y2.shape[-1]
            d_b2, d_g2 = red[2 * c1:2 * c1 + c2], red[2 * c1 + c2:]
        if training:
            if sync is not None:
                red = red.clone()
                sync.all_reduce_(red)
            red1 = red[:2 * c1].view(2, c1)
            red2 = red[2 * c1:].view(2, -1) if two else None
            d_y1, dzm = P.bn_bwd_elemt(dout, out, y1, p1, g1, red1, count, relu,
                                       want_dzm=has_res)
            if two:
                d_y2, _ = P.bn_bwd_elemt(dout, out, y2, p2, g2, red2, count, relu)
        else:
            d_y1, dzm = P.bn_bwd_elemt_eval(dout, out, p1, relu, want_dzm=has_res)
            if two:
                d_y2, _ = P.bn_bwd_elemt_eval(dout, out, p2, relu)
        if has_res:
            d_res = dzm
        return None, d_y1, None, d_g1, d_b1, d_res, d_y2, None, d_g2, d_b2


def bn_add_act(y, stats, bn, residual=None, res_y=None, res_stats=None, res_bn=None, relu=True):
    training = bn.training
    cfg = (bn, res_bn, relu, training)
    if res_y is not None:
        return _BNActFn.apply(cfg, y, stats, bn.weight, bn.bias, None,
                              res_y, res_stats, res_bn.weight, res_bn.bias)
    return _BNActFn.apply(cfg, y, stats, bn.weight, bn.bias, residual, None, None, None, None)


def conv_bn_act(x, conv_mod, bn, relu=True):
    y, s = conv(x, conv_mod, want_stats=bn.training)
    return bn_add_act(y, s, bn, relu=relu)


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
        ctx.is_cuda = x.is_cuda
        return prims_for(x).avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dout):
        return prims_for(dout).avgpool_bwd(dout.contiguous(), ctx.xshape, ctx.dtype)


def global_avg_pool(x):
    """[N,H,W,C] -> [N,C] fp32."""
    return _AvgPoolFn.apply(x)


def linear(x, lin):
    return torch.nn.functional.linear(x, lin.weight, lin.bias)


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
        return P.xent_bwd(gloss.reshape(1).float(), logits, target, lse), None


def cross_entropy(logits, target):
    """Mean softmax cross-entropy (== nn.CrossEntropyLoss(), reference main.py:48)."""
    return _XentFn.apply(logits, target)


def correct_count(logits, target):
    """Device-side top-1 correct count (int64 [1]); no host sync."""
    return prims_for(logits).correct_count(logits, target)
