"""gfx950 primitives: thin Python shims over the in-tree ``_C`` extension.

Same contracts as :mod:`.torch_prims` (NHWC bf16 activations, fp32
statistics, BN params packed [4, C]).  There is deliberately no fallback:
importing this module on a GPU box without the built extension raises.

Statistics buffers: conv epilogues and BN-backward reductions accumulate into
``[kStatSlots=64, 2, C]`` fp32 slot buffers (spreads atomics).  They come
from a small per-(device, C) pool of *already zeroed* buffers; the collapse
kernels read-and-clear them, after which they go back to the pool -- so the
hot loop issues no memset launches for statistics.  All of this is ordered by
the current HIP stream.
"""
from __future__ import annotations

import torch

from . import torch_prims as _TP
from .native import C as _C

SLOTS = 64
_POOL: dict = {}


def _acquire(c, dev):
    lst = _POOL.get((dev, c))
    if lst:
        return lst.pop()
    return torch.zeros(SLOTS, 2, c, dtype=torch.float32, device=dev)


def _release(*bufs):
    for b in bufs:
        if b is not None:
            _POOL.setdefault((b.device, b.shape[-1]), []).append(b)


SUPPORTS_FP8 = True


# ---------------------------------------------------------------------- fp8
def quant_bf16_fp8(x, scale, amax):
    return _C.quant_bf16_fp8(x, scale, amax)


def quant_weight_fp8(w, cin, scale, amax):
    return _C.quant_weight_fp8(w.detach(), int(cin), scale, amax)


def conv_fp8_fwd(xq, wq, sx, sw, stride, pad, want_stats):
    want, shift = _TP.stats_request(want_stats)
    if want:
        buf = _acquire(wq.shape[0], xq.device)
        y, st = _C.conv_fp8_fwd(xq, wq, sx, sw, int(stride), int(pad), True, buf, shift)
        return y, st
    return _C.conv_fp8_fwd(xq, wq, sx, sw, int(stride), int(pad), False, None)[0], None


# --------------------------------------------------------------------- conv
def conv_weight(w, dtype, cin, want_t=True):
    if dtype != torch.bfloat16:
        raise TypeError(f"gfx950 conv path computes in bf16, got activations of {dtype}")
    return tuple(_C.conv_weight_prep(w.detach(), int(cin), bool(want_t)))


def conv_fwd(x, wpack, stride, pad, want_stats):
    """``want_stats``: False, True, or the BN statistics shift (fp32 [K], see
    torch_prims.conv_fwd): the slots then hold sums about that shift."""
    want, shift = _TP.stats_request(want_stats)
    if want:
        buf = _acquire(wpack[0].shape[0], x.device)
        y, st = _C.conv_fwd(x, wpack[0], int(stride), int(pad), True, buf, shift)
        return y, st
    return _C.conv_fwd(x, wpack[0], int(stride), int(pad), False, None)[0], None


def conv_dgrad(dy, wpack, x_shape, stride, pad, addend=None, bnred=None, addend_mask=None, addend_bias=None):
    """dX (+ addend [* relu bitmask addend_mask]).  ``bnred = (mask, [(y, params)] or
    [(y1, p1), (y2, p2)])`` fuses the BN-backward reduce of dX into the epilogue
    and returns ``(dx, [slot buffers])`` (same contract as :func:`bn_bwd_reduce`)."""
    if len(wpack) < 2:
        raise RuntimeError("dgrad image was not prepared (input did not require grad)")
    if bnred is None:
        return _C.conv_dgrad(dy, wpack[1], int(x_shape[1]), int(x_shape[2]), int(stride), int(pad),
                             addend, None, None, None, None, None, None, None, addend_mask, addend_bias)
    mask, sets = bnred
    # a set's y may be None (sum-only reduce of the linear-BN backward): size from the params
    bufs = [_acquire(p.shape[-1], dy.device) for _, p in sets]
    (y0, p0), (y1, p1) = sets[0], (sets[1] if len(sets) > 1 else (None, None))
    dx = _C.conv_dgrad(dy, wpack[1], int(x_shape[1]), int(x_shape[2]), int(stride), int(pad),
                       addend, mask, y0, p0, bufs[0], y1, p1, bufs[1] if len(bufs) > 1 else None,
                       addend_mask, addend_bias)
    return dx, bufs


def conv_dgrad_fp8(dyq, sdy, wtq, sw, x_shape, stride, pad, addend=None, bnred=None, addend_mask=None):
    """dX (bf16) of e5m2 dY (scale sdy) x the e4m3 transposed weight image ``wtq``
    [Cp,R,S,K] (scale sw), with :func:`conv_dgrad`'s epilogue options."""
    if bnred is None:
        return _C.conv_dgrad_fp8(dyq, wtq, sdy, sw, int(x_shape[1]), int(x_shape[2]), int(stride), int(pad),
                                 addend, addend_mask=addend_mask)
    mask, sets = bnred
    bufs = [_acquire(p.shape[-1], dyq.device) for _, p in sets]
    (y0, p0), (y1, p1) = sets[0], (sets[1] if len(sets) > 1 else (None, None))
    dx = _C.conv_dgrad_fp8(dyq, wtq, sdy, sw, int(x_shape[1]), int(x_shape[2]), int(stride), int(pad),
                           addend, mask, y0, p0, bufs[0], y1, p1, bufs[1] if len(bufs) > 1 else None,
                           addend_mask)
    return dx, bufs


def conv_wgrad_fp8(dyq, sdy, xq, sx, wk_shape, stride, pad, out=None):
    """dW of e5m2 dY (scale sdy) x e4m3 X (scale sx), ADDED to ``out`` ([K,R,S,C])."""
    return _C.conv_wgrad_fp8(dyq, xq, sdy, sx, int(wk_shape[1]), int(wk_shape[2]), int(stride), int(pad), out)


def conv_wgrad(dy, x, wk_shape, stride, pad, out=None):
    """fp32 [K,R,S,C]; with ``out`` the gradient is accumulated into it."""
    return _C.conv_wgrad(dy, x, int(wk_shape[1]), int(wk_shape[2]), int(stride), int(pad), out)


# ----------------------------------------------------------------------- BN
def bn_finalize(sums, count, gamma, beta, eps, running_mean=None, running_var=None,
                momentum=0.1, num_batches_tracked=None, shift=None):
    return _C.bn_finalize(sums, count, gamma.detach(), beta.detach(), float(eps), running_mean,
                          running_var, float(momentum), num_batches_tracked, False, shift)


def stats_finalize_local(slots, count, gamma, beta, eps, running_mean=None, running_var=None,
                         momentum=0.1, num_batches_tracked=None, shift=None):
    p = _C.stats_finalize_local(slots, float(count), gamma.detach(), beta.detach(), float(eps),
                                running_mean, running_var, float(momentum), num_batches_tracked, shift)
    _release(slots)
    return p


def bn_eval_params(running_mean, running_var, gamma, beta, eps):
    return _C.bn_finalize(None, None, gamma.detach(), beta.detach(), float(eps), running_mean,
                          running_var, 0.0, None, True)


def stats_collapse(a, b=None, count=None, acc_a=None, acc_b=None):
    """[S,2,Ca] (+[S,2,Cb]) slot statistics -> flat [2Ca (+2Cb) (+1 count)];
    the slot buffers are cleared and recycled.  ``acc_*`` = (d_beta, d_gamma)
    fp32 targets that receive += the local sums."""
    aa = acc_a or (None, None)
    ab = acc_b or (None, None)
    out = _C.stats_collapse(a, b, None if count is None else float(count), True,
                            aa[0], aa[1], ab[0], ab[1])
    _release(a, b)
    return out


def bn_apply(y1, p1, res=None, y2=None, p2=None, relu=True, fp8=None, fp8_only=False):
    """-> (out, mask): mask is the ReLU bitmask (uint8 per 8-channel chunk) the
    backward reads instead of re-reading ``out`` (1/16 of the bytes).
    ``fp8=(scale, amax)`` -> (out, mask, q): q is an e4m3 copy of out * scale;
    ``fp8_only``: q is the only activation written (out is None)."""
    if fp8 is not None:
        r = _C.bn_apply(y1, p1, res, y2, p2, True, True, fp8[0], fp8[1], bool(fp8_only))
        return r[0], r[1], r[2]
    r = _C.bn_apply(y1, p1, res, y2, p2, bool(relu), True, None, None)
    return (r[0], r[1]) if relu else (r[0], None)


def bn_bwd_reduce(dout, mask, y, p, relu):
    buf = _acquire(y.shape[-1], y.device)
    return _C.bn_bwd_reduce(dout, mask, y, p, bool(relu), buf)


# ------------------------------------------------- linear-BN backward (torch_prims notes)
def bnlin_coeff(red, count, gamma, p, wk, c):
    cnt_t = count if torch.is_tensor(count) else None
    r = _C.bnlin_coeff(red, cnt_t, 0.0 if cnt_t is not None else float(count), gamma.detach(), p, wk, int(c))
    return (None, r[0]), r[1], r[2]          # G as a dgrad pack (the kernel reads wpack[1]), bias, abc


def bnlin_dimg(gamma, p, wk, c):
    return (wk, _C.bnlin_dimg(gamma.detach(), p, wk, int(c)))   # dgrad pack: (forward image, scaled image)


def colsum(x):
    return _C.colsum(x)


def bnlin_wgrad_(out, abc, T, wk, gz, cs):
    _C.bnlin_wgrad(out, abc, T, wk, gz, cs)


def bn_bwd_elemt(dout, mask, y, p, gamma, red, count, relu, want_dzm=False, q8=None, q8_only=False):
    """-> (dy, dzm).  ``q8=(scale, amax)``: dy also gets an e5m2 copy (dy * scale) for the
    fp8 weight / data gradients, attached as ``dy._pmd_q8 = (dyq, scale)``; with
    ``q8_only`` the e5m2 copy is the only one written and is itself returned as dy."""
    qs, qa = (q8[0], q8[1]) if q8 is not None else (None, None)
    if torch.is_tensor(count):
        r = _C.bn_bwd_elemt(dout, mask, y, p, gamma.detach(), red, count, 0.0, bool(relu),
                            bool(want_dzm), False, qs, qa, bool(q8_only))
    else:
        r = _C.bn_bwd_elemt(dout, mask, y, p, gamma.detach(), red, None, float(count), bool(relu),
                            bool(want_dzm), False, qs, qa, bool(q8_only))
    if q8 is not None:
        d = r[1] if q8_only else r[0]
        d._pmd_q8 = (r[1], q8[0])
        return d, None
    return (r[0], r[1]) if want_dzm else (r[0], None)


def bn_bwd_elemt_eval(dout, mask, p, relu, want_dzm=False):
    r = _C.bn_bwd_elemt(dout, mask, dout, p, p[2], None, None, 1.0, bool(relu), bool(want_dzm),
                        True)
    return (r[0], r[1]) if want_dzm else (r[0], None)


# -------------------------------------------------------------------- pools
def maxpool_fwd(x):
    out, arg = _C.maxpool_fwd(x)
    return out, arg


def maxpool_bwd(dout, arg, x_shape):
    return _C.maxpool_bwd(dout, arg, int(x_shape[1]), int(x_shape[2]))


def stem_pool_fwd(y, p):
    """BN + ReLU + 3x3/s2 max-pool of the conv1 output in one pass -> (out, argmax taps)."""
    return tuple(_C.stem_pool_fwd(y, p))


def stem_pool_bwd_reduce(dout, arg, y, p):
    buf = _acquire(y.shape[-1], y.device)
    return _C.stem_pool_bwd_reduce(dout, arg, y, p, buf)


def stem_pool_bwd_elemt(dout, arg, y, p, gamma, red, count, eval_mode=False):
    if torch.is_tensor(count):
        return _C.stem_pool_bwd_elemt(dout, arg, y, p, gamma.detach(), red, count, 0.0, bool(eval_mode))
    return _C.stem_pool_bwd_elemt(dout, arg, y, p, gamma.detach(), red, None,
                                  float(count or 1.0), bool(eval_mode))


def stem_wgrad_fused(dout, arg, y, p, gamma, red, count, xs, pad):
    """Stem conv weight gradient (s2d image, fp32 [64,4,4,16]) with the stem's max-pool + BN
    backward elementwise pass inside the kernel; None when the geometry is outside its plan."""
    if torch.is_tensor(count):
        r = _C.stem_wgrad_fused(dout, arg, y, p, gamma.detach(), red, count, 0.0, xs, int(pad))
    else:
        r = _C.stem_wgrad_fused(dout, arg, y, p, gamma.detach(), red, None, float(count or 1.0), xs, int(pad))
    return r if r is not None and r.numel() > 0 else None


def avgpool_fwd(x):
    return _C.avgpool_fwd(x)


def avgpool_bwd(dout, x_shape, dtype):
    return _C.avgpool_bwd(dout.float().contiguous(), int(x_shape[1]), int(x_shape[2]))


# ------------------------------------------------------------- classifier
def linear_fwd(x, w, b):
    return _C.linear_fwd(x.float().contiguous(), w.detach(), None if b is None else b.detach())


def linear_dgrad(dout, w):
    return _C.linear_dgrad(dout.contiguous(), w.detach())


def linear_wgrad(dout, x, dw, db, accumulate):
    """dw (+)= dout^T x, db (+)= column sums of dout, into the given fp32 targets."""
    _C.linear_wgrad(dout.contiguous(), x.contiguous(), dw, db, bool(accumulate))


# --------------------------------------------------------------- loss/acc
def xent_fwd(logits, target):
    loss, lse, _ = _C.xent_fwd(logits.float().contiguous(), target)
    return loss, lse


def xent_bwd(gloss, logits, target, lse):
    g = _C.xent_bwd(logits.float().contiguous(), target, lse, gloss)
    return g.to(logits.dtype)


def correct_count(logits, target):
    return _C.xent_fwd(logits.float().contiguous(), target)[2]


# -------------------------------------------------------------------- optim
def sgd_nesterov_(params, grads, bufs, lr, momentum, weight_decay, nesterov, first_step,
                  dampening=0.0, lr_dev=None):
    _C.sgd_(params, grads, bufs, float(lr), float(momentum), float(weight_decay),
            float(dampening), bool(nesterov), bool(first_step), lr_dev)


# ------------------------------------------------------------------- debug
def _install_sync_debug():
    from ..utils.trace import sync_debug_enabled, wrap_sync_debug
    if sync_debug_enabled():
        names = [n for n, v in globals().items()
                 if callable(v) and not n.startswith("_") and getattr(v, "__module__", "") == __name__]
        wrap_sync_debug(globals(), names)


_install_sync_debug()
