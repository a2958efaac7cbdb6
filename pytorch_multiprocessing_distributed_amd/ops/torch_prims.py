"""PyTorch reference implementations of every primitive the fused ops use.

Each function here has the exact contract of the matching gfx950 kernel in
``csrc/kernels`` (NHWC activations, channel = last dim, fp32 statistics).
They serve two roles:
  * the CPU backend (BASELINE config 1: ResNet-18 CIFAR on gloo), and
  * the fp32 oracle the GPU numerics tests compare each HIP kernel against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _f(x):
    """Upcast to the accumulation dtype: fp32, or fp64 for fp64 inputs (tests)."""
    return x if x.dtype == torch.float64 else x.float()


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


# --------------------------------------------------------------------- conv
def conv_weight(w, dtype, cin, want_t=True):
    """[K,C,R,S] param -> (wk,) with wk the [K,R,S,cin] compute copy
    (zero-padded channels).  The HIP backend also returns the dgrad image."""
    wk = w.detach().permute(0, 2, 3, 1).to(dtype)
    if cin != wk.shape[-1]:
        wk = F.pad(wk, (0, cin - wk.shape[-1]))
    return (wk.contiguous(),)


def stats_request(want_stats):
    """``want_stats``: False/True, or the BN statistics shift K (a [C] tensor; True = K 0).
    -> (want, shift or None)."""
    if torch.is_tensor(want_stats):
        return True, want_stats
    return bool(want_stats), None


def conv_fwd(x, wpack, stride, pad, want_stats):
    """y and, when requested, the BN statistics of the (rounded) output about the
    shift K: [sum (y-K), sum (y-K)^2] (csrc/kernels/common.h bn_moments)."""
    want, shift = stats_request(want_stats)
    wk = wpack[0]
    y = F.conv2d(_f(_nchw(x)), _f(wk.permute(0, 3, 1, 2)), stride=stride, padding=pad)
    y = _nhwc(y).to(x.dtype)
    stats = None
    if want:
        yf = _f(y).reshape(-1, y.shape[-1])
        if shift is not None:
            yf = yf - _f(shift)
        stats = torch.stack([yf.sum(0), (yf * yf).sum(0)])
    return y, stats


def conv_dgrad(dy, wpack, x_shape, stride, pad, addend=None, bnred=None, addend_mask=None, addend_bias=None):
    """dX (+ addend).  With ``bnred = (mask, [(y, params), ...])`` also returns
    the BN-backward reduce of the result for each set (the fused form of
    ``bn_bwd_reduce(dx, mask, y, params, relu=mask is not None)``)."""
    wk = wpack[0]
    n, h, w, c = x_shape
    dx = torch.nn.grad.conv2d_input((n, c, h, w), _f(wk.permute(0, 3, 1, 2)),
                                    _f(_nchw(dy)), stride=stride, padding=pad)
    dx = _nhwc(dx)
    if addend is not None:
        dx = dx + (_dzm(addend, addend_mask, True) if addend_mask is not None else _f(addend))
        if addend_bias is not None:
            dx = dx + _f(addend_bias)
    if bnred is None:
        return dx.to(dy.dtype)
    mask, sets = bnred
    # same contract as the gfx950 kernel: the output IS the BN site's dz, stored already
    # gated by that site's ReLU mask (its consumers then skip the mask)
    dx = (_dzm(dx, mask, True) if mask is not None else dx).to(dy.dtype)
    return dx, [bn_bwd_reduce(dx, mask, y, p, mask is not None) for y, p in sets]


def conv_wgrad(dy, x, wk_shape, stride, pad, out=None):
    """fp32 [K,R,S,C]; with ``out`` the gradient is accumulated into it."""
    k, r, s, c = wk_shape
    dw = torch.nn.grad.conv2d_weight(_f(_nchw(x)), (k, c, r, s), _f(_nchw(dy)),
                                     stride=stride, padding=pad)
    dw = dw.permute(0, 2, 3, 1)
    if out is not None:
        out.add_(dw.to(out.dtype))
        return out
    return dw.contiguous()          # fp32 [K,R,S,C]


# ----------------------------------------------------------------------- BN
# BN "params" are one fp32 [4, C] tensor: rows mean, invstd, scale=gamma*invstd,
# shift=beta-mean*scale (the same packing the HIP kernels use).
def bn_finalize(sums, count, gamma, beta, eps, running_mean=None, running_var=None,
                momentum=0.1, num_batches_tracked=None, shift=None):
    """Global (sum (y-K), sum (y-K)^2, count) -> params; updates running stats with
    the unbiased variance (torch batch_norm_gather_stats_with_counts semantics).
    ``count`` is a 1-element fp32 tensor so no host sync is needed.  ``shift`` = K
    (None: 0) is overwritten with the batch mean, the next step's shift."""
    cnt = _f(count)
    d = sums[0] / cnt
    mean = d if shift is None else _f(shift) + d
    var = (sums[1] / cnt - d * d).clamp_min(0.0)
    if shift is not None:
        shift.copy_(mean.to(shift.dtype))
    invstd = torch.rsqrt(var + eps)
    scale = _f(gamma.detach()) * invstd
    shift = _f(beta.detach()) - mean * scale
    if running_mean is not None:
        unbiased = var * (cnt / (cnt - 1.0).clamp_min(1.0))
        running_mean.mul_(1.0 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
        running_var.mul_(1.0 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
    if num_batches_tracked is not None:
        num_batches_tracked.add_(1)
    return torch.stack([mean, invstd, scale, shift])


def stats_finalize_local(stats, count, gamma, beta, eps, running_mean=None, running_var=None,
                         momentum=0.1, num_batches_tracked=None, shift=None):
    cnt = torch.full((1,), float(count), dtype=stats.dtype, device=stats.device)
    return bn_finalize(stats, cnt, gamma, beta, eps, running_mean, running_var, momentum,
                       num_batches_tracked, shift)


def bn_eval_params(running_mean, running_var, gamma, beta, eps):
    mean = _f(running_mean)
    invstd = torch.rsqrt(_f(running_var) + eps)
    scale = _f(gamma.detach()) * invstd
    shift = _f(beta.detach()) - mean * scale
    return torch.stack([mean, invstd, scale, shift])


def stats_collapse(a, b=None, count=None, acc_a=None, acc_b=None):
    """Per-channel stat blocks -> one flat buffer [2Ca (+2Cb) (+1 count)];
    ``acc_*`` = (d_beta, d_gamma) targets that receive += the sums."""
    for st, acc in ((a, acc_a), (b, acc_b)):
        if acc is not None and st is not None:
            for row, tgt in enumerate(acc):
                if tgt is not None:
                    tgt.add_(st[row].to(tgt.dtype))
    parts = [a.reshape(-1)]
    if b is not None:
        parts.append(b.reshape(-1))
    if count is not None:
        parts.append(torch.full((1,), float(count), dtype=a.dtype, device=a.device))
    return torch.cat(parts)


def bn_apply(y1, p1, res=None, y2=None, p2=None, relu=True):
    """-> (out, mask); mask = ReLU mask (bool, same shape) or None."""
    o = _f(y1) * p1[2] + p1[3]
    if y2 is not None:
        o = o + _f(y2) * p2[2] + p2[3]
    elif res is not None:
        o = o + _f(res)
    mask = None
    if relu:
        mask = o > 0
        o = o.clamp_min(0.0)
    return o.to(y1.dtype), mask


def _dzm(dout, mask, relu):
    d = _f(dout)
    if relu:
        d = d * mask
    return d


def bn_bwd_reduce(dout, mask, y, p, relu):
    """-> fp32 [2, C]: (sum dzm, sum dzm*xhat), dzm = dout * relu_mask.  ``y=None``: the
    sum-only form of the linear-BN backward, (sum dzm, -mean * invstd * sum dzm)."""
    c = dout.shape[-1]
    d = _dzm(dout, mask, relu).reshape(-1, c)
    if y is None:
        s = d.sum(0)
        return torch.stack([s, -(p[0] * p[1]) * s])
    xhat = (_f(y).reshape(-1, c) - p[0]) * p[1]
    return torch.stack([d.sum(0), (d * xhat).sum(0)])


# ------------------------------------------------- linear-BN backward (1x1 conv -> BN)
# y = z W^T (the 1x1 conv feeding the BN, W = its compute weight image), so dy never needs
# to be formed (ops/functional.py _bnlin_final):
#   dy = A dz + B y + Cc   =>   dz_in = dz (A W) + z (W^T B W) + Cc W     (dgrad, bias)
#                               dW    = A T + B (W Gz) + Cc (x) colsum(z), T = dz^T z, Gz = z^T z
def _w2(wk, c):
    return _f(wk).reshape(wk.shape[0], -1)[:, :c]


def bnlin_coeff(red, count, gamma, p, wk, c):
    """Global (sum dz, sum dz*xhat) -> (G [c,1,1,c]: image of W^T diag(B) W (symmetric: the
    dgrad image of the z G GEMM), bias [c] = Cc W (fp32), abc [3, K] fp32 = A, B, Cc)."""
    cnt = _f(count) if torch.is_tensor(count) else float(count)
    red = _f(red).reshape(2, -1)
    inv, mean = p[1], p[0]
    a = _f(gamma.detach()) * inv
    mdy, mdyx = red[0] / cnt, red[1] / cnt
    b = -a * inv * mdyx
    cc = a * (mean * inv * mdyx - mdy)
    w = _w2(wk, c)
    g = (w.t() @ (b[:, None] * w)).reshape(c, 1, 1, c).to(wk.dtype)
    return (g,), cc @ w, torch.stack([a, b, cc])      # G as a dgrad pack (this module reads wpack[0])


def bnlin_dimg(gamma, p, wk, c):
    """The dgrad weight pack of diag(gamma * invstd) W (forward quantities only)."""
    w = _w2(wk, c)
    a = _f(gamma.detach()) * p[1]
    return ((a[:, None] * w).reshape(w.shape[0], 1, 1, c).to(wk.dtype),)   # this module's dgrad reads wpack[0]


def colsum(x):
    """fp32 [C] column sums of an NHWC activation."""
    return _f(x).reshape(-1, x.shape[-1]).sum(0)


def bnlin_wgrad_(out, abc, T, wk, gz, cs):
    """out [K,1,1,C] (fp32, += ) = A T + B (W Gz) + Cc (x) colsum."""
    k = T.shape[0]
    t = _f(T).reshape(k, -1)
    c = t.shape[1]
    w = _w2(wk, c)
    g = _f(gz).reshape(c, c)
    dw = abc[0][:, None] * t + abc[1][:, None] * (w @ g) + abc[2][:, None] * _f(cs)[None, :]
    out.add_(dw.reshape(out.shape).to(out.dtype))


def bn_bwd_elemt(dout, mask, y, p, gamma, red, count, relu, want_dzm=False):
    d = _dzm(dout, mask, relu)
    xhat = (_f(y) - p[0]) * p[1]
    cnt = _f(count) if torch.is_tensor(count) else float(count)
    mdy = red[0] / cnt
    mdyx = red[1] / cnt
    dy = ((d - mdy - xhat * mdyx) * (_f(gamma.detach()) * p[1])).to(y.dtype)
    return dy, (d.to(y.dtype) if want_dzm else None)


def bn_bwd_elemt_eval(dout, mask, p, relu, want_dzm=False):
    d = _dzm(dout, mask, relu)
    dy = (d * p[2]).to(dout.dtype)
    return dy, (d.to(dout.dtype) if want_dzm else None)


# -------------------------------------------------------------------- pools
def maxpool_fwd(x):
    """3x3/s2/p1 max-pool; the auxiliary output is the input itself (the
    backward re-derives the routing so overlapping windows that pick the
    same element accumulate, which max_unpool2d would not)."""
    out = F.max_pool2d(_f(_nchw(x)), 3, 2, 1)
    return _nhwc(out).to(x.dtype), x


def maxpool_bwd(dout, x, x_shape):
    with torch.enable_grad():
        xf = _f(_nchw(x)).detach().requires_grad_(True)
        out = F.max_pool2d(xf, 3, 2, 1)
        (dx,) = torch.autograd.grad(out, xf, _f(_nchw(dout)))
    return _nhwc(dx).to(dout.dtype)


def stem_pool_fwd(y, p):
    """Composite reference of the fused stem tail: bn_apply(+ReLU) then max-pool.
    The auxiliary output carries (activation, ReLU mask) for the backward."""
    a, mask = bn_apply(y, p, relu=True)
    out, _ = maxpool_fwd(a)
    return out, (a, mask)


def stem_pool_bwd_reduce(dout, arg, y, p):
    a, mask = arg
    da = maxpool_bwd(dout, a, tuple(a.shape))
    return bn_bwd_reduce(da, mask, y, p, True)


def stem_pool_bwd_elemt(dout, arg, y, p, gamma, red, count, eval_mode=False):
    a, mask = arg
    da = maxpool_bwd(dout, a, tuple(a.shape))
    if eval_mode:
        return bn_bwd_elemt_eval(da, mask, p, True)[0]
    return bn_bwd_elemt(da, mask, y, p, gamma, red, count, True)[0]


def avgpool_fwd(x):
    return _f(x).mean(dim=(1, 2))


def avgpool_bwd(dout, x_shape, dtype):
    n, h, w, c = x_shape
    return (_f(dout) / (h * w)).reshape(n, 1, 1, c).expand(n, h, w, c).to(dtype).contiguous()


# ------------------------------------------------------------- classifier
def linear_fwd(x, w, b):
    return F.linear(_f(x), _f(w.detach()), None if b is None else _f(b.detach()))


def linear_dgrad(dout, w):
    return _f(dout) @ _f(w.detach())


def linear_wgrad(dout, x, dw, db, accumulate):
    g = _f(dout).t() @ _f(x)
    if accumulate:
        dw.add_(g.to(dw.dtype))
    else:
        dw.copy_(g)
    if db is not None:
        s = _f(dout).sum(0)
        if accumulate:
            db.add_(s.to(db.dtype))
        else:
            db.copy_(s)


# --------------------------------------------------------------- loss/acc
def xent_fwd(logits, target):
    """Mean softmax cross-entropy; returns (loss[1] fp32, lse[N] fp32)."""
    lf = _f(logits)
    lse = torch.logsumexp(lf, dim=1)
    loss = (lse - lf.gather(1, target.view(-1, 1)).squeeze(1)).mean()
    return loss.reshape(1), lse


def xent_bwd(gloss, logits, target, lse):
    lf = _f(logits)
    p = torch.exp(lf - lse[:, None])
    p[torch.arange(lf.shape[0], device=lf.device), target] -= 1.0
    return (p * (_f(gloss) / lf.shape[0])).to(logits.dtype)


def correct_count(logits, target):
    return (logits.argmax(1) == target).sum().to(torch.int64).reshape(1)


# -------------------------------------------------------------------- optim
def sgd_nesterov_(params, grads, bufs, lr, momentum, weight_decay, nesterov, first_step,
                  dampening=0.0, lr_dev=None):
    """In-place SGD over flat fp32 arenas (torch.optim.SGD semantics)."""
    if lr_dev is not None:
        lr = float(lr_dev.item())
    g = grads
    if weight_decay != 0:
        g = g.add(params, alpha=weight_decay)
    if momentum != 0:
        if first_step:
            bufs.copy_(g)
        else:
            bufs.mul_(momentum).add_(g, alpha=1.0 - dampening)
        g = g.add(bufs, alpha=momentum) if nesterov else bufs
    params.add_(g, alpha=-lr)
