"""Winograd F(2x2, 3x3) convolution for the stride-1, pad-1
3x3 layers of the reference's blocks (BasicBlock conv1/conv2 at stride 1,
Bottleneck conv2 at stride 1: model/resnet.py:20-24, 50-51).

GPU path: three gfx950 transform kernels (csrc/kernels/winograd.hip) around the
16 per-position GEMMs, each run as a 1x1 convolution on the framework's
implicit-GEMM MFMA kernel (``C.winograd_gemm``; no library GEMM):

    U  = winograd_filter(wk)            [16, K, C]   (G g G^T)
    V  = winograd_input(x)              [16, T, C]   (B^T d B), T = N ceil(H/2) ceil(W/2)
    M  = winograd_gemm(V, U)            [16, T, K]   M[b] = V[b] U[b]^T
    y  = winograd_output(M)             [N, H, W, K] (A^T M A) + fused BN statistics

Dgrad of the same layer is the same pipeline on dY with the flipped,
channel-transposed filter (explicit API, :func:`conv_dgrad`): the unfused pipeline moves
the transformed operands (4x the activation bytes) through HBM and loses to the implicit
GEMM on every ResNet-50 layer (profiles/winograd_r02_native_gemm.txt,
profiles/pmc_winograd_r03.txt).

The FUSED forward (:func:`conv_fwd_fused`, ``winograd_fused_fwd_kernel``) keeps V and M on
the CU: per block the input transform of 32 tiles x 64 channels goes into LDS, 4 waves run
the 16 transformed-domain GEMMs on v_mfma_f32_16x16x32_bf16 (4 positions each), and the
output transform + BN-statistics epilogue read the accumulators back through LDS.  It is
candidate 14 of the conv autotuner (kernels/conv_igemm.hip: the filter transform + the fused
kernel, timed against the implicit-GEMM tiles on the live operands), so the tuning tables
adopt it for exactly the stride-1 3x3 shapes where it wins (profiles/winograd_fused_r06.txt).

``conv_ref`` is the same algorithm in plain torch fp32 -- the CPU numerics
reference of the transforms (tests/test_winograd_cpu.py).
"""
from __future__ import annotations

import torch

BT = torch.tensor([[1., 0., -1., 0.], [0., 1., 1., 0.], [0., -1., 1., 0.], [0., 1., 0., -1.]])
G = torch.tensor([[1., 0., 0.], [.5, .5, .5], [.5, -.5, .5], [0., 0., 1.]])
AT = torch.tensor([[1., 1., 1., 0.], [0., 1., -1., -1.]])


def eligible(wk_shape, stride, pad, cin=None) -> bool:
    """Stride-1 pad-1 3x3 with power-of-two channel chunk counts (kernel grid contract)."""
    K, R, S, C = wk_shape
    if cin is not None and cin != C:
        return False

    def p2(c):
        c8 = c // 8
        return c % 8 == 0 and 0 < c8 <= 256 and (c8 & (c8 - 1)) == 0
    return R == 3 and S == 3 and int(stride) == 1 and int(pad) == 1 and p2(K) and p2(C)


# ------------------------------------------------------------------ reference
def conv_ref(x, wk, flip=False):
    """fp32 Winograd F(2x2,3x3) on NHWC ``x`` with weight image ``wk`` [K,3,3,C]
    (``flip``: the dgrad filter, i.e. ``x`` is dY [N,H,W,K] and the result dX)."""
    xf = x.float()
    g = wk.float()
    if flip:                       # g'[c][r][s][k] = wk[k][2-r][2-s][c]
        g = g.flip(1, 2).permute(3, 1, 2, 0)
    N, H, W, C = xf.shape
    K = g.shape[0]
    TH, TW = (H + 1) // 2, (W + 1) // 2
    # zero-pad to 2*T + 2 rows/cols: rows 2 th - 1 .. 2 th + 2
    xp = torch.zeros(N, 2 * TH + 2, 2 * TW + 2, C)
    xp[:, 1:H + 1, 1:W + 1] = xf
    d = xp.unfold(1, 4, 2).unfold(2, 4, 2)             # [N, TH, TW, C, 4, 4]
    V = torch.einsum("ia,ntwcab,jb->ntwcij", BT, d, BT)  # B^T d B
    U = torch.einsum("ir,kcrs,js->kcij", G, g.permute(0, 3, 1, 2), G)  # G g G^T
    M = torch.einsum("ntwcij,kcij->ntwkij", V, U)
    Y = torch.einsum("ai,ntwkij,bj->ntwkab", AT, M, AT)  # [N, TH, TW, K, 2, 2]
    y = Y.permute(0, 1, 4, 2, 5, 3).reshape(N, 2 * TH, 2 * TW, K)
    return y[:, :H, :W].contiguous()


# ------------------------------------------------------------------ gfx950 path
def _c():
    from .native import C
    return C


def conv_fwd(x, wk, want_stats, stats_buf=None, shift=None):
    """Forward (+ conv_fwd-compatible [slots,2,K] statistics about ``shift``) on the
    gfx950 transforms."""
    C = _c()
    U = C.winograd_filter(wk, False)                 # [16, K, C]
    V = C.winograd_input(x)                          # [16, T, C]
    M = C.winograd_gemm(V, U)                        # [16, T, K]  MFMA igemm
    N, H, W, _ = x.shape
    out = C.winograd_output(M, N, H, W, bool(want_stats), stats_buf, shift)
    return (out[0], out[1]) if want_stats else (out[0], None)


def conv_dgrad(dy, wk, x_shape):
    """dX of a stride-1 pad-1 3x3 conv = the Winograd forward of dY with the flipped filter."""
    C = _c()
    U = C.winograd_filter(wk, True)                  # [16, Cp, K]
    V = C.winograd_input(dy)                         # [16, T, K]
    M = C.winograd_gemm(V, U)                        # [16, T, Cp]
    N, H, W, _ = x_shape
    return C.winograd_output(M, N, H, W, False, None)[0]


def fused_eligible(wk_shape, stride, pad) -> bool:
    """The fused forward's contract: stride-1 pad-1 3x3 with C % 64 == 0 and K % 64 == 0."""
    K, R, S, C = wk_shape
    return R == 3 and S == 3 and int(stride) == 1 and int(pad) == 1 and C % 64 == 0 and K % 64 == 0


def conv_fwd_fused(x, wk, want_stats, stats_buf=None, shift=None):
    """Forward (+ conv_fwd-compatible [slots,2,K] statistics about ``shift``) in ONE fused
    kernel after the filter transform."""
    C = _c()
    U = C.winograd_filter(wk, False)                 # [16, K, C]
    out = C.winograd_fused_fwd(x, U, bool(want_stats), stats_buf, shift)
    return (out[0], out[1]) if want_stats else (out[0], None)

