// Fused ImageNet stem tail: BatchNorm + ReLU + 3x3/s2 max-pool in ONE pass
// forward, and max-pool backward + BatchNorm(+ReLU) backward in two passes
// (reduce, elementwise) -- the [N,112,112,64] stem activation is never
// materialised (forward: it was written by bn_apply and re-read by the pool;
// backward: the pool gradient was written and re-read twice by the BN
// backward).  Same arithmetic and tie-breaking as the composite path
// (bn_apply -> maxpool_fwd; maxpool_bwd -> bn_bwd_reduce -> bn_bwd_elemt):
//   a = bf16(relu(y*scale + shift)), window max = first strictly greater a,
//   ReLU mask bit = (y*scale + shift > 0), pool gradient rounded to bf16.
// Reference: model/resnet.py:97 (conv -> SyncBN -> relu) followed by the
// ImageNet max-pool this framework adds for 224x224 inputs.
#include "common.h"
#include "stem_tile.h"

namespace pmd {

__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// y [N,H,W,C] bf16 (conv output), params [4][C] (mean, invstd, scale, shift)
// -> out [N,P,Q,C] bf16, arg [N,P,Q,C] uint8 tap (0..8) of the window max.
// grid.y = output row (n, p); x covers Q * C/8 chunks.
__global__ __launch_bounds__(256) void stem_pool_fwd_kernel(const bf16_t* __restrict__ y,
                                                            const float* __restrict__ params,
                                                            bf16_t* __restrict__ out,
                                                            uint8_t* __restrict__ arg, int H, int W,
                                                            int C, int P, int Q, int log2C8) {
  const int C8 = C >> 3;
  const int row = blockIdx.y;
  const int n = row / P, p = row - (row / P) * P;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Q * C8) return;
  const int q = j >> log2C8, cc = j & (C8 - 1);
  float sc[8], sh[8];
  ld8(params + 2 * C + cc * 8, sc);
  ld8(params + 3 * C + cc * 8, sh);
  float best[8];
  int bi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    best[k] = -INFINITY;
    bi[k] = 0;
  }
  const bf16_t* yb = y + (size_t)n * H * W * C + cc * 8;
  // branch-free taps: out-of-range taps load a clamped (valid) pixel and are
  // masked out, so all 9 loads are independent and can be in flight together
  uint4 raw[9];
  bool ok[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ih = p * 2 - 1 + t / 3, iw = q * 2 - 1 + t % 3;
    ok[t] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    const int ch = min(max(ih, 0), H - 1), cw = min(max(iw, 0), W - 1);
    raw[t] = ld16n<NT_STEM>(yb + ((size_t)ch * W + cw) * C);
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    float v[8];
    unpack8(raw[t], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = round_bf(fmaxf(v[k] * sc[k] + sh[k], 0.f));
      if (ok[t] && a > best[k]) {
        best[k] = a;
        bi[k] = t;
      }
    }
  }
  const size_t o = (size_t)row * Q * C8 + j;
  reinterpret_cast<uint4*>(out)[o] = pack8(best);
  uint2 packed;
  packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
  packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
  reinterpret_cast<uint2*>(arg)[o] = packed;
}

// Pass 1: per-channel sum(dz), sum(dz * xhat) into kStatSlots slot copies.
// Dynamic LDS: 2*Q*C*2 B pooled gradient + 2*Q*C B taps; the 256x17 partials
// reuse the same bytes after the compute loop.
__global__ __launch_bounds__(256) void stem_pool_bwd_reduce_kernel(
    const bf16_t* __restrict__ dout, const uint8_t* __restrict__ arg, const bf16_t* __restrict__ y,
    const float* __restrict__ params, float* __restrict__ red, int N, int H, int W, int C, int P, int Q,
    int log2C8, int nslots) {
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_lds[];
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int cc = tid & (C8 - 1);
  const int n = blockIdx.x / P, p = blockIdx.x - n * P;
  bf16_t* dl = reinterpret_cast<bf16_t*>(stem_lds);
  uint8_t* al = stem_lds + (size_t)2 * Q * C * 2;
  stem_stage_pooled(dout, arg, dl, al, n, p, P, Q, C8);
  float mean[8], inv[8], sc[8], sh[8];
  ld8(params + cc * 8, mean);
  ld8(params + C + cc * 8, inv);
  ld8(params + 2 * C + cc * 8, sc);
  ld8(params + 3 * C + cc * 8, sh);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
  __syncthreads();
  const StemBwdTile t{dl, al, p, P, Q, C8};
  const int per_row = W * C8;
  const int h0 = 2 * p, nrow = min(2, H - h0);
  for (int j = tid; j < nrow * per_row; j += 256) {
    const int r = j >= per_row ? 1 : 0;
    const int jj = j - r * per_row;
    const int h = h0 + r, w = jj >> log2C8;
    float v[8], d[8];
    unpack8(ld16n<NT_STEM>(reinterpret_cast<const uint4*>(y) + (((size_t)n * H + h) * per_row + jj)), v);
    t.dz(h, w, cc, v, sc, sh, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s1[k] += d[k];
      s2[k] += d[k] * (v[k] - mean[k]);  // * invstd once, below
    }
  }
  __syncthreads();  // the staged pooled rows are dead: the partials reuse the LDS
  float* part = reinterpret_cast<float*>(stem_lds);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    part[tid * 17 + k] = s1[k];
    part[tid * 17 + 8 + k] = s2[k] * inv[k];
  }
  __syncthreads();
  for (int e = tid; e < C8 * 16; e += 256) {
    const int col = e >> 4, k = e & 15;
    float a = 0.f;
    for (int r = col; r < 256; r += C8) a += part[r * 17 + k];
    float* slot = red + stat_slot(blockIdx.x, nslots) * 2 * C;
    atomicAdd(slot + (k < 8 ? 0 : C) + col * 8 + (k & 7), a);
  }
}

// Pass 2: dy = a*dz + b*y + c with the globally reduced sums (train), or
// dy = scale*dz (eval: running statistics, no batch dependence).
template <bool EVAL>
__global__ __launch_bounds__(256) void stem_pool_bwd_elemt_kernel(
    const bf16_t* __restrict__ dout, const uint8_t* __restrict__ arg, const bf16_t* __restrict__ y,
    const float* __restrict__ params, const float* __restrict__ gamma, const float* __restrict__ red,
    const float* __restrict__ count, float count_h, bf16_t* __restrict__ dy, int N, int H, int W, int C,
    int P, int Q, int log2C8) {
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_lds[];
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int cc = tid & (C8 - 1);
  const int c0 = cc * 8;
  const int n = blockIdx.x / P, p = blockIdx.x - n * P;
  bf16_t* dl = reinterpret_cast<bf16_t*>(stem_lds);
  uint8_t* al = stem_lds + (size_t)2 * Q * C * 2;
  stem_stage_pooled(dout, arg, dl, al, n, p, P, Q, C8);
  float sc[8], sh[8], ca[8], cb[8], ccf[8];
  ld8(params + 2 * C + c0, sc);
  ld8(params + 3 * C + c0, sh);
  if (EVAL) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ca[k] = sc[k];
      cb[k] = ccf[k] = 0.f;
    }
  } else {
    const float inv_cnt = 1.f / (count ? count[0] : count_h);
    float mean[8], inv[8], g[8], q0[8], q1[8];
    ld8(params + c0, mean);
    ld8(params + C + c0, inv);
    ld8(gamma + c0, g);
    ld8(red + c0, q0);
    ld8(red + C + c0, q1);
#pragma unroll
    for (int k = 0; k < 8; ++k) stem_bwd_coeffs(g[k], inv[k], mean[k], q0[k] * inv_cnt, q1[k] * inv_cnt, ca[k], cb[k], ccf[k]);
  }
  __syncthreads();
  const StemBwdTile t{dl, al, p, P, Q, C8};
  const int per_row = W * C8;
  const int h0 = 2 * p, nrow = min(2, H - h0);
  for (int j = tid; j < nrow * per_row; j += 256) {
    const int r = j >= per_row ? 1 : 0;
    const int jj = j - r * per_row;
    const int h = h0 + r, w = jj >> log2C8;
    const size_t i = ((size_t)n * H + h) * per_row + jj;
    float v[8], d[8], o[8];
    unpack8(ld16n<NT_STEM>(reinterpret_cast<const uint4*>(y) + i), v);
    t.dz(h, w, cc, v, sc, sh, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = EVAL ? ca[k] * d[k] : stem_bwd_dy(ca[k], cb[k], ccf[k], d[k], v[k]);
    reinterpret_cast<uint4*>(dy)[i] = pack8(o);
  }
}

static int l2e(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

int stem_pool_fwd_launch(const bf16_t* y, const float* params, bf16_t* out, uint8_t* arg, int N, int H,
                         int W, int C, int P, int Q, hipStream_t st) {
  const int l = l2e(C / 8);
  if (C % 8 || l < 0 || (C / 8) > 256 || N * P > 65535) return 1;
  const dim3 grid((Q * (C / 8) + 255) / 256, N * P);
  hipLaunchKernelGGL(stem_pool_fwd_kernel, grid, dim3(256), 0, st, y, params, out, arg, H, W, C, P, Q, l);
  return 0;
}

// dynamic LDS of the backward kernels: two staged pooled rows (gradient + taps),
// reused for the 256x17 fp32 partials of the reduce
static size_t stem_bwd_lds(int Q, int C) {
  const size_t staged = (size_t)2 * Q * C * 3;
  const size_t part = (size_t)256 * 17 * 4;
  return staged > part ? staged : part;
}

int stem_pool_bwd_reduce_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y,
                                const float* params, float* red, int N, int H, int W, int C, int P, int Q,
                                hipStream_t st) {
  const int l = l2e(C / 8);
  if (C % 8 || l < 0 || (C / 8) > 256 || 2 * P < H || 2 * Q < W) return 1;
  const size_t lds = stem_bwd_lds(Q, C);
  if (lds > 64 * 1024) return 2;
  DetStats det;
  const int ns = det_begin(det, &red, nullptr, N * P, 2 * C, st);
  if (ns < 1) return 3;
  hipLaunchKernelGGL(stem_pool_bwd_reduce_kernel, dim3(N * P), dim3(256), lds, st, dout, arg, y, params, red,
                     N, H, W, C, P, Q, l, ns);
  det_end(det, st);
  return 0;
}

int stem_pool_bwd_elemt_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y, const float* params,
                               const float* gamma, const float* red, const float* count, float count_h,
                               bf16_t* dy, int N, int H, int W, int C, int P, int Q, bool eval_mode,
                               hipStream_t st) {
  const int l = l2e(C / 8);
  if (C % 8 || l < 0 || (C / 8) > 256 || 2 * P < H || 2 * Q < W) return 1;
  const size_t lds = stem_bwd_lds(Q, C);
  if (lds > 64 * 1024) return 2;
  if (eval_mode)
    hipLaunchKernelGGL(stem_pool_bwd_elemt_kernel<true>, dim3(N * P), dim3(256), lds, st, dout, arg, y, params,
                       gamma, red, count, count_h, dy, N, H, W, C, P, Q, l);
  else
    hipLaunchKernelGGL(stem_pool_bwd_elemt_kernel<false>, dim3(N * P), dim3(256), lds, st, dout, arg, y,
                       params, gamma, red, count, count_h, dy, N, H, W, C, P, Q, l);
  return 0;
}

// ---------------------------------------------------------------------------
// Space-to-depth ImageNet stem.  The 7x7/s2/pad-3 conv over 3 channels is
// re-expressed on the 2x2-blocked image xs[n][u][v][(dy*2+dx)*4 + c] =
// x[n][2u+dy][2v+dx][c] (c < 4; the 3-channel input is zero-padded to 8, so
// c = 3 is already 0) as a 4x4/s1 conv over 16 channels with pad 2 on the
// top/left and 1 on the bottom/right (the launcher passes OH = H/2 explicitly):
//   output p reads input rows 2p-3 .. 2p+3 = blocks u = p-2 .. p+1, i.e.
//   tap i = 2 r + dy - 1 of the 7x7 filter (zero where i = -1 or 7).
// The reduction shrinks from 7*7*8 = 392 (62% zero padding, a 128-wide wgrad
// tile left 23% empty) to 4*4*16 = 256 (25% padding, exactly 2 wgrad tiles).
__global__ __launch_bounds__(256) void stem_s2d_input_kernel(const bf16_t* __restrict__ x,
                                                             bf16_t* __restrict__ xs, int N, int H,
                                                             int W) {
  const int Hs = H >> 1, Ws = W >> 1;
  const long long total = (long long)N * Hs * Ws;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int v = (int)(i % Ws), u = (int)((i / Ws) % Hs), n = (int)(i / ((long long)Ws * Hs));
    uint2 q[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int h = 2 * u + (d >> 1), w = 2 * v + (d & 1);
      q[d] = *reinterpret_cast<const uint2*>(x + (((size_t)n * H + h) * W + w) * 8);  // channels 0..3
    }
    uint4* o = reinterpret_cast<uint4*>(xs + (size_t)i * 16);
    o[0] = make_uint4(q[0].x, q[0].y, q[1].x, q[1].y);
    o[1] = make_uint4(q[2].x, q[2].y, q[3].x, q[3].y);
  }
}

// bf16 forward image ws[k][r][s][(dy*2+dx)*4 + c] of the fp32 7x7 weight
// w[k][i][j][c] (channels_last parameter storage, C input channels <= 4).
__global__ __launch_bounds__(256) void stem_s2d_weight_kernel(const float* __restrict__ w,
                                                              bf16_t* __restrict__ ws, int K, int C) {
  const int total = K * 4 * 4 * 16;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int ch = t & 15, s = (t >> 4) & 3, r = (t >> 6) & 3, k = t >> 8;
    const int q = ch >> 2, c = ch & 3, dy = q >> 1, dx = q & 1;
    const int i = 2 * r + dy - 1, j = 2 * s + dx - 1;
    const bool ok = c < C && i >= 0 && i < 7 && j >= 0 && j < 7;
    ws[t] = f2bf(ok ? w[(((size_t)k * 7 + i) * 7 + j) * C + c] : 0.f);
  }
}

// dw[k][i][j][c] (+)= dws[k][r][s][(dy*2+dx)*4 + c] -- every 7x7 tap has exactly
// one (r, dy) / (s, dx) preimage; dw is the [K][7][7][C] fp32 gradient (arena view).
__global__ __launch_bounds__(256) void stem_s2d_wgrad_fold_kernel(const float* __restrict__ dws,
                                                                  float* __restrict__ dw, int K, int C,
                                                                  int accumulate) {
  const int total = K * 49 * C;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int c = t % C, j = (t / C) % 7, i = (t / (7 * C)) % 7, k = t / (49 * C);
    const int r = (i + 1) >> 1, dy = (i + 1) & 1, s = (j + 1) >> 1, dx = (j + 1) & 1;
    const float g = dws[(((size_t)k * 4 + r) * 4 + s) * 16 + (dy * 2 + dx) * 4 + c];
    dw[t] = accumulate ? dw[t] + g : g;
  }
}

int stem_s2d_input_launch(const bf16_t* x, bf16_t* xs, int N, int H, int W, hipStream_t st) {
  if ((H | W) & 1) return 1;
  long long b = ((long long)N * (H / 2) * (W / 2) + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(stem_s2d_input_kernel, dim3((int)b), dim3(256), 0, st, x, xs, N, H, W);
  return 0;
}

int stem_s2d_weight_launch(const float* w, bf16_t* ws, int K, int C, hipStream_t st) {
  if (C > 4) return 1;
  hipLaunchKernelGGL(stem_s2d_weight_kernel, dim3((K * 256 + 255) / 256), dim3(256), 0, st, w, ws, K, C);
  return 0;
}

int stem_s2d_wgrad_fold_launch(const float* dws, float* dw, int K, int C, bool accumulate, hipStream_t st) {
  if (C > 4) return 1;
  hipLaunchKernelGGL(stem_s2d_wgrad_fold_kernel, dim3((K * 49 * C + 255) / 256), dim3(256), 0, st, dws, dw,
                     K, C, accumulate ? 1 : 0);
  return 0;
}

}  // namespace pmd
