// Synchronised-BatchNorm family on NHWC bf16 activations (gfx950).
//
// Statistics are produced by the conv epilogue (conv_igemm.hip); these
// kernels cover the rest of torch's SyncBN autograd Function
// (torch:nn/modules/_functions.py:39-207) with the ReLU and residual add of
// the ResNet block (reference model/resnet.py:36-39, 66-70) fused in:
//
//   bn_finalize   (sum, sum^2, count) -> mean, invstd, scale, shift;
//                 running_mean/var momentum update (unbiased var) and
//                 num_batches_tracked += 1, all on device (no host sync)
//   bn_apply      out = relu(y1*sc1+sh1 [+ y2*sc2+sh2 | + res])       1 pass
//   bn_bwd_reduce sum(dz*mask), sum(dz*mask*xhat) per channel          1 pass
//   bn_bwd_elemt  dy = a*dzm + b*y + c (per-channel a,b,c), optional
//                 dzm output for the identity-shortcut gradient        1 pass
//
// All elementwise kernels move 16 B (8 channels) per lane per stream and keep
// a fixed channel chunk per thread (grid*256 is a multiple of C/8), so the
// per-channel coefficients are loaded once per thread.
#include "common.h"

#ifndef PMD_EW_U
#define PMD_EW_U 1
#endif

namespace pmd {

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// params out: [4][C] = mean, invstd, scale, shift
__global__ void bn_finalize_kernel(const float* __restrict__ sums, const float* __restrict__ count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ params, float* running_mean,
                                   float* running_var, long long* nbt, float* shift, int C,
                                   float eps, float momentum, int eval_mode) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
    float mean, var;
    if (eval_mode) {
      mean = running_mean[c];
      var = running_var[c];
    } else {
      bn_moments(sums[c], sums[C + c], count[0], shift ? shift[c] : 0.f, mean, var);
      if (shift) shift[c] = mean;  // the next step's statistics shift
    }
    const float invstd = rsqrtf(var + eps);
    const float sc = gamma[c] * invstd;
    params[c] = mean;
    params[C + c] = invstd;
    params[2 * C + c] = sc;
    params[3 * C + c] = beta[c] - mean * sc;
    if (!eval_mode && running_mean) {
      const float cnt = count[0];
      const float unb = var * (cnt / fmaxf(cnt - 1.f, 1.f));
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  }
  if (!eval_mode && nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

// MODE 0: out = act(y1*s1+b1); 1: + res; 2: + y2*s2+b2
// Q8: also emit an e4m3 copy q = sat(out * qscale) (the fp8 conv's input, BASELINE
// config 5) and accumulate amax(|out|) for the next step's delayed scale.
template <int MODE, bool RELU, bool Q8>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ y1,
                                                       const float* __restrict__ p1,
                                                       const bf16_t* __restrict__ r,
                                                       const float* __restrict__ p2,
                                                       bf16_t* __restrict__ out,
                                                       uint8_t* __restrict__ mask_out,
                                                       uint8_t* __restrict__ q_out,
                                                       const float* __restrict__ qscale,
                                                       float* __restrict__ qamax,
                                                       long long nchunk, int C) {
  float qs = 0.f, qm = 0.f;
  if (Q8) qs = qscale[0];
  const int C8 = C >> 3;
  const long long start = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long step = (long long)gridDim.x * blockDim.x;
  const int c0 = (int)(start % C8) * 8;
  float s1[8], b1[8], s2[8], b2[8];
  load8f(p1 + 2 * C + c0, s1);
  load8f(p1 + 3 * C + c0, b1);
  if (MODE == 2) {
    load8f(p2 + 2 * C + c0, s2);
    load8f(p2 + 3 * C + c0, b2);
  }
  // U chunks per thread per trip, all loads issued before any store.  Measured
  // (bench/ab_so.sh, full R50 step): U=2 is 0.4% SLOWER than U=1 -- the
  // 2048x256-thread grid at full occupancy already covers HBM latency -- so the
  // default stays 1; the knob is kept for A/B builds (PMD_EXTRA_CFLAGS).
  constexpr int U = PMD_EW_U;
  for (long long i0 = start; i0 < nchunk; i0 += U * step) {
    uint4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * step;
      if (i < nchunk) {
        yv[u] = ld16n<NT_BNA_Y>(reinterpret_cast<const uint4*>(y1) + i);
        if (MODE >= 1) rv[u] = ld16n<NT_BNA_R>(reinterpret_cast<const uint4*>(r) + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * step;
      if (i >= nchunk) break;
      float v[8], w[8];
      unpack8(yv[u], v);
      if (MODE >= 1) unpack8(rv[u], w);
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float o = v[k] * s1[k] + b1[k];
        if (MODE == 1) o += w[k];
        if (MODE == 2) o += w[k] * s2[k] + b2[k];
        if (RELU) {
          bits |= (uint32_t)(o > 0.f) << k;
          o = fmaxf(o, 0.f);
        }
        v[k] = o;
      }
      const uint4 pk = pack8(v);
      // Q8 with out == nullptr: the e4m3 copy is the ONLY activation (its consumers --
      // the fp8 conv and the fp8 wgrad -- never read a bf16 one)
      if (!Q8 || out) st16n<NT_EW_ST>(reinterpret_cast<uint4*>(out) + i, pk);
      if (RELU && mask_out) mask_out[i] = (uint8_t)bits;
      if (Q8) {
        float o[8];
        unpack8(pk, o);  // quantise the bf16 value the bf16 consumers see
        // the convert does not saturate (|v| > 448 -> NaN code): clamp with v_med3
        float c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_fmed3f(o[k] * qs, -448.f, 448.f);
        int w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
        w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w0, true);
        int w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
        w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], w1, true);
        reinterpret_cast<uint2*>(q_out)[i] = make_uint2((uint32_t)w0, (uint32_t)w1);
#pragma unroll
        for (int k = 0; k < 8; ++k) qm = fmaxf(qm, fabsf(o[k]));
      }
    }
  }
  if (Q8) block_amax_update(qamax, qm);
}

// red out: [slot][2][C] += (sum dzm, sum dzm*xhat).
// Grid: x = row blocks, y = channel tiles of CT8 = min(C/8, 32) 16-B chunks
// (256 channels).  A block covers its channel tile for 256/CT8 rows per
// iteration, two rows in flight per thread; the row-block count is sized so
// each thread streams ~32 rows -- few enough blocks that the per-block
// partials (one atomic per channel per block, spread over kStatSlots slot
// copies) stay far below the streaming cost even at 7x7x2048.
template <bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const bf16_t* __restrict__ dout,
                                                            const uint8_t* __restrict__ mask,
                                                            const bf16_t* __restrict__ y,
                                                            const float* __restrict__ params,
                                                            float* __restrict__ red, int M, int C,
                                                            int CT8, int nslots) {
  __shared__ float part[256 * 17];
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  const int cc = blockIdx.y * CT8 + tid % CT8;
  const int rpi = 256 / CT8;
  const int c0 = cc * 8;
  float mean[8], inv[8];
  load8f(params + c0, mean);
  load8f(params + C + c0, inv);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
  const int stride = gridDim.x * rpi;
  int row = blockIdx.x * rpi + tid / CT8;
  for (; row + stride < M; row += 2 * stride) {
    const long long i0 = (long long)row * C8 + cc;
    const long long i1 = i0 + (long long)stride * C8;
    const uint4 d0 = reinterpret_cast<const uint4*>(dout)[i0];
    const uint4 d1 = reinterpret_cast<const uint4*>(dout)[i1];
    const uint4 y0 = reinterpret_cast<const uint4*>(y)[i0];
    const uint4 y1 = reinterpret_cast<const uint4*>(y)[i1];
    const uint32_t m0 = RELU ? mask[i0] : 0xffu;
    const uint32_t m1 = RELU ? mask[i1] : 0xffu;
    float d[8], v[8];
    unpack8(d0, d);
    unpack8(y0, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dz = ((m0 >> k) & 1u) ? d[k] : 0.f;
      s1[k] += dz;
      s2[k] += dz * (v[k] - mean[k]) * inv[k];
    }
    unpack8(d1, d);
    unpack8(y1, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dz = ((m1 >> k) & 1u) ? d[k] : 0.f;
      s1[k] += dz;
      s2[k] += dz * (v[k] - mean[k]) * inv[k];
    }
  }
  if (row < M) {
    const long long i = (long long)row * C8 + cc;
    float d[8], v[8];
    unpack8(reinterpret_cast<const uint4*>(dout)[i], d);
    const uint32_t mb = RELU ? mask[i] : 0xffu;
    unpack8(reinterpret_cast<const uint4*>(y)[i], v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dz = ((mb >> k) & 1u) ? d[k] : 0.f;
      s1[k] += dz;
      s2[k] += dz * (v[k] - mean[k]) * inv[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    part[tid * 17 + k] = s1[k];
    part[tid * 17 + 8 + k] = s2[k];
  }
  __syncthreads();
  // 16 values per chunk column: thread (col, k) sums one of them over the rpi rows
  for (int e = tid; e < CT8 * 16; e += 256) {
    const int col = e >> 4, k = e & 15;
    float a = 0.f;
    for (int rr = 0; rr < rpi; ++rr) a += part[(rr * CT8 + col) * 17 + k];
    const int c = (blockIdx.y * CT8 + col) * 8 + (k & 7);
    float* slot = red + stat_slot(blockIdx.x, nslots) * 2 * C;
    atomicAdd(slot + (k < 8 ? 0 : C) + c, a);
  }
}

// dy = a*dzm + b*y + c.  train: a = g*inv, b = -a*inv*mdyx, c = a*(mean*inv*mdyx - mdy)
//                        eval : a = scale, b = c = 0
// Q8: also write dy as OCP e5m2 (bf8) * qscale -- the fp8 weight gradient's dY operand
// (kernels/conv_wgrad.hip) -- quantised from the bf16-rounded value the dgrad reads,
// saturated to +-57344, and accumulate amax |dy| for the next step's scale.
template <bool RELU, bool DZM, bool EVAL, bool Q8 = false>
__global__ __launch_bounds__(256) void bn_bwd_elemt_kernel(
    const bf16_t* __restrict__ dout, const uint8_t* __restrict__ mask, const bf16_t* __restrict__ y,
    const float* __restrict__ params, const float* __restrict__ gamma,
    const float* __restrict__ red, const float* __restrict__ count, float count_h,
    bf16_t* __restrict__ dy, bf16_t* __restrict__ dzm_out, long long nchunk, int C,
    uint8_t* __restrict__ q_out = nullptr, const float* __restrict__ qscale = nullptr,
    float* __restrict__ qamax = nullptr) {
  float qs = 0.f, qm = 0.f;
  if (Q8) qs = qscale[0];
  const int C8 = C >> 3;
  const long long start = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long step = (long long)gridDim.x * blockDim.x;
  const int c0 = (int)(start % C8) * 8;
  float ca[8], cb[8], cc[8];
  if (EVAL) {
    load8f(params + 2 * C + c0, ca);
#pragma unroll
    for (int k = 0; k < 8; ++k) cb[k] = cc[k] = 0.f;
  } else {
    const float inv_cnt = 1.f / (count ? count[0] : count_h);
    float mean[8], inv[8], g[8], r0[8], r1[8];
    load8f(params + c0, mean);
    load8f(params + C + c0, inv);
    load8f(gamma + c0, g);
    load8f(red + c0, r0);
    load8f(red + C + c0, r1);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = g[k] * inv[k];
      const float mdy = r0[k] * inv_cnt, mdyx = r1[k] * inv_cnt;
      ca[k] = a;
      cb[k] = -a * inv[k] * mdyx;
      cc[k] = a * (mean[k] * inv[k] * mdyx - mdy);
    }
  }
  constexpr int U = PMD_EW_U;  // chunks in flight per thread (see bn_apply_kernel)
  for (long long i0 = start; i0 < nchunk; i0 += U * step) {
    uint4 dv[U], yv[U];
    uint32_t mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * step;
      if (i < nchunk) {
        dv[u] = ld16n<NT_BNB_D>(reinterpret_cast<const uint4*>(dout) + i);
        mv[u] = RELU ? mask[i] : 0xffu;
        if (!EVAL) yv[u] = ld16n<NT_BNB_Y>(reinterpret_cast<const uint4*>(y) + i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * step;
      if (i >= nchunk) break;
      float d[8], o[8], v[8];
      unpack8(dv[u], d);
      const uint32_t mb = mv[u];
      if (!EVAL) unpack8(yv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dz = ((mb >> k) & 1u) ? d[k] : 0.f;
        d[k] = dz;
        o[k] = EVAL ? ca[k] * dz : ca[k] * dz + cb[k] * v[k] + cc[k];
      }
      const uint4 pk = pack8(o);
      // Q8 with dy == nullptr: the e5m2 copy is the only dY (every consumer -- the fp8
      // wgrad and the fp8 dgrad -- reads it)
      if (!Q8 || dy) st16n<NT_EW_ST>(reinterpret_cast<uint4*>(dy) + i, pk);
      if (DZM) st16n<NT_EW_ST>(reinterpret_cast<uint4*>(dzm_out) + i, pack8(d));
      if (Q8) {
        float r[8], c[8];
        unpack8(pk, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          qm = fmaxf(qm, fabsf(r[k]));
          c[k] = __builtin_amdgcn_fmed3f(r[k] * qs, -57344.f, 57344.f);
        }
        int w0 = __builtin_amdgcn_cvt_pk_bf8_f32(c[0], c[1], 0, false);
        w0 = __builtin_amdgcn_cvt_pk_bf8_f32(c[2], c[3], w0, true);
        int w1 = __builtin_amdgcn_cvt_pk_bf8_f32(c[4], c[5], 0, false);
        w1 = __builtin_amdgcn_cvt_pk_bf8_f32(c[6], c[7], w1, true);
        reinterpret_cast<uint2*>(q_out)[i] = make_uint2((uint32_t)w0, (uint32_t)w1);
      }
    }
  }
  if (Q8) block_amax_update(qamax, qm);
}

// out[0:2Ca] = sum_slots a[slot][2][Ca]; out[2Ca:2Ca+2Cb] = same for b; out[last] = count.
// clear: zero the slot buffers after reading (they return to the host-side pool
// ready for the next conv epilogue / reduce -- no memset launch).
// acc_a/acc_b: optional [2][C] fp32 gradient targets (d_beta | d_gamma rows)
// that receive += the collapsed local sums (direct-to-arena BN param grads).
// The slot buffers were filled by memory-side fp32 atomics, so nothing of them
// is in L2: every read is a full HBM/MALL round trip.  A thread therefore sums
// only kStatSlots/4 slots of one output with all its loads in flight at once,
// and the 4 slot groups of an output are combined through LDS -- one memory
// latency per kernel instead of kStatSlots/8 dependent batches.
constexpr int kSlotGroups = 4;
constexpr int kSlotsPerGroup = kStatSlots / kSlotGroups;

__global__ __launch_bounds__(256) void stats_collapse_kernel(
    float* __restrict__ a, int Ca, float* __restrict__ b, int Cb, float count, float* __restrict__ out,
    int with_count, int clear, float* __restrict__ acc_a0, float* __restrict__ acc_a1,
    float* __restrict__ acc_b0, float* __restrict__ acc_b1) {
  __shared__ float part[kSlotGroups][64];
  const int na = 2 * Ca, nb = b ? 2 * Cb : 0;
  const int li = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + li;
  float s = 0.f;
  if (i < na + nb) {
    float* src = i < na ? a + i : b + (i - na);
    const int n = i < na ? na : nb;
    float v[kSlotsPerGroup];
#pragma unroll
    for (int k = 0; k < kSlotsPerGroup; ++k) v[k] = src[(size_t)(g * kSlotsPerGroup + k) * n];
#pragma unroll
    for (int k = 0; k < kSlotsPerGroup; ++k) s += v[k];
    if (clear) {
#pragma unroll
      for (int k = 0; k < kSlotsPerGroup; ++k) src[(size_t)(g * kSlotsPerGroup + k) * n] = 0.f;
    }
  }
  part[g][li] = s;
  __syncthreads();
  if (g == 0) {
    if (i < na + nb) {
      // fixed order: bitwise identical to a sequential sum over the groups
      s = ((part[0][li] + part[1][li]) + part[2][li]) + part[3][li];
      out[i] = s;
      const int j = i < na ? i : i - na;
      const int C = i < na ? Ca : Cb;
      float* acc = i < na ? (j < C ? acc_a0 : acc_a1) : (j < C ? acc_b0 : acc_b1);
      if (acc) acc[j < C ? j : j - C] += s;
    } else if (with_count && i == na + nb) {
      out[i] = count;
    }
  }
}

int stats_collapse_launch(float* a, int Ca, float* b, int Cb, float count, float* out,
                          bool with_count, bool clear, float* acc_a0, float* acc_a1, float* acc_b0,
                          float* acc_b1, hipStream_t st) {
  const int n = 2 * Ca + (b ? 2 * Cb : 0) + (with_count ? 1 : 0);
  hipLaunchKernelGGL(stats_collapse_kernel, dim3((n + 63) / 64), dim3(256), 0, st, a, Ca, b, Cb,
                     count, out, with_count ? 1 : 0, clear ? 1 : 0, acc_a0, acc_a1, acc_b0, acc_b1);
  return 0;
}

// Single-replica BN statistics: collapse (and clear) the slots and finalize
// in one launch -- used when there is no SyncBN all-reduce between the two.
__global__ __launch_bounds__(256) void stats_finalize_local_kernel(
    float* __restrict__ slots, float count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ params, float* running_mean,
    float* running_var, long long* nbt, float* shift, int C, float eps, float momentum) {
  __shared__ float part[2][kSlotGroups][64];
  const int li = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + li;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    float v1[kSlotsPerGroup], v2[kSlotsPerGroup];
#pragma unroll
    for (int k = 0; k < kSlotsPerGroup; ++k) {
      const float* p = slots + (size_t)(g * kSlotsPerGroup + k) * 2 * C;
      v1[k] = p[c];
      v2[k] = p[C + c];
    }
#pragma unroll
    for (int k = 0; k < kSlotsPerGroup; ++k) {
      s1 += v1[k];
      s2 += v2[k];
      float* p = slots + (size_t)(g * kSlotsPerGroup + k) * 2 * C;
      p[c] = 0.f;
      p[C + c] = 0.f;
    }
  }
  part[0][g][li] = s1;
  part[1][g][li] = s2;
  __syncthreads();
  if (g == 0 && c < C) {
    s1 = ((part[0][0][li] + part[0][1][li]) + part[0][2][li]) + part[0][3][li];
    s2 = ((part[1][0][li] + part[1][1][li]) + part[1][2][li]) + part[1][3][li];
    float mean, var;
    bn_moments(s1, s2, count, shift ? shift[c] : 0.f, mean, var);
    if (shift) shift[c] = mean;
    const float invstd = rsqrtf(var + eps);
    const float sc = gamma[c] * invstd;
    params[c] = mean;
    params[C + c] = invstd;
    params[2 * C + c] = sc;
    params[3 * C + c] = beta[c] - mean * sc;
    if (running_mean) {
      const float unb = var * (count / fmaxf(count - 1.f, 1.f));
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
    }
  }
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) nbt[0] += 1;
}

int stats_finalize_local_launch(float* slots, float count, const float* gamma, const float* beta,
                                float* params, float* rm, float* rv, long long* nbt, float* shift, int C,
                                float eps, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(stats_finalize_local_kernel, dim3((C + 63) / 64), dim3(256), 0, st, slots, count,
                     gamma, beta, params, rm, rv, nbt, shift, C, eps, momentum);
  return 0;
}

static int ew_grid(long long nchunk, int C8) {
  long long b = (nchunk + 255) / 256;
#ifndef PMD_EW_BLOCKS
#define PMD_EW_BLOCKS 2048
#endif
  if (b > PMD_EW_BLOCKS) b = PMD_EW_BLOCKS;
  if (b < 1) b = 1;
  // keep grid*256 a multiple of C8 (C8 is a power of two <= 256, so always true)
  return (int)b;
}

int bn_finalize_launch(const float* sums, const float* count, const float* gamma, const float* beta,
                       float* params, float* rm, float* rv, long long* nbt, float* shift, int C,
                       float eps, float momentum, bool eval_mode, hipStream_t st) {
  const int blocks = (C + 255) / 256;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(blocks), dim3(256), 0, st, sums, count, gamma, beta,
                     params, rm, rv, nbt, shift, C, eps, momentum, eval_mode ? 1 : 0);
  return 0;
}

int bn_apply_launch(const bf16_t* y1, const float* p1, const bf16_t* r, const float* p2, bf16_t* out,
                    uint8_t* mask, long long M, int C, int mode, bool relu, uint8_t* q8,
                    const float* qscale, float* qamax, hipStream_t st) {
  if (C % 8 || (C >> 3) > 256 || ((C >> 3) & ((C >> 3) - 1))) return 1;
  if (q8 && (!qscale || !qamax)) return 2;
  const long long nchunk = M * (C / 8);
  const int g = ew_grid(nchunk, C / 8);
#define APPLY(MD, RL, Q)                                                                              \
  hipLaunchKernelGGL((bn_apply_kernel<MD, RL, Q>), dim3(g), dim3(256), 0, st, y1, p1, r, p2, out, mask, \
                     q8, qscale, qamax, nchunk, C)
  if (q8) {
    if (!relu) return 3;  // fp8 copies are only made of ReLU outputs (conv inputs)
    if (mode == 0) APPLY(0, true, true); else if (mode == 1) APPLY(1, true, true); else APPLY(2, true, true);
  } else if (relu) {
    if (mode == 0) APPLY(0, true, false); else if (mode == 1) APPLY(1, true, false); else APPLY(2, true, false);
  } else {
    if (mode == 0) APPLY(0, false, false); else if (mode == 1) APPLY(1, false, false);
    else APPLY(2, false, false);
  }
#undef APPLY
  return 0;
}

int bn_bwd_reduce_launch(const bf16_t* dout, const uint8_t* mask, const bf16_t* y,
                         const float* params, float* red, int M, int C, bool relu, hipStream_t st) {
  const int C8 = C / 8;
  if (C % 8 || C8 > 256 || (C8 & (C8 - 1))) return 1;
  const int CT8 = C8 < 32 ? C8 : 32;
  const int ctiles = C8 / CT8;
  const int rpi = 256 / CT8;
  long long b = ((long long)M + rpi * 32 - 1) / (rpi * 32);  // ~32 rows per thread
  const long long bmax = 1024 / ctiles;
  if (b > bmax) b = bmax;
  if (b < 1) b = 1;
  const dim3 grid((unsigned)b, (unsigned)ctiles);
  DetStats det;
  const int ns = det_begin(det, &red, nullptr, (int)b, 2 * C, st);
  if (ns < 1) return 2;
  if (relu)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<true>), grid, dim3(256), 0, st, dout, mask, y, params, red,
                       M, C, CT8, ns);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<false>), grid, dim3(256), 0, st, dout, mask, y, params,
                       red, M, C, CT8, ns);
  det_end(det, st);
  return 0;
}

int bn_bwd_elemt_launch(const bf16_t* dout, const uint8_t* mask, const bf16_t* y, const float* params,
                        const float* gamma, const float* red, const float* count, float count_h,
                        bf16_t* dy, bf16_t* dzm, long long M, int C, bool relu, bool eval_mode,
                        hipStream_t st, uint8_t* q8, const float* qscale, float* qamax) {
  if (C % 8 || (C >> 3) > 256 || ((C >> 3) & ((C >> 3) - 1))) return 1;
  const long long nchunk = M * (C / 8);
  const int g = ew_grid(nchunk, C / 8);
  if (q8) {
    // the fp8 wgrad's e5m2 dY copy: training mode, no dzm output
    if (!qscale || !qamax || eval_mode || dzm) return 2;
    if (relu)
      hipLaunchKernelGGL((bn_bwd_elemt_kernel<true, false, false, true>), dim3(g), dim3(256), 0, st, dout, mask,
                         y, params, gamma, red, count, count_h, dy, dzm, nchunk, C, q8, qscale, qamax);
    else
      hipLaunchKernelGGL((bn_bwd_elemt_kernel<false, false, false, true>), dim3(g), dim3(256), 0, st, dout, mask,
                         y, params, gamma, red, count, count_h, dy, dzm, nchunk, C, q8, qscale, qamax);
    return 0;
  }
#define EL(RL, DZ, EV)                                                                            \
  hipLaunchKernelGGL((bn_bwd_elemt_kernel<RL, DZ, EV>), dim3(g), dim3(256), 0, st, dout, mask, y, \
                     params, gamma, red, count, count_h, dy, dzm, nchunk, C)
  const bool dz = dzm != nullptr;
  if (eval_mode) {
    if (relu) { if (dz) EL(true, true, true); else EL(true, false, true); }
    else { if (dz) EL(false, true, true); else EL(false, false, true); }
  } else {
    if (relu) { if (dz) EL(true, true, false); else EL(true, false, false); }
    else { if (dz) EL(false, true, false); else EL(false, false, false); }
  }
#undef EL
  return 0;
}

}  // namespace pmd
