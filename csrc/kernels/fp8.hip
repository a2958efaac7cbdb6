// FP8 (OCP e4m3) support for the fp8 training path (BASELINE config 5, K20):
//   * per-tensor quantisation with delayed scaling: q = sat_e4m3(x * scale),
//     scale read from device memory (no host sync), amax of the input
//     accumulated for the NEXT step's scale: block max, then atomicMax on the
//     float bits of |x| (order-preserving for non-negative floats) into one of
//     kAmaxSlots slots per site;
//   * weight images: fp32 master [K,R,S,C] -> e4m3 [K][R][S][Cp] (+ amax);
//   * a probe of the v_mfma_scale_f32_16x16x128_f8f6f4 operand lane map,
//     checked with exact integer data (tests/test_fp8_gpu.py).
#include "common.h"

namespace pmd {

typedef __attribute__((ext_vector_type(8))) int i32x8;

// v_cvt_pk_fp8_f32 rounds to nearest even but does NOT saturate: |v| > 448
// becomes the e4m3fn NaN code.  Clamp first (one v_med3_f32).
__device__ __forceinline__ float sat_e4m3(float v) { return __builtin_amdgcn_fmed3f(v, -448.f, 448.f); }

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(a), sat_e4m3(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(c), sat_e4m3(d), w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ float fp8_to_f32(uint32_t byte) {
  return __builtin_amdgcn_cvt_f32_fp8((int)byte, 0);
}

// OCP e5m2 (bf8, the gradient format of the fp8 wgrad): max normal 57344; the
// convert does not saturate either
__device__ __forceinline__ uint32_t pack4_bf8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_bf8_f32(__builtin_amdgcn_fmed3f(a, -57344.f, 57344.f),
                                          __builtin_amdgcn_fmed3f(b, -57344.f, 57344.f), 0, false);
  w = __builtin_amdgcn_cvt_pk_bf8_f32(__builtin_amdgcn_fmed3f(c, -57344.f, 57344.f),
                                      __builtin_amdgcn_fmed3f(d, -57344.f, 57344.f), w, true);
  return (uint32_t)w;
}


// bf16 [n] (n % 16 == 0) -> e4m3 (BF8: e5m2) [n]; amax_in += max |x|
template <bool BF8>
__global__ __launch_bounds__(256) void quant_bf16_fp8_kernel(const bf16_t* __restrict__ x,
                                                            uint8_t* __restrict__ q,
                                                            const float* __restrict__ scale,
                                                            float* __restrict__ amax, long long n16) {
  const float s = scale[0];
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (long long)gridDim.x * blockDim.x) {
    const uint4 a = reinterpret_cast<const uint4*>(x)[2 * i];
    const uint4 b = reinterpret_cast<const uint4*>(x)[2 * i + 1];
    float f[16];
    unpack8(a, *reinterpret_cast<float(*)[8]>(f));
    unpack8(b, *reinterpret_cast<float(*)[8]>(f + 8));
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(f[4 * k + e]));
      w[k] = BF8 ? pack4_bf8(f[4 * k] * s, f[4 * k + 1] * s, f[4 * k + 2] * s, f[4 * k + 3] * s)
                 : pack4_fp8(f[4 * k] * s, f[4 * k + 1] * s, f[4 * k + 2] * s, f[4 * k + 3] * s);
    }
    reinterpret_cast<uint4*>(q)[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if (amax) block_amax_update(amax, m);
}

// fp32 master [K][RS][C] (channels_last physical) -> e4m3 [K][RS][Cp] (zero padded), and
// optionally the transposed image qt [Cp][RS][K] (the fp8 dgrad's B^T, same scale)
__global__ void quant_weight_fp8_kernel(const float* __restrict__ w, uint8_t* __restrict__ q,
                                        const float* __restrict__ scale, float* __restrict__ amax,
                                        int K, int RS, int C, int Cp, uint8_t* __restrict__ qt) {
  const float s = scale[0];
  float m = 0.f;
  const int total = K * RS * Cp;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % Cp;
    const int krs = i / Cp;
    const float v = c < C ? w[(size_t)krs * C + c] : 0.f;
    m = fmaxf(m, fabsf(v));
    const uint8_t b = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(v * s), 0.f, 0, false) & 0xff);
    q[i] = b;
    if (qt) {
      const int k = krs / RS, rs = krs - k * RS;
      qt[((size_t)c * RS + rs) * K + k] = b;
    }
  }
  if (amax) block_amax_update(amax, m);
}

// Grouped form: block b finds its descriptor in the block-start table (a few
// dozen entries), then walks 64 (k) x 64 (c) tiles of each tap of that weight:
// q rows written along c, and the transposed image qt through LDS so its rows
// are written along k too (not one byte per K-strided address); amax goes to the
// weight's own slots (one atomicMax per block, every block of one weight).
__global__ __launch_bounds__(256) void quant_weight_fp8_grouped_kernel(const Fp8WeightDesc* __restrict__ descs,
                                                                       const int* __restrict__ block_start, int n) {
  __shared__ int e_sh;
  __shared__ uint32_t tile[64][65];
  if (threadIdx.x == 0) {
    int e = 0;
    while (e + 1 < n && block_start[e + 1] <= (int)blockIdx.x) ++e;
    e_sh = e;
  }
  __syncthreads();
  const Fp8WeightDesc d = descs[e_sh];
  const int lb = blockIdx.x - block_start[e_sh];
  const int nb = block_start[e_sh + 1] - block_start[e_sh];
  const float s = d.scale[0];
  float m = 0.f;
  const int kt = (d.K + 63) / 64, ct = (d.Cp + 63) / 64;
  const int ntiles = d.RS * kt * ct;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int t = lb; t < ntiles; t += nb) {
    const int rs = t / (kt * ct);
    const int rem = t - rs * kt * ct;
    const int k0 = (rem / ct) * 64, c0 = (rem % ct) * 64;
#pragma unroll 4
    for (int r = ty; r < 64; r += 4) {
      const int k = k0 + r, c = c0 + tx;
      if (k < d.K && c < d.Cp) {
        const size_t krs = (size_t)k * d.RS + rs;
        const float v = c < d.C ? d.w[krs * d.C + c] : 0.f;
        m = fmaxf(m, fabsf(v));
        const uint8_t b = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(sat_e4m3(v * s), 0.f, 0, false) & 0xff);
        d.q[krs * d.Cp + c] = b;
        tile[r][tx] = b;
      }
    }
    if (d.qt) {
      __syncthreads();
#pragma unroll 4
      for (int r = ty; r < 64; r += 4) {
        const int c = c0 + r, k = k0 + tx;
        if (c < d.Cp && k < d.K) d.qt[((size_t)c * d.RS + rs) * d.K + k] = (uint8_t)tile[tx][r];
      }
      __syncthreads();
    }
  }
  // block_amax_update picks slot blockIdx % kAmaxSlots of the weight's own site
  block_amax_update(d.amax, m);
}

void quant_weight_fp8_grouped_launch(const Fp8WeightDesc* d_descs, const int* d_block_start, int n,
                                     int total_blocks, hipStream_t st) {
  hipLaunchKernelGGL(quant_weight_fp8_grouped_kernel, dim3(total_blocks), dim3(256), 0, st, d_descs,
                     d_block_start, n);
}

// Delayed-scaling update of every fp8 site in one launch (Fp8Scaling.update): one wave
// per site folds its kAmaxSlots amax copies, sets scale = fmax / amax where an amax was
// observed (else keeps the scale) and clears the slots for the next step.
__global__ __launch_bounds__(256) void fp8_update_scales_kernel(float* __restrict__ amax,
                                                                 float* __restrict__ scale, int n, float fmax) {
  const int site = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (site >= n) return;
  float* slots = amax + (size_t)site * kAmaxSlots;
  float a = 0.f;
  for (int i = lane; i < kAmaxSlots; i += 64) a = fmaxf(a, slots[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
  for (int i = lane; i < kAmaxSlots; i += 64) slots[i] = 0.f;
  if (lane == 0 && a > 0.f) scale[site] = fmax / fmaxf(a, 1e-12f);
}

int fp8_update_scales_launch(float* amax, float* scale, int n, float fmax, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fp8_update_scales_kernel, dim3((n + 3) / 4), dim3(256), 0, st, amax, scale, n, fmax);
  return 0;
}

// e4m3 (BF8: e5m2) -> fp32 (tests / debugging)
template <bool BF8>
__global__ void dequant_fp8_kernel(const uint8_t* __restrict__ q, float* __restrict__ out,
                                   const float* __restrict__ inv_scale, long long n) {
  const float s = inv_scale ? inv_scale[0] : 1.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    out[i] = (BF8 ? __builtin_amdgcn_cvt_f32_bf8((int)q[i], 0) : fp8_to_f32(q[i])) * s;
}

// One 16x16x128 scaled-MFMA tile: C[16][16] = A[16][128] * B[128][16], A row-major
// e4m3 [16][128], Bt = B^T row-major e4m3 [16][128].  Lane map under test:
// lane l holds A[l & 15][32 (l >> 4) + j], j = 0..31 (and the same for B^T).
__global__ void fp8_mfma_probe_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                                      float* __restrict__ C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  const int* pa = reinterpret_cast<const int*>(A + (l & 15) * 128 + 32 * (l >> 4));
  const int* pb = reinterpret_cast<const int*>(Bt + (l & 15) * 128 + 32 * (l >> 4));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = pa[i];
    b[i] = pb[i];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
#pragma unroll
  for (int e = 0; e < 4; ++e) C[((l >> 4) * 4 + e) * 16 + (l & 15)] = acc[e];
}

static int blocks_for(long long n, int per) {
  long long b = (n + per - 1) / per;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

int quant_bf16_fp8_launch(const bf16_t* x, uint8_t* q, const float* scale, float* amax, long long n,
                          hipStream_t st, bool bf8) {
  if (n % 16) return 1;
  if (bf8)
    hipLaunchKernelGGL(quant_bf16_fp8_kernel<true>, dim3(blocks_for(n / 16, 256)), dim3(256), 0, st, x, q, scale,
                       amax, n / 16);
  else
    hipLaunchKernelGGL(quant_bf16_fp8_kernel<false>, dim3(blocks_for(n / 16, 256)), dim3(256), 0, st, x, q, scale,
                       amax, n / 16);
  return 0;
}

int quant_weight_fp8_launch(const float* w, uint8_t* q, const float* scale, float* amax, int K, int RS,
                            int C, int Cp, hipStream_t st, uint8_t* qt) {
  hipLaunchKernelGGL(quant_weight_fp8_kernel, dim3(blocks_for((long long)K * RS * Cp, 256 * 16)), dim3(256), 0,
                     st, w, q, scale, amax, K, RS, C, Cp, qt);
  return 0;
}

int dequant_fp8_launch(const uint8_t* q, float* out, const float* inv_scale, long long n, hipStream_t st,
                       bool bf8) {
  if (bf8)
    hipLaunchKernelGGL(dequant_fp8_kernel<true>, dim3(blocks_for(n, 256)), dim3(256), 0, st, q, out, inv_scale, n);
  else
    hipLaunchKernelGGL(dequant_fp8_kernel<false>, dim3(blocks_for(n, 256)), dim3(256), 0, st, q, out, inv_scale, n);
  return 0;
}

int fp8_mfma_probe_launch(const uint8_t* A, const uint8_t* Bt, float* C, hipStream_t st) {
  hipLaunchKernelGGL(fp8_mfma_probe_kernel, dim3(1), dim3(64), 0, st, A, Bt, C);
  return 0;
}

}  // namespace pmd

namespace pmd {

__device__ __attribute__((aligned(16))) unsigned char g_zero16_f8[64];

// ---------------------------------------------------------------------------
// FP8 implicit-GEMM forward convolution on v_mfma_scale_f32_16x16x128_f8f6f4
// (e4m3 x e4m3, unit block scales; 2x the bf16 MFMA rate per clock):
//   Y[m][k] = (1 / (sx * sw)) * sum_{r,s,c} Xq[n, ...] * Wq[k, r, s, c]
// Same tiling as the bf16 kernel (BM x BN tile, 4 waves in 2x2, LDS-DMA
// double buffer) with a K-tile of 128 fp8 = 128-B LDS rows (fp8 chunk swizzle
// swz_f8, common.h: conflict-free 32-B fragment reads) and one 16x16x128 MFMA per fragment pair.  bf16 output + fused
// per-channel (sum, sum^2) statistics for BatchNorm, as the bf16 kernel.
struct Fp8ConvArgs {
  const uint8_t* src;  // NHWC e4m3 [N,H,W,C]
  const uint8_t* wt;   // e4m3 [K][R][S][C]
  bf16_t* out;         // [M][K]
  float* stats;        // BN statistic slots about the shift K (see bn_moments)
  const float* shift;  // K [Nout] (nullable: 0)
  const float* sx;     // device scalars: the per-tensor scales the operands were quantised with
  const float* sw;
  int N, H, W, Cs, log2Cs, OH, OW, Nout, R, S, stride, pad, M, Kg;
  int nslots;          // statistics slot count (stat_slot, common.h)
};

template <int BM, int BN, bool STATS>
__global__ __launch_bounds__(256, 2) void conv_fp8_fwd_kernel(Fp8ConvArgs a) {
  constexpr int BK = 128;             // fp8 elements per K-tile (128 B rows)
  constexpr int PA = BM / 32, PB = BN / 32;  // DMA instructions per thread (8 rows each / wave)
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int A_B = BM * BK, B_B = BN * BK;  // bytes
  constexpr int STAGE = A_B + B_B;
  constexpr int LDC = BN + 8;
  constexpr int SMEM_MAIN = 2 * STAGE;
  constexpr int SMEM_EPI = BM * LDC * 2;
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) char smem[SMEM + (STATS ? 2 * 2 * BN * 4 : 0)];
  uint8_t* lds = reinterpret_cast<uint8_t*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesN = (a.Nout + BN - 1) / BN;
  const int tilesM = (a.M + BM - 1) / BM;
  const int L = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int m0 = (L / tilesN) * BM, n0 = (L % tilesN) * BN;
  if (m0 >= a.M) return;

  // logical 16-B chunk this lane fetches into row 8 i + lane / 8 (mod 16) of its 8-row piece:
  // fp8 swizzle (common.h swz_f8), which depends on the row parity of the piece (i & 1)
  const int chunk2[2] = {(lane & 7) ^ swz_f8(lane >> 3), (lane & 7) ^ swz_f8(8 + (lane >> 3))};
  int a_base[PA], a_h[PA], a_w[PA];
  bool a_ok[PA];
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int m = m0 + wid * (BM / 4) + 8 * i + (lane >> 3);
    a_ok[i] = m < a.M;
    const int mm = a_ok[i] ? m : 0;
    const int n = mm / ohw, rem = mm - n * ohw;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    a_base[i] = n * a.H * a.W;
    a_h[i] = oh * a.stride - a.pad;
    a_w[i] = ow * a.stride - a.pad;
  }
  const uint8_t* b_row[PB];
  bool b_ok[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int nn = n0 + wid * (BN / 4) + 8 * i + (lane >> 3);
    b_ok[i] = nn < a.Nout;
    b_row[i] = a.wt + (size_t)(b_ok[i] ? nn : 0) * a.Kg;
  }
  const int nk = (a.Kg + BK - 1) / BK;
  auto load_tile = [&](int kt, int buf) {
    // the two chunk variants' taps (a K-tile of 128 spans two taps when Cs = 64)
    int kr[2], ks[2], kc[2], kb[2];
    bool kk[2];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int k0 = kt * BK + chunk2[v] * 16;
      kk[v] = k0 < a.Kg;
      const int tap = k0 >> a.log2Cs;
      kc[v] = k0 & (a.Cs - 1);
      kr[v] = tap / a.S;
      ks[v] = tap - kr[v] * a.S;
      kb[v] = ((kr[v] * a.S + ks[v]) << a.log2Cs) + kc[v];
    }
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int r = kr[i & 1], s = ks[i & 1], c = kc[i & 1];
      const bool kok = kk[i & 1];
      const int ih = a_h[i] + r, iw = a_w[i] + s;
      const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const void* src = g_zero16_f8;
      if (ok) src = a.src + (((size_t)(a_base[i] + ih * a.W + iw)) << a.log2Cs) + c;
      uint8_t* dst = lds + buf * STAGE + (wid * (BM / 4) + 8 * i) * BK;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const void* src = (b_ok[i] && kk[i & 1]) ? (const void*)(b_row[i] + kb[i & 1]) : (const void*)g_zero16_f8;
      uint8_t* dst = lds + buf * STAGE + A_B + (wid * (BN / 4) + 8 * i) * BK;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15;
  const int q0 = 2 * (lane >> 4);  // lane holds k = 32 (lane>>4) + 0..31 = chunks q0, q0+1
  auto frag = [&](const uint8_t* base, int r) {
    const uint4 lo = *reinterpret_cast<const uint4*>(base + r * BK + ((q0 ^ swz_f8(r)) << 4));
    const uint4 hi = *reinterpret_cast<const uint4*>(base + r * BK + (((q0 + 1) ^ swz_f8(r)) << 4));
    i32x8 v;
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    return v;
  };
  auto compute = [&](int buf) {
    const uint8_t* As = lds + buf * STAGE;
    const uint8_t* Bs = As + A_B;
    i32x8 af[MI], bfg[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = frag(As, wm * (BM / 2) + i * 16 + frow);
#pragma unroll
    for (int j = 0; j < NI; ++j) bfg[j] = frag(Bs, wn * (BN / 2) + j * 16 + frow);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfg[j], acc[i][j], 0, 0, 0,
                                                                      127, 0, 127);
  };
  if (nk > 0) load_tile(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + 1 < nk) load_tile(kt + 1, (kt + 1) & 1);
    compute(kt & 1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: descale, bf16, BN statistics, LDS-staged coalesced stores
  const float ds = 1.f / (a.sx[0] * a.sw[0]);
  bf16_t* Cs = reinterpret_cast<bf16_t*>(smem);
  const int crow0 = wm * (BM / 2) + (lane >> 4) * 4;
  const int ccol0 = wn * (BN / 2) + (lane & 15);
  float csum[NI], csq[NI], cshift[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    csum[j] = csq[j] = cshift[j] = 0.f;
    if (STATS && a.shift && n0 + ccol0 + j * 16 < a.Nout) cshift[j] = a.shift[n0 + ccol0 + j * 16];
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16_t h = f2bf(acc[i][j][e] * ds);
        Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = h;
        if (STATS) {
          const float v = m0 + crow0 + i * 16 + e < a.M ? bf2f(h) - cshift[j] : 0.f;
          csum[j] += v;
          csq[j] += v * v;
        }
      }
  if (STATS) {
    float* st = reinterpret_cast<float*>(smem + SMEM);
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      float s1 = csum[j], s2 = csq[j];
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 16) {
        st[(wm * 2 + 0) * BN + ccol0 + j * 16] = s1;
        st[(wm * 2 + 1) * BN + ccol0 + j * 16] = s2;
      }
    }
  }
  __syncthreads();
  if (STATS) {
    const float* st = reinterpret_cast<const float*>(smem + SMEM);
    for (int c = tid; c < 2 * BN; c += 256) {
      const int which = c / BN, col = c % BN;
      if (n0 + col < a.Nout) {
        const float v = st[which * BN + col] + st[(2 + which) * BN + col];
        atomicAdd(a.stats + (stat_slot(m0 / BM, a.nslots) * 2 + which) * a.Nout + n0 + col, v);
      }
    }
  }
  constexpr int CPR = BN / 8;
  for (int idx = tid; idx < BM * CPR; idx += 256) {
    const int row = idx / CPR, cc = idx % CPR;
    const int m = m0 + row, n = n0 + cc * 8;
    if (m < a.M && n < a.Nout)
      st16n<NT_CONV_ST>(a.out + (size_t)m * a.Nout + n, *reinterpret_cast<const uint4*>(Cs + row * LDC + cc * 8));
  }
}

int conv_fp8_fwd_launch(const uint8_t* x, const uint8_t* w, bf16_t* out, float* stats, const float* sx,
                        const float* sw, int N, int H, int W, int C, int OH, int OW, int K, int R,
                        int S, int stride, int pad, hipStream_t st, const float* shift) {
  if (C % 16 != 0 || (C & (C - 1)) != 0) return 1;  // a 16-B chunk = 16 channels of one tap
  if (K % 8 != 0) return 2;
  Fp8ConvArgs a;
  a.src = x;
  a.wt = w;
  a.out = out;
  a.stats = stats;
  a.shift = stats ? shift : nullptr;
  a.sx = sx;
  a.sw = sw;
  a.N = N; a.H = H; a.W = W; a.Cs = C;
  int l = 0;
  while ((1 << l) < C) ++l;
  a.log2Cs = l;
  a.OH = OH; a.OW = OW; a.Nout = K; a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  const long long M = (long long)N * OH * OW;
  if (M >= (1ll << 31)) return 4;
  a.M = (int)M;
  a.Kg = R * S * C;
  const int BN = K <= 64 ? 64 : 128;
  const int tiles = (int)((M + 127) / 128) * ((K + BN - 1) / BN);
  DetStats det;
  a.nslots = det_begin(det, &a.stats, nullptr, (int)((M + 127) / 128), 2 * K, st);
  if (a.nslots < 1) return 10;
  if (BN == 64) {
    if (stats) hipLaunchKernelGGL((conv_fp8_fwd_kernel<128, 64, true>), dim3(tiles), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_fp8_fwd_kernel<128, 64, false>), dim3(tiles), dim3(256), 0, st, a);
  } else {
    if (stats) hipLaunchKernelGGL((conv_fp8_fwd_kernel<128, 128, true>), dim3(tiles), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((conv_fp8_fwd_kernel<128, 128, false>), dim3(tiles), dim3(256), 0, st, a);
  }
  det_end(det, st);
  return 0;
}

}  // namespace pmd
