// Convolution weight gradient on gfx950 MFMA, split-K over the batch*spatial axis.
//
//   dW[k][(r,s,c)] = sum_{m=(n,p,q)} dY[m][k] * X[n, p*st-pad+r, q*st-pad+s, c]
//
// GEMM view: rows = output channels (BM), cols = Kg = R*S*C (BN), reduction
// over m = N*P*Q (hundreds of thousands).  Both operands arrive reduction-
// major (m rows, channels contiguous), so each 64-row chunk of dY and of the
// im2col'd X is staged into LDS in natural row order and the MFMA fragments
// (8 consecutive m of one column) are read with the CDNA4 hardware transpose
// read ds_read_b64_tr_b16.  LDS rows are XOR-swizzled at 32-byte granularity
// so the 8 rows a 32-lane half touches in one transposed read land in 8
// distinct bank windows.
//
// The m axis is split over blocks (enough blocks to fill the 256 CUs); each
// block reduces its range in registers and writes its fp32 partial tile with
// plain stores into a [split][K][Kg] workspace; wgrad_reduce then adds the
// splits into dW in a fixed order (deterministic, and plain stores run ~4-5x
// the chip's fp32-atomic byte rate).  With a single split the block adds its
// tile into dW directly.  Each thread's im2col column (r, s, c) is fixed for
// the whole kernel and the per-row (n, p, q) coordinates advance by
// single-carry increments, so the gather costs no integer divisions in the
// main loop.
#include "common.h"
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <vector>
#include <mutex>

namespace pmd {

struct WgradArgs {
  const bf16_t* dy;  // [M][K]
  const bf16_t* x;   // NHWC [N, H, W, C]
  float* dw;         // [K][Kg] fp32 accumulation target
  float* ws;         // [splits][K][Kg] partials, or nullptr when splits == 1
  int N, H, W, C, log2C;
  int P, Q, K, R, S, stride, pad;
  int M, Kg;
  int chunks_per_split;  // 64-row chunks per block
};

constexpr int BR = 64;  // reduction rows per stage

template <int ROWB>
__device__ __forceinline__ int swz(int row) {
  // 256-B and 512-B rows: both put every row at the same bank offset, so the same
  // 3-bit window XOR spreads the 8 rows of a transposed read over 8 windows
  if (ROWB >= 256) return (row & 3) | (((row >> 3) & 1) << 2);
  return ((row >> 1) & 1) | ((row >> 2) & 2);  // 128-byte rows
}

// byte offset of element `col` of `row` in a [BR][COLS] bf16 tile with 32-B-window swizzle
template <int COLS>
__device__ __forceinline__ int toff(int row, int col) {
  constexpr int ROWB = COLS * 2;
  const int byte = col * 2;
  return row * ROWB + (((byte >> 5) ^ swz<ROWB>(row)) << 5) + (byte & 31);
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int A_BYTES = BR * BM * 2, B_BYTES = BR * BN * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesM = a.K / BM + (a.K % BM != 0);
  const int tilesN = (a.Kg + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles;
  const int t = L % tiles;
  const int k0 = (t / tilesN) * BM;
  const int g0 = (t % tilesN) * BN;
  const int mbeg = split * a.chunks_per_split * BR;
  if (mbeg >= a.M) return;
  int mend = mbeg + a.chunks_per_split * BR;
  if (mend > a.M) mend = a.M;
  const int nchunks = (mend - mbeg + BR - 1) / BR;

  // dY loader: CA chunks (16 B) per row, RA rows per pass
  constexpr int CA = BM / 8, RA = 256 / CA, PA = BR / RA;
  const int a_col = (tid % CA) * 8;
  const int a_row = tid / CA;
  const bool a_colok = k0 + a_col < a.K;
  // X loader: CB chunks per row
  constexpr int CB = BN / 8, RB = 256 / CB, PB = BR / RB;
  const int b_col = (tid % CB) * 8;
  const int b_row = tid / CB;
  const int kg = g0 + b_col;
  const bool b_colok = kg < a.Kg;
  const int tap = kg >> a.log2C;
  const int cch = kg & (a.C - 1);
  const int rr = tap / a.S, ss = tap - (tap / a.S) * a.S;
  // per-pass row coordinates (n, p, q) of m = mbeg + b_row + RB*i, advanced by BR per chunk
  int bn_[PB], bp_[PB], bq_[PB];
  const int pq = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int m = mbeg + b_row + RB * i;
    const int n = m / pq, rem = m - n * pq;
    bn_[i] = n;
    bp_[i] = rem / a.Q;
    bq_[i] = rem - bp_[i] * a.Q;
  }
  const int dq = BR % a.Q, dp = (BR / a.Q) % a.P, dn = BR / pq;

  uint4 ra[PA], rb[PB];
  auto load = [&](int ch) {
    const int mb = mbeg + ch * BR;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int m = mb + a_row + RA * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_colok && m < mend) v = *reinterpret_cast<const uint4*>(a.dy + (size_t)m * a.K + k0 + a_col);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int m = mb + b_row + RB * i;
      const int ih = bp_[i] * a.stride - a.pad + rr;
      const int iw = bq_[i] * a.stride - a.pad + ss;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b_colok && m < mend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) {
        const size_t pix = ((size_t)bn_[i] * a.H + ih) * a.W + iw;
        v = *reinterpret_cast<const uint4*>(a.x + (pix << a.log2C) + cch);
      }
      rb[i] = v;
      // advance this row by BR (single-carry; dq < Q, dp < P)
      int q = bq_[i] + dq, c1 = q >= a.Q;
      q -= c1 ? a.Q : 0;
      int p = bp_[i] + dp + c1, c2 = p >= a.P;
      p -= c2 ? a.P : 0;
      bq_[i] = q;
      bp_[i] = p;
      bn_[i] += dn + c2;
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < PA; ++i)
      *reinterpret_cast<uint4*>(As + toff<BM>(a_row + RA * i, a_col)) = ra[i];
#pragma unroll
    for (int i = 0; i < PB; ++i)
      *reinterpret_cast<uint4*>(Bs + toff<BN>(b_row + RB * i, b_col)) = rb[i];
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(0);
  store(0);
  __syncthreads();

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int buf = ch & 1;
    if (ch + 1 < nchunks) load(ch + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BR / 32; ++ks) {
      bf16x8 af[MI], bfg[NI];
      const int r0 = ks * 32 + 8 * g + q4;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wm * (BM / 2) + i * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + toff<BM>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + toff<BM>(r0 + 4, col)));
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wn * (BN / 2) + j * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + toff<BN>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + toff<BN>(r0 + 4, col)));
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfg[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    if (ch + 1 < nchunks) store(buf ^ 1);
    __syncthreads();
  }

  // epilogue: partial tile -> workspace slice of this split (or += dW when unsplit)
  float* dst = a.ws ? a.ws + (size_t)split * a.K * a.Kg : a.dw;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + e;
        const int gg = g0 + wn * (BN / 2) + j * 16 + (lane & 15);
        if (k < a.K && gg < a.Kg) {
          float* p = dst + (size_t)k * a.Kg + gg;
          if (a.ws)
            *p = acc[i][j][e];
          else
            *p += acc[i][j][e];
        }
      }
}

// LDS-DMA variant: both operand tiles are copied global->LDS with
// global_load_lds_dwordx4 (no VGPR round trip, no ds_write pass) into an NST-deep
// ring of BR-row stages, ONE barrier per stage (publishes stage ch and retires the
// reads of the buffer the next DMA overwrites), counted vmcnt so NST-2 stages stay
// in flight across it.  The DMA writes lane-linearly, and the thread->(row, 16-B
// chunk) map of the register path is already lane-linear per wave (a wave covers
// 1024 contiguous bytes = whole rows), so the 32-B-window swizzle moves to the
// SOURCE: the thread at physical chunk p of a row loads logical window
// (p >> 1) ^ swz(row).  swz only depends on row bits 0..3 and every pass adds a
// multiple of 16 rows, so each thread's logical column (hence its im2col tap and
// channel) stays fixed for the whole kernel, exactly as on the register path.
__device__ __attribute__((aligned(16))) unsigned char g_wzero16[64];

template <int N>
__device__ __forceinline__ void wg_wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, int BN, int BRD, int NST, int WM = 2, int WN = 2>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_wgrad_dma_kernel(WgradArgs a) {
  constexpr int NT = 64 * WM * WN;
  constexpr int MI = BM / (16 * WM), NI = BN / (16 * WN);
  constexpr int A_BYTES = BRD * BM * 2, B_BYTES = BRD * BN * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tilesM = a.K / BM + (a.K % BM != 0);
  const int tilesN = (a.Kg + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles;
  const int t = L % tiles;
  const int k0 = (t / tilesN) * BM;
  const int g0 = (t % tilesN) * BN;
  const int mbeg = split * a.chunks_per_split * BR;  // split plan is in BR=64-row chunks
  if (mbeg >= a.M) return;
  int mend = mbeg + a.chunks_per_split * BR;
  if (mend > a.M) mend = a.M;
  const int nchunks = (mend - mbeg + BRD - 1) / BRD;

  constexpr int CA = BM / 8, RA = NT / CA, PA = BRD / RA;
  constexpr int CB = BN / 8, RB = NT / CB, PB = BRD / RB;
  static_assert(PA >= 1 && PB >= 1 && RA % 16 == 0 && RB % 16 == 0, "DMA wgrad tile shape");
  static_assert(NST * STAGE <= 160 * 1024, "exceeds the 160 KiB LDS of a CU");
  constexpr int LPT = PA + PB;  // DMA instructions per thread per stage
  const int a_row = tid / CA, b_row = tid / CB;
  const int a_pc = tid % CA, b_pc = tid % CB;  // physical 16-B chunk in the row
  const int a_col = ((((a_pc >> 1) ^ swz<BM * 2>(a_row)) << 1) | (a_pc & 1)) * 8;
  const int b_col = ((((b_pc >> 1) ^ swz<BN * 2>(b_row)) << 1) | (b_pc & 1)) * 8;
  const bool a_colok = k0 + a_col < a.K;
  const int kg = g0 + b_col;
  const bool b_colok = kg < a.Kg;
  const int tap = b_colok ? (kg >> a.log2C) : 0;
  const int cch = kg & (a.C - 1);
  const int rr = tap / a.S, ss = tap - (tap / a.S) * a.S;
  int bn_[PB], bp_[PB], bq_[PB];
  const int pq = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int m = mbeg + b_row + RB * i;
    const int n = m / pq, rem = m - n * pq;
    bn_[i] = n;
    bp_[i] = rem / a.Q;
    bq_[i] = rem - bp_[i] * a.Q;
  }
  const int dq = BRD % a.Q, dp = (BRD / a.Q) % a.P, dn = BRD / pq;
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);

  auto load = [&](int ch, int buf) {
    const int mb = mbeg + ch * BRD;
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int m = mb + a_row + RA * i;
      const void* src = (a_colok && m < mend) ? (const void*)(a.dy + (size_t)m * a.K + k0 + a_col)
                                             : (const void*)g_wzero16;
      char* dst = As + (RA * i) * (BM * 2) + wid_s * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int m = mb + b_row + RB * i;
      const int ih = bp_[i] * a.stride - a.pad + rr;
      const int iw = bq_[i] * a.stride - a.pad + ss;
      const bool ok = b_colok && m < mend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const size_t pix = ((size_t)bn_[i] * a.H + ih) * a.W + iw;
      const void* src = ok ? (const void*)(a.x + (pix << a.log2C) + cch) : (const void*)g_wzero16;
      char* dst = Bs + (RB * i) * (BN * 2) + wid_s * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      int q = bq_[i] + dq, c1 = q >= a.Q;
      q -= c1 ? a.Q : 0;
      int p = bp_[i] + dp + c1, c2 = p >= a.P;
      p -= c2 ? a.P : 0;
      bq_[i] = q;
      bp_[i] = p;
      bn_[i] += dn + c2;
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BRD / 32; ++ks) {
      bf16x8 af[MI], bfg[NI];
      const int r0 = ks * 32 + 8 * g + q4;
      typedef __attribute__((ext_vector_type(8))) short s16x8;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wm * (BM / WM) + i * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + toff<BM>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + toff<BM>(r0 + 4, col)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wn * (BN / WN) + j * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + toff<BN>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + toff<BN>(r0 + 4, col)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfg[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nchunks) load(s, s);
  for (int ch = 0; ch < nchunks; ++ch) {
    const int rem = min(NST - 2, nchunks - 1 - ch);
    if constexpr (NST >= 4) {
      if (rem >= 2) wg_wait_vmcnt<2 * LPT>();
      else if (rem == 1) wg_wait_vmcnt<LPT>();
      else wg_wait_vmcnt<0>();
    } else if constexpr (NST == 3) {
      if (rem >= 1) wg_wait_vmcnt<LPT>();
      else wg_wait_vmcnt<0>();
    } else {
      wg_wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ch + NST - 1 < nchunks) load(ch + NST - 1, (ch + NST - 1) % NST);
    compute(ch % NST);
  }

  float* dst = a.ws ? a.ws + (size_t)split * a.K * a.Kg : a.dw;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + e;
        const int gg = g0 + wn * (BN / WN) + j * 16 + (lane & 15);
        if (k < a.K && gg < a.Kg) {
          float* p = dst + (size_t)k * a.Kg + gg;
          if (a.ws)
            *p = acc[i][j][e];
          else
            *p += acc[i][j][e];
        }
      }
}

// dW[i] += sum_s ws[s][i].  blockIdx.y = split group of <= kSplitGroup slices:
// one group -> plain read-modify-write in fixed order (deterministic); several
// groups (tiny outputs with hundreds of splits) -> one fp32 atomic per group.
constexpr int kSplitGroup = 32;
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, int splits,
                                    long long n4) {
  const int s0 = blockIdx.y * kSplitGroup;
  const int s1 = s0 + kSplitGroup < splits ? s0 + kSplitGroup : splits;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int s = s0; s < s1; ++s) {
      const float4 v = reinterpret_cast<const float4*>(ws)[(long long)s * n4 + i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    if (gridDim.y == 1) {
      float4 d = reinterpret_cast<float4*>(dw)[i];
      d.x += acc.x;
      d.y += acc.y;
      d.z += acc.z;
      d.w += acc.w;
      reinterpret_cast<float4*>(dw)[i] = d;
    } else {
      float* p = dw + 4 * i;
      atomicAdd(p, acc.x);
      atomicAdd(p + 1, acc.y);
      atomicAdd(p + 2, acc.z);
      atomicAdd(p + 3, acc.w);
    }
  }
}

static int ilog2w(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// Total blocks the split-K plan aims for, by filter size.  Isolated per-layer timing
// (profiles/conv_bench_r01_wgrad_blocks.txt) favoured 512 (1x1) / 1024 (3x3) / 2048
// (7x7 stem); in the step, where the wgrads run on the side stream next to the
// main-stream kernels, fewer, longer splits win (less fp32 partial + reduce traffic,
// fewer co-resident blocks): 384 / 384 measured +0.9% step over 512 / 1024 in three
// interleaved A/B sessions (profiles/wgrad_blocks_step_ab_r02.txt).  Overridable:
// PMD_WGRAD_BLOCKS_R1 / _R3 / _R7.
static int env_int(const char* k, int dflt) {
  const char* e = getenv(k);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}
static int wgrad_target_blocks(int R) {
  static const int t1 = env_int("PMD_WGRAD_BLOCKS_R1", 384);
  static const int t3 = env_int("PMD_WGRAD_BLOCKS_R3", 384);
  static const int t7 = env_int("PMD_WGRAD_BLOCKS_R7", 2048);
  return R == 1 ? t1 : (R <= 3 ? t3 : t7);
}

// Variant (conv_wgrad_set_impl or PMD_WGRAD_IMPL): 0 register staging
// (2 stages), 1 LDS-DMA 64-row stages x2 (default: autotuned per shape over
// {0, 1, 4, 5}), 2 LDS-DMA 32-row x4, 3 LDS-DMA 64-row x3, 4 8-wave 256x256
// LDS-DMA 64-row x2, 5 8-wave 256x128 (4/5 need K >= 256; else 1 is used).
static int g_wgrad_impl = -1;
void conv_wgrad_set_impl(int impl) { g_wgrad_impl = impl; }
static int wgrad_impl() {
  if (g_wgrad_impl < 0) {
    const char* e = getenv("PMD_WGRAD_IMPL");
    g_wgrad_impl = (e && e[0] >= '0' && e[0] <= '5') ? e[0] - '0' : 1;
  }
  return g_wgrad_impl;
}

// Per-shape autotuning of the staging variant (register staging vs LDS-DMA),
// like the conv fwd/dgrad tuner: timed on the live operands outside graph
// capture, the partial tile written to a scratch dW so nothing is accumulated
// twice into the caller's gradient.  PMD_WGRAD_AUTOTUNE=0 disables it.
struct WgradKey {
  int v[11];
  bool operator<(const WgradKey& o) const {
    for (int i = 0; i < 11; ++i)
      if (v[i] != o.v[i]) return v[i] < o.v[i];
    return false;
  }
};
static std::map<WgradKey, int> g_wtune;
static std::mutex g_wtune_mu;

// flat table export/import: 11 key fields + the chosen variant per entry
std::vector<int> wgrad_autotune_export() {
  std::lock_guard<std::mutex> lk(g_wtune_mu);
  std::vector<int> out;
  for (const auto& kv : g_wtune) {
    out.insert(out.end(), kv.first.v, kv.first.v + 11);
    out.push_back(kv.second);
  }
  return out;
}
int wgrad_autotune_import(const std::vector<int>& flat) {
  if (flat.size() % 12) return -1;
  std::lock_guard<std::mutex> lk(g_wtune_mu);
  for (size_t i = 0; i < flat.size(); i += 12) {
    WgradKey k;
    for (int j = 0; j < 11; ++j) k.v[j] = flat[i + j];
    g_wtune[k] = flat[i + 11];
  }
  return (int)(flat.size() / 12);
}
void wgrad_autotune_clear() {
  std::lock_guard<std::mutex> lk(g_wtune_mu);
  g_wtune.clear();
}
static bool wgrad_autotune_on() {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("PMD_WGRAD_AUTOTUNE");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on == 1;
}

// Output tile of a staging variant: 4-wave 128-row tiles (BM 64 for K = 64),
// 8-wave 256x256 / 256x128 tiles (K >= 256).  The split-K plan aims at
// target blocks; an 8-wave block is one per CU and does 2-4x the work of a
// 128-row one, so it aims at a quarter / half as many (but >= 256).
struct WgradCfg {
  int impl, BM, BN, target;
};

static bool wgrad_cfg_ok(int impl, const WgradArgs& a) {
  if (impl == 4) return a.K >= 256 && a.Kg >= 256;
  if (impl == 5) return a.K >= 256;
  return true;
}

static WgradCfg wgrad_cfg(int impl, const WgradArgs& a) {
  const int t = wgrad_target_blocks(a.R);
  if (impl == 4) return {4, 256, 256, t / 4 > 256 ? t / 4 : 256};
  if (impl == 5) return {5, 256, 128, t / 2 > 256 ? t / 2 : 256};
  return {impl, a.K == 64 ? 64 : 128, 128, t};
}

static void plan(const WgradArgs& a, const WgradCfg& cfg, int* splits_out, int* cps_out) {
  const int tiles = ((a.K + cfg.BM - 1) / cfg.BM) * ((a.Kg + cfg.BN - 1) / cfg.BN);
  const int chunks = (a.M + BR - 1) / BR;
  int splits = (cfg.target + tiles - 1) / tiles;
  const int max_splits = (chunks + 3) / 4;
  if (splits > max_splits) splits = max_splits;
  // keep the partial workspace bounded (<= 96 MiB)
  const long long per = (long long)a.K * a.Kg * 4;
  while (splits > 1 && per * splits > (96ll << 20)) --splits;
  if (splits < 1) splits = 1;
  const int cps = (chunks + splits - 1) / splits;
  *cps_out = cps;
  *splits_out = (chunks + cps - 1) / cps;
}

// One full weight gradient with variant `impl`: split-K plan, kernel, split reduce.
static void wgrad_run(int impl, WgradArgs a, float* ws, hipStream_t st) {
  const WgradCfg cfg = wgrad_cfg(impl, a);
  int splits, cps;
  plan(a, cfg, &splits, &cps);
  a.chunks_per_split = cps;
  a.ws = splits > 1 ? ws : nullptr;
  const int tiles = ((a.K + cfg.BM - 1) / cfg.BM) * ((a.Kg + cfg.BN - 1) / cfg.BN);
  const dim3 grid(tiles * splits);
  const bool k64 = a.K == 64;
  switch (impl) {
    case 0:
      if (k64) hipLaunchKernelGGL((conv_wgrad_kernel<64, 128>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_kernel<128, 128>), grid, dim3(256), 0, st, a);
      break;
    case 2:  // DMA, 32-row stages, 4-deep ring
      if (k64) hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 128, 32, 4>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 128, 32, 4>), grid, dim3(256), 0, st, a);
      break;
    case 3:  // DMA, 64-row stages, 3-deep ring (1 block/CU at BM=128)
      if (k64) hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 128, 64, 3>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 128, 64, 3>), grid, dim3(256), 0, st, a);
      break;
    case 4:  // 8 waves, 256x256, DMA 64-row x2
      hipLaunchKernelGGL((conv_wgrad_dma_kernel<256, 256, 64, 2, 2, 4>), grid, dim3(512), 0, st, a);
      break;
    case 5:  // 8 waves, 256x128, DMA 64-row x2
      hipLaunchKernelGGL((conv_wgrad_dma_kernel<256, 128, 64, 2, 4, 2>), grid, dim3(512), 0, st, a);
      break;
    default:  // 1: DMA, 64-row stages, 2-deep ring
      if (k64) hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 128, 64, 2>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 128, 64, 2>), grid, dim3(256), 0, st, a);
      break;
  }
  if (splits > 1) {
    const long long n4 = (long long)a.K * a.Kg / 4;
    const int groups = (splits + kSplitGroup - 1) / kSplitGroup;
    long long b = (n4 + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((int)b, groups), dim3(256), 0, st, a.ws, a.dw, splits, n4);
  }
}

static int wgrad_tune(const WgradArgs& a0, float* ws, hipStream_t st) {
  WgradArgs a = a0;
  static float* scratch = nullptr;
  static size_t scratch_n = 0;
  const size_t need = (size_t)a.K * a.Kg;
  if (need > scratch_n) {
    if (scratch) (void)hipFree(scratch);
    if (hipMalloc(&scratch, sizeof(float) * need) != hipSuccess) return -1;
    scratch_n = need;
  }
  a.dw = scratch;  // kernel (+ split reduce) accumulate into a scratch dW, not the caller's
  static hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!e0) {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
  }
  int best = -1;
  float best_ms = 1e30f;
  for (int c : {0, 1, 4, 5}) {
    if (!wgrad_cfg_ok(c, a)) continue;
    wgrad_run(c, a, ws, st);
    float t = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0, st);
      wgrad_run(c, a, ws, st);
      (void)hipEventRecord(e1, st);
      if (hipEventSynchronize(e1) != hipSuccess) return -1;
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      t = ms < t ? ms : t;
    }
    if (t < best_ms) {
      best_ms = t;
      best = c;
    }
  }
  const char* lg = getenv("PMD_CONV_AUTOTUNE_LOG");
  if (lg && lg[0] == '1')
    fprintf(stderr, "[pmd autotune] wgrad N=%d H=%d W=%d C=%d K=%d R=%d s=%d: impl %d (%.1f us)\n", a.N,
            a.H, a.W, a.C, a.K, a.R, a.stride, best, best_ms * 1e3f);
  return best;
}

static void fill_args(WgradArgs& a, int N, int H, int W, int C, int P, int Q, int K, int R, int S,
                      int stride, int pad) {
  a.N = N;
  a.H = H;
  a.W = W;
  a.C = C;
  a.log2C = ilog2w(C);
  a.P = P;
  a.Q = Q;
  a.K = K;
  a.R = R;
  a.S = S;
  a.stride = stride;
  a.pad = pad;
  a.M = (int)((long long)N * P * Q);
  a.Kg = R * S * C;
}

// workspace slices the caller must provide: the max over every variant the
// launcher may pick (the autotuner chooses at launch time)
int conv_wgrad_splits(int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride,
                      int pad) {
  WgradArgs a;
  fill_args(a, N, H, W, C, P, Q, K, R, S, stride, pad);
  int best = 1;
  for (int impl : {0, 1, 4, 5}) {
    if (!wgrad_cfg_ok(impl, a)) continue;
    int splits, cps;
    plan(a, wgrad_cfg(impl, a), &splits, &cps);
    best = splits > best ? splits : best;
  }
  return best;
}

int conv_wgrad_launch(const bf16_t* dy, const bf16_t* x, float* dw, float* ws, int N, int H, int W,
                      int C, int P, int Q, int K, int R, int S, int stride, int pad, hipStream_t st) {
  if (C % 8 != 0 || (C & (C - 1)) != 0) return 1;
  if (K % 64 != 0) return 2;
  if ((long long)N * P * Q >= (1ll << 31)) return 4;
  WgradArgs a;
  a.dy = dy;
  a.x = x;
  a.dw = dw;
  fill_args(a, N, H, W, C, P, Q, K, R, S, stride, pad);
  if (!ws && conv_wgrad_splits(N, H, W, C, P, Q, K, R, S, stride, pad) > 1) return 5;
  int impl = wgrad_impl();
  if (!wgrad_cfg_ok(impl, a)) impl = 1;
  if (impl == 1 && wgrad_autotune_on()) {
    const WgradKey key{{N, H, W, C, P, Q, K, R, S, stride, pad}};
    int c = -1;
    {
      std::lock_guard<std::mutex> lk(g_wtune_mu);
      auto it = g_wtune.find(key);
      if (it != g_wtune.end()) c = it->second;
    }
    if (c < 0) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(st, &cs);
      if (cs == hipStreamCaptureStatusNone) {
        c = wgrad_tune(a, ws, st);
        if (c >= 0) {
          std::lock_guard<std::mutex> lk(g_wtune_mu);
          g_wtune[key] = c;
        }
      }
    }
    if (c >= 0) impl = c;
  }
  wgrad_run(impl, a, ws, st);
  return 0;
}

}  // namespace pmd
