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
#include "stem_tile.h"
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
  // operands read by a single tile column / row: non-temporal (see glds16)
  const bool dy_once = tilesN == 1, x_once = tilesM == 1 && a.R == 1 && a.S == 1;

  uint4 ra[PA], rb[PB];
  auto load = [&](int ch) {
    const int mb = mbeg + ch * BR;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int m = mb + a_row + RA * i;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_colok && m < mend) v = ld16c<2>(a.dy + (size_t)m * a.K + k0 + a_col, dy_once);
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
        v = ld16c<4>(a.x + (pix << a.log2C) + cch, x_once);
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
            stfn<NT_WS_ST>(p, acc[i][j][e]);
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
  // an operand read by a single tile column (dY) / row (X) of this split: non-temporal
  // (X of a 3x3 wgrad is re-gathered for every tap: kept cacheable)
  const bool dy_once = tilesN == 1, x_once = tilesM == 1 && a.R == 1 && a.S == 1;

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
      glds16<2>(src, dst, dy_once);
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
      glds16<4>(src, dst, x_once);
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
            stfn<NT_WS_ST>(p, acc[i][j][e]);
          else
            *p += acc[i][j][e];
        }
      }
}

// ---------------------------------------------------------------------------
// FP8 wgrad (BASELINE config 5): dY as OCP e5m2 (bf8) x X as e4m3 on the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 (A format bf8, B format fp8, unit block scales):
// 128 reduction rows (m) per MFMA, twice the bf16 MFMA rate per clock, and half the
// operand bytes of the bf16 kernel.  Both operands arrive m-major ([m][channels],
// 1 B per element), are copied to LDS by LDS-DMA in natural row order (128-row
// stages, 2-deep ring, one barrier per stage), and each MFMA fragment -- 32
// consecutive m of ONE column per lane -- is read with four ds_read_b64_tr_b8
// (per 16-lane group: an 8-row x 16-column byte block delivered column-major, lane j
// receiving column j of the 8 rows).  The 16-B chunk of a 128-B LDS row is XOR-
// swizzled with row bits 0..2 and 5 (on the DMA SOURCE address, as the bf16 DMA
// kernel), so the 8 rows x 2 lane-groups of a 32-lane half hit 16 distinct 4-bank
// slots.  Epilogue: acc / (s_dy * s_x) into the split workspace (or += dW).
struct WgradF8Args {
  const uint8_t* dy;  // e5m2 [M][K]
  const uint8_t* x;   // e4m3 NHWC [N,H,W,C]
  const float* sdy;   // device scalars the operands were quantised with
  const float* sx;
  float* dw;
  float* ws;
  int N, H, W, C, log2C, P, Q, K, R, S, stride, pad, M, Kg;
  int chunks_per_split;  // 128-row chunks per block
};

__device__ __forceinline__ int swz8(int row) { return (row & 7) ^ ((row >> 5) & 1); }
typedef __attribute__((ext_vector_type(8))) int i32x8;

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_wgrad_fp8_kernel(WgradF8Args a) {
  constexpr int BRF = 128;  // reduction rows per stage = one MFMA K
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int CA = BM / 16, CB = BN / 16;  // 16-B chunks per row
  constexpr int RA = 256 / CA, RB = 256 / CB;  // rows per block-wide DMA round
  constexpr int PA = BRF / RA, PB = BRF / RB;
  constexpr int A_BYTES = BRF * BM, B_BYTES = BRF * BN, STAGE = A_BYTES + B_BYTES;
  constexpr int LPT = PA + PB;
  static_assert(RA % 64 == 0 || RA == 32, "DMA rows per round");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tilesM = (a.K + BM - 1) / BM, tilesN = (a.Kg + BN - 1) / BN;
  const int tiles = tilesM * tilesN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int split = L / tiles, t = L % tiles;
  const int k0 = (t / tilesN) * BM, g0 = (t % tilesN) * BN;
  const int mbeg = split * a.chunks_per_split * BRF;
  if (mbeg >= a.M) return;
  const int mend = min(mbeg + a.chunks_per_split * BRF, a.M);
  const int nchunks = (mend - mbeg + BRF - 1) / BRF;

  // DMA map: thread -> (row tid / C? + R? i, physical chunk tid % C?); the logical chunk
  // (source column) is the physical one XOR swz8(row), fixed per (thread, instruction)
  const int a_row0 = tid / CA, a_pc = tid % CA;
  const int b_row0 = tid / CB, b_pc = tid % CB;
  int a_col[PA], b_tap_r[PB], b_tap_s[PB], b_c[PB];
  bool a_colok[PA], b_colok[PB];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = a_row0 + RA * i;
    a_col[i] = ((a_pc ^ swz8(row)) & (CA - 1)) * 16;
    a_colok[i] = k0 + a_col[i] < a.K;
  }
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int row = b_row0 + RB * i;
    const int g = g0 + ((b_pc ^ swz8(row)) & (CB - 1)) * 16;
    b_colok[i] = g < a.Kg;
    const int tap = b_colok[i] ? (g >> a.log2C) : 0;
    b_tap_r[i] = tap / a.S;
    b_tap_s[i] = tap - b_tap_r[i] * a.S;
    b_c[i] = g & (a.C - 1);
  }
  // per-instruction row coordinates (n, p, q) of m = mbeg + row, advanced by BRF per stage
  int bn_[PB], bp_[PB], bq_[PB];
  const int pq = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int m = mbeg + b_row0 + RB * i;
    const int n = m / pq, rem = m - n * pq;
    bn_[i] = n;
    bp_[i] = rem / a.Q;
    bq_[i] = rem - bp_[i] * a.Q;
  }
  const int dq = BRF % a.Q, dp = (BRF / a.Q) % a.P, dn = BRF / pq;
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);

  auto load = [&](int ch, int buf) {
    const int mb = mbeg + ch * BRF;
    uint8_t* As = smem + buf * STAGE;
    uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int m = mb + a_row0 + RA * i;
      const void* src = (a_colok[i] && m < mend) ? (const void*)(a.dy + (size_t)m * a.K + k0 + a_col[i])
                                                 : (const void*)g_wzero16;
      uint8_t* dst = As + (RA * i) * BM + wid_s * 1024;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int m = mb + b_row0 + RB * i;
      const int ih = bp_[i] * a.stride - a.pad + b_tap_r[i];
      const int iw = bq_[i] * a.stride - a.pad + b_tap_s[i];
      const bool ok = b_colok[i] && m < mend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const size_t pix = ((size_t)bn_[i] * a.H + ih) * a.W + iw;
      const void* src = ok ? (const void*)(a.x + (pix << a.log2C) + b_c[i]) : (const void*)g_wzero16;
      uint8_t* dst = Bs + (RB * i) * BN + wid_s * 1024;
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

  // fragment read: lane j of 16-lane group g4 supplies row 32 g4 + 8 t + (j >> 1), byte
  // half (j & 1) of the column block's 16-B chunk, and receives column j of those 8 rows
  const int g4 = lane >> 4, jl = lane & 15;
  typedef __attribute__((ext_vector_type(2))) int v2i;
  auto frag = [&](const uint8_t* base, int rowb, int col) {
    // col: first column of the 16-column block (a multiple of 16); rowb: row bytes
    i32x8 v;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int row = 32 * g4 + 8 * tt + (jl >> 1);
      const int off = row * rowb + ((((col >> 4) ^ swz8(row)) & (rowb / 16 - 1)) << 4) + (jl & 1) * 8;
      const v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(base + off));
      v[2 * tt] = r[0];
      v[2 * tt + 1] = r[1];
    }
    return v;
  };
  auto compute = [&](int buf) {
    const uint8_t* As = smem + buf * STAGE;
    const uint8_t* Bs = As + A_BYTES;
    i32x8 af[MI], bfg[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) af[i] = frag(As, BM, wm * (BM / 2) + i * 16);
#pragma unroll
    for (int j = 0; j < NI; ++j) bfg[j] = frag(Bs, BN, wn * (BN / 2) + j * 16);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfg[j], acc[i][j], 1, 0, 0, 127, 0,
                                                                      127);
  };

  load(0, 0);
  for (int ch = 0; ch < nchunks; ++ch) {
    wg_wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ch + 1 < nchunks) load(ch + 1, (ch + 1) & 1);
    compute(ch & 1);
  }
  (void)LPT;

  const float ds = 1.f / (a.sdy[0] * a.sx[0]);
  float* dst = a.ws ? a.ws + (size_t)split * a.K * a.Kg : a.dw;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm * (BM / 2) + i * 16 + g4 * 4 + e;
        const int gg = g0 + wn * (BN / 2) + j * 16 + jl;
        if (k < a.K && gg < a.Kg) {
          float* p = dst + (size_t)k * a.Kg + gg;
          if (a.ws)
            stfn<NT_WS_ST>(p, acc[i][j][e] * ds);
          else
            *p += acc[i][j][e] * ds;
        }
      }
}

// ---------------------------------------------------------------------------
// HALO wgrad: stride-1 convolutions with K == 64 output channels whose im2col is
// mostly redundancy -- the ImageNet stem as a 4x4 conv over the space-to-depth
// image (16 taps x 16 channels: every input pixel appears in 16 im2col columns)
// and the 64-channel 3x3 convs (9 taps).  The generic kernels gather every
// im2col row from L2 (9-16x the activation bytes through the L2->CU path, which
// bounds them: 13-14 % MFMA, 1.2 TB/s HBM, profiles/pmc_wgrad_layers_r03.txt).
//
// Here a block owns a BAND of PB whole output rows of one image (PB*Q = up to
// 224 reduction rows = 7 MFMA k-steps) at a time and stages, per band,
//   * the band's input rows + halo (PB+R-1 rows x Q+S-1 pixels, zero-padded)
//     ONCE, as C/8 "octet planes" [plane][pixel][8 channels] (16 B per pixel per
//     plane -- one LDS-DMA chunk, contiguous in global memory), and
//   * the band's dY rows [m][64] (32-B-window XOR swizzle, as the DMA kernel),
// both by LDS-DMA into a 2-stage ring (the next band's DMA flies while this
// band's MFMAs run).  The output tile is ALL K=64 x Kg columns (Kg = R*S*C <= 576:
// 16 NI columns per wave), so the halo is read from L2 once per band instead of
// once per tap.  B fragments (8 consecutive m of 16 consecutive kg) come straight
// out of the halo with ds_read_b64_tr_b16: for tap (r, s) and channel quad c the
// row address is  plane(c) + 16 * (rowpix(m) + r*HWp + s) + 8 * ((c >> 2) & 1),
// a per-lane constant per fragment plus a per-lane constant per k-step -- one add
// per read, no swizzle arithmetic.  A plane's pitch is 64 B mod 256, so the 8
// pixels x 2 planes x 2 halves a 32-lane read group touches tile the 64 banks.
struct HaloArgs {
  int PB;        // output rows per band
  int HWp;       // halo width  = Q + S - 1
  int HR;        // halo rows   = PB + R - 1
  int pitchC;    // 16-B chunks per octet plane (== 4 mod 16)
  int CO;        // octet planes = C / 8
  int bands_img; // bands per image = ceil(P / PB)
  int bands;     // N * bands_img
  int bpb;       // bands per block
};
constexpr int kHaloRows = 224;  // reduction rows per band buffer (7 k-steps)

template <int NI, int HCH>
__global__ __launch_bounds__(256, 1) void conv_wgrad_halo_kernel(WgradArgs a, HaloArgs h) {
  constexpr int KS = kHaloRows / 32;
  constexpr int HBYTES = HCH * 16;
  constexpr int DBYTES = kHaloRows * 128;  // [224][64] bf16
  constexpr int STAGE = HBYTES + DBYTES;
  constexpr int HPT = HCH / 256;           // halo DMA chunks per thread
  constexpr int DPT = kHaloRows * 8 / 256; // dY DMA chunks per thread
  static_assert(HCH % 256 == 0 && 2 * STAGE <= 160 * 1024, "halo wgrad LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  const int b0 = blockIdx.x * h.bpb;
  if (b0 >= h.bands) return;
  const int b1 = min(b0 + h.bpb, h.bands);

  // ---- per-thread DMA work lists (identical for every band)
  int hsrc[HPT];  // (plane << 20) | (halo row << 12) | halo col, -1 = unused chunk
#pragma unroll
  for (int t = 0; t < HPT; ++t) {
    const int L = t * 256 + wid * 64 + lane;
    const int o = L / h.pitchC, pix = L - o * h.pitchC;
    hsrc[t] = (o < h.CO && pix < h.HR * h.HWp) ? ((o << 20) | ((pix / h.HWp) << 12) | (pix % h.HWp)) : -1;
  }
  // dY chunk (row, physical 16-B chunk pc) of instruction t: row = 32 t + 8 wid + lane / 8
  const int d_pc = lane & 7;
  const int d_row0 = wid * 8 + (lane >> 3);
  const int d_col = ((((d_pc >> 1) ^ swz<128>(d_row0)) << 1) | (d_pc & 1)) * 8;

  auto load = [&](int band, int buf) {
    const int n = band / h.bands_img, pb = band - n * h.bands_img;
    const int p0 = pb * h.PB;
    const int rows = min(h.PB, a.P - p0) * a.Q;  // valid reduction rows of this band
    const size_t mrow0 = ((size_t)n * a.P + p0) * a.Q;
    char* Hs = smem + buf * STAGE;
    char* Ds = Hs + HBYTES;
#pragma unroll
    for (int t = 0; t < HPT; ++t) {
      const int e = hsrc[t];
      if (e >= 0) {
        const int o = e >> 20, hr = (e >> 12) & 0xff, hc = e & 0xfff;
        const int ih = p0 - a.pad + hr, iw = hc - a.pad;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const void* src = ok ? (const void*)(a.x + ((((size_t)n * a.H + ih) * a.W + iw) << a.log2C) + 8 * o)
                             : (const void*)g_wzero16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(Hs + (t * 256 + wid_s * 64) * 16),
                                         16, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < DPT; ++t) {
      const int row = t * 32 + d_row0;
      const void* src = row < rows ? (const void*)(a.dy + (mrow0 + row) * 64 + d_col) : (const void*)g_wzero16;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(Ds + (t * 256 + wid_s * 64) * 16),
                                       16, 0, 0);
    }
  };

  // ---- fragment address constants
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  int rofs[KS][2];  // per k-step and half: 16 * halo pixel of the row's tap (0, 0)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      const int mr = ks * 32 + 8 * g + q4 + 4 * hl;
      const int pr = mr / a.Q;
      rofs[ks][hl] = mr < h.PB * a.Q ? 16 * (pr * h.HWp + (mr - pr * a.Q)) : 0;
    }
  int cofs[NI];  // per fragment: plane + tap shift + half for this lane's channel quad
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int kgc = wid * (16 * NI) + j * 16 + 4 * p4;
    const int tap = kgc >> a.log2C, c = kgc & (a.C - 1);
    const int r = tap / a.S, s = tap - r * a.S;
    cofs[j] = (c >> 3) * h.pitchC * 16 + 16 * (r * h.HWp + s) + 8 * ((c >> 2) & 1);
  }

  f32x4 acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __attribute__((ext_vector_type(8))) short s16x8;
  auto compute = [&](int buf) {
    const char* Hs = smem + buf * STAGE;
    const char* Ds = Hs + HBYTES;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[4], bfg[NI];
      const int r0 = ks * 32 + 8 * g + q4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Ds + toff<64>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Ds + toff<64>(r0 + 4, col)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Hs + cofs[j] + rofs[ks][0]));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Hs + cofs[j] + rofs[ks][1]));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfg[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
  };

  load(b0, 0);
  for (int b = b0; b < b1; ++b) {
    wg_wait_vmcnt<0>();
    // publishes band b's stage AND retires every wave's reads of the other stage
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (b + 1 < b1) load(b + 1, (b + 1 - b0) & 1);
    compute((b - b0) & 1);
  }

  float* dst = a.ws ? a.ws + (size_t)blockIdx.x * 64 * a.Kg : a.dw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = i * 16 + (lane >> 4) * 4 + e;
        const int gg = wid * (16 * NI) + j * 16 + (lane & 15);
        float* p = dst + (size_t)k * a.Kg + gg;
        if (a.ws)
          stfn<NT_WS_ST>(p, acc[i][j][e]);
        else
          *p += acc[i][j][e];
      }
}

// The halo variant applies to stride-1 convs with K == 64, C in {16, 64}, Kg = 256
// (stem: 4x4 x 16) or 576 (3x3 x 64), and bands of whole rows that fit 224 rows.
static bool halo_cfg(const WgradArgs& a, HaloArgs* h, int* nich) {
  if (a.stride != 1 || a.K != 64 || !(a.C == 16 || a.C == 64)) return false;
  if (!(a.Kg == 256 || a.Kg == 576)) return false;
  if (a.Q > kHaloRows || a.Q < 7) return false;
  HaloArgs c;
  c.PB = kHaloRows / a.Q;
  if (c.PB > a.P) c.PB = a.P;
  c.HWp = a.Q + a.S - 1;
  c.HR = c.PB + a.R - 1;
  const int pix = c.HR * c.HWp;
  c.pitchC = pix + ((4 - pix % 16) + 16) % 16;
  c.CO = a.C / 8;
  const int hch_need = c.CO * c.pitchC;
  const int hch = a.Kg == 256 ? 1280 : 3072;
  if (hch_need > hch || c.HWp >= 4096 || c.HR >= 256) return false;
  // the halo must cover every tap of every band row: q + s - pad in [-pad, Q + S - 1 - pad)
  c.bands_img = (a.P + c.PB - 1) / c.PB;
  c.bands = a.N * c.bands_img;
  const int target = 256;  // one 150 KB block per CU
  const int blocks = c.bands < target ? c.bands : target;
  c.bpb = (c.bands + blocks - 1) / blocks;
  *h = c;
  *nich = a.Kg == 256 ? 4 : 9;
  return true;
}

static int halo_splits(const HaloArgs& h) { return (h.bands + h.bpb - 1) / h.bpb; }

// ---------------------------------------------------------------------------
// Fused ImageNet-stem backward: the max-pool + BatchNorm(+ReLU) backward elementwise pass
// (stem.hip stem_pool_bwd_elemt_kernel: dy = a * dz + b * y + c, dz = the pooled gradient
// routed to each window's argmax, gated by the ReLU of BN(y)) computes each band's dY rows
// straight into the halo weight gradient's dY stage (same swizzled [224][64] layout the
// LDS-DMA fills in conv_wgrad_halo_kernel), so the [N,112,112,64] stem gradient is never
// written nor read back: per step 2 x 411 MB of HBM traffic and one launch less at the end
// of the backward's critical path.  Band b = (image n, pooled row pb) = output rows 2 pb,
// 2 pb + 1 (the halo plan's 2-row bands of the 112-wide stem output), whose candidate windows
// are pooled rows pb and pb + 1, staged in LDS.  The next band's y rows, pooled rows and halo
// are in flight while this band's MFMAs run.
struct StemDyArgs {
  const bf16_t* dout;   // pooled gradient [N, P2, Q2, 64]
  const uint8_t* arg;   // window argmax taps [N, P2, Q2, 64]
  const bf16_t* y;      // stem conv output = BN input [N, P, Q, 64]
  const float* params;  // BN [4][64]: mean, invstd, scale, shift
  const float* gamma;   // [64]
  const float* red;     // [2][64] global sums of dz, dz * xhat
  const float* count;   // [1] global element count per channel, or null: count_h
  float count_h;
  int P2, Q2;
};
constexpr int kStemPoolMaxQ = 64;  // staged pooled row width (LDS)

__global__ __launch_bounds__(512, 1) void stem_wgrad_fused_kernel(WgradArgs a, HaloArgs h, StemDyArgs s) {
  // 8 waves (2 per SIMD): one wave's in-kernel dY production overlaps another's MFMAs; a
  // two-stage ring (the next band's halo / y / pooled rows in flight during this band's MFMAs)
  constexpr int NT = 512, NI = 2, HCH = 1280;
  constexpr int KS = kHaloRows / 32;
  constexpr int HBYTES = HCH * 16;
  constexpr int DBYTES = kHaloRows * 128;
  constexpr int STAGE = HBYTES + DBYTES;
  constexpr int HPT = (HCH + NT - 1) / NT;
  constexpr int YPT = (kHaloRows * 8 + NT - 1) / NT;        // dY chunks produced per thread (3.5)
  constexpr int PBYTES = 2 * kStemPoolMaxQ * 64 * 3;        // pooled gradient + taps of 2 rows
  constexpr int PPT = (2 * kStemPoolMaxQ * 8 + NT - 1) / NT;  // staged pooled chunks per thread
  static_assert(2 * STAGE + PBYTES <= 160 * 1024, "fused stem wgrad LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + PBYTES];
  bf16_t* dl = reinterpret_cast<bf16_t*>(smem + 2 * STAGE);
  uint8_t* al = reinterpret_cast<uint8_t*>(smem + 2 * STAGE + 2 * kStemPoolMaxQ * 64 * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);
  const int b0 = blockIdx.x * h.bpb;
  if (b0 >= h.bands) return;
  const int b1 = min(b0 + h.bpb, h.bands);

  // BN-backward coefficients of this thread's fixed 8-channel chunk (j & 7 == tid & 7)
  const int cc = tid & 7;
  float sc[8], sh[8], ca[8], cb[8], cz[8];
  {
    const float inv_cnt = 1.f / (s.count ? s.count[0] : s.count_h);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cc * 8 + k;
      const float mean = s.params[c], inv = s.params[64 + c], gm = s.gamma[c];
      sc[k] = s.params[128 + c];
      sh[k] = s.params[192 + c];
      stem_bwd_coeffs(gm, inv, mean, s.red[c] * inv_cnt, s.red[64 + c] * inv_cnt, ca[k], cb[k], cz[k]);
    }
  }
  int hsrc[HPT];
#pragma unroll
  for (int t = 0; t < HPT; ++t) {
    const int L = t * NT + wid * 64 + lane;
    const int o = L / h.pitchC, pix = L - o * h.pitchC;
    hsrc[t] = (L < HCH && o < h.CO && pix < h.HR * h.HWp) ? ((o << 20) | ((pix / h.HWp) << 12) | (pix % h.HWp)) : -1;
  }
  uint4 yv[YPT], pg[PPT];
  uint2 pa[PPT];
  // global loads of band `band`: halo (LDS-DMA into stage buf), y rows and pooled rows (registers)
  auto issue = [&](int band, int buf) {
    const int n = band / h.bands_img, pb = band - n * h.bands_img;
    const int p0 = pb * h.PB;
    char* Hs = smem + buf * STAGE;
#pragma unroll
    for (int t = 0; t < HPT; ++t) {
      const int e = hsrc[t];
      if (e >= 0) {
        const int o = e >> 20, hr = (e >> 12) & 0xff, hc = e & 0xfff;
        const int ih = p0 - a.pad + hr, iw = hc - a.pad;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const void* src = ok ? (const void*)(a.x + ((((size_t)n * a.H + ih) * a.W + iw) << a.log2C) + 8 * o)
                             : (const void*)g_wzero16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(Hs + (t * NT + wid_s * 64) * 16),
                                         16, 0, 0);
      }
    }
    const size_t yrow0 = ((size_t)n * a.P + p0) * a.Q;
#pragma unroll
    for (int t = 0; t < YPT; ++t) {
      const int row = (t * NT + tid) >> 3;            // < PB * Q rows (launcher: PB * Q == 224)
      if (row < kHaloRows) yv[t] = *reinterpret_cast<const uint4*>(s.y + (yrow0 + row) * 64 + cc * 8);
    }
    const int prow = pb + 1 < s.P2 ? 2 : 1;
    const size_t pbase = ((size_t)n * s.P2 + pb) * s.Q2 * 8;
#pragma unroll
    for (int t = 0; t < PPT; ++t) {
      const int i = t * NT + tid;
      if (i < prow * s.Q2 * 8) {
        pg[t] = reinterpret_cast<const uint4*>(s.dout)[pbase + i];
        pa[t] = reinterpret_cast<const uint2*>(s.arg)[pbase + i];
      }
    }
  };
  // dY rows of band `band` into the dY stage of buf (from the registers `issue` filled)
  auto produce = [&](int band, int buf) {
    const int n = band / h.bands_img, pb = band - n * h.bands_img;
    (void)n;
    const int prow = pb + 1 < s.P2 ? 2 : 1;
#pragma unroll
    for (int t = 0; t < PPT; ++t) {
      const int i = t * NT + tid;
      if (i < prow * s.Q2 * 8) {
        reinterpret_cast<uint4*>(dl)[i] = pg[t];
        reinterpret_cast<uint2*>(al)[i] = pa[t];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    char* Ds = smem + buf * STAGE + HBYTES;
    const StemBwdTile tl{dl, al, pb, s.P2, s.Q2, 8};
#pragma unroll
    for (int t = 0; t < YPT; ++t) {
      const int row = (t * NT + tid) >> 3;
      if (row >= kHaloRows) break;
      const int r = row / a.Q, w = row - r * a.Q;
      float v[8], d[8], o[8];
      unpack8(yv[t], v);
      tl.dz(pb * 2 + r, w, cc, v, sc, sh, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = stem_bwd_dy(ca[k], cb[k], cz[k], d[k], v[k]);
      *reinterpret_cast<uint4*>(Ds + row * 128 + ((((cc >> 1) ^ swz<128>(row)) << 5) | ((cc & 1) << 4))) = pack8(o);
    }
  };

  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  int rofs[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      const int mr = ks * 32 + 8 * g + q4 + 4 * hl;
      const int pr = mr / a.Q;
      rofs[ks][hl] = mr < h.PB * a.Q ? 16 * (pr * h.HWp + (mr - pr * a.Q)) : 0;
    }
  int cofs[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int kgc = wid * (16 * NI) + j * 16 + 4 * p4;
    const int tap = kgc >> a.log2C, c = kgc & (a.C - 1);
    const int r = tap / a.S, sx = tap - r * a.S;
    cofs[j] = (c >> 3) * h.pitchC * 16 + 16 * (r * h.HWp + sx) + 8 * ((c >> 2) & 1);
  }
  f32x4 acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  auto compute = [&](int buf) {
    const char* Hs = smem + buf * STAGE;
    const char* Ds = Hs + HBYTES;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[4], bfg[NI];
      const int r0 = ks * 32 + 8 * g + q4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * p4;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Ds + toff<64>(r0, col)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Ds + toff<64>(r0 + 4, col)));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Hs + cofs[j] + rofs[ks][0]));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Hs + cofs[j] + rofs[ks][1]));
        s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfg[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
  };

  issue(b0, 0);
  for (int b = b0; b < b1; ++b) {
    const int buf = (b - b0) & 1;
    wg_wait_vmcnt<0>();
    // every wave is done with the previous band's MFMAs (the other stage) and its dz reads
    // of the staged pooled rows, which produce() overwrites
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    produce(b, buf);
    if (b + 1 < b1) issue(b + 1, buf ^ 1);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // dY stage of band b published
    compute(buf);
  }

  float* dst = a.ws ? a.ws + (size_t)blockIdx.x * 64 * a.Kg : a.dw;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = i * 16 + (lane >> 4) * 4 + e;
        const int gg = wid * (16 * NI) + j * 16 + (lane & 15);
        float* pp = dst + (size_t)k * a.Kg + gg;
        if (a.ws)
          stfn<NT_WS_ST>(pp, acc[i][j][e]);
        else
          *pp += acc[i][j][e];
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
// fp8 weight gradients (128-row chunks, half the bytes per row): fewer, longer splits --
// 256 blocks measured +0.4% on the fp8 step (14,761 / 14,787 vs 14,712 / 14,728 img/s,
// profiles/ab_r03_nt_loads.txt) where 256 for the bf16 wgrads is -0.3%.  PMD_WGRAD_BLOCKS_F8.
static int wgrad_target_blocks_f8(int R) {
  static const int t = env_int("PMD_WGRAD_BLOCKS_F8", 256);
  return R <= 3 ? t : wgrad_target_blocks(R);
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
    g_wgrad_impl = (e && e[0] >= '0' && e[0] <= '7') ? e[0] - '0' : 1;
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

static bool halo_cfg(const WgradArgs& a, HaloArgs* h, int* nich);
static bool wgrad_cfg_ok(int impl, const WgradArgs& a) {
  if (impl == 4) return a.K >= 256 && a.Kg >= 256;
  if (impl == 5) return a.K >= 256;
  if (impl == 6) {
    HaloArgs h;
    int ni;
    return halo_cfg(a, &h, &ni);
  }
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
  // (a bytes-aware cap on the split count measured -2% to -36%: profiles/cu_mask_wgrad_blocks_r05.txt)
  if (splits < 1) splits = 1;
  const int cps = (chunks + splits - 1) / splits;
  *cps_out = cps;
  *splits_out = (chunks + cps - 1) / cps;
}

static void wgrad_reduce_launch(const WgradArgs& a, int splits, hipStream_t st);


// One full weight gradient with variant `impl`: split-K plan, kernel, split reduce.
static void wgrad_run(int impl, WgradArgs a, float* ws, hipStream_t st) {
  if (impl == 6) {
    HaloArgs h;
    int ni;
    if (halo_cfg(a, &h, &ni)) {
      const int splits = halo_splits(h);
      a.ws = splits > 1 ? ws : nullptr;
      if (ni == 4)
        hipLaunchKernelGGL((conv_wgrad_halo_kernel<4, 1280>), dim3(splits), dim3(256), 0, st, a, h);
      else
        hipLaunchKernelGGL((conv_wgrad_halo_kernel<9, 3072>), dim3(splits), dim3(256), 0, st, a, h);
      if (splits > 1) wgrad_reduce_launch(a, splits, st);
      return;
    }
    impl = 1;
  }
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
    case 7:  // DMA, 32-row stages, 3-deep ring: 48 KB (co-resides with a main-stream conv block)
      if (k64) hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 128, 32, 3>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 128, 32, 3>), grid, dim3(256), 0, st, a);
      break;
    default:  // 1: DMA, 64-row stages, 2-deep ring
      if (k64) hipLaunchKernelGGL((conv_wgrad_dma_kernel<64, 128, 64, 2>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_dma_kernel<128, 128, 64, 2>), grid, dim3(256), 0, st, a);
      break;
  }
  if (splits > 1) wgrad_reduce_launch(a, splits, st);
}

// ---- split-K reduction, grouped: ONE launch adds the partial slices of up to 16 weight
// gradients into their dW (a block backward's 3-4 convs when deferred, see wgrad_set_defer).
// Block b of descriptor d owns EB = 256 / G float4 elements; its G thread groups each sum the
// slices s = grp, grp + G, ... in increasing order, and the group partials are combined in
// group order through LDS: a fixed summation order, so the result is bitwise reproducible
// run to run (no fp32 atomics), in a single pass even for tiny outputs with hundreds of
// slices (the layer-1 1x1 gradients: 64 x 64 outputs, ~200 slices).
struct WsDesc {
  const float* ws;
  float* dw;
  long long n4;
  int splits, G, blocks;
};
constexpr int kWsGroupMax = 16;
struct WsGroup {
  WsDesc d[kWsGroupMax];
  int start[kWsGroupMax + 1];
  int n;
};

__global__ __launch_bounds__(256) void wgrad_reduce_grouped_kernel(WsGroup g) {
  __shared__ float4 part[256];
  int e = 0;
  while (e + 1 < g.n && g.start[e + 1] <= (int)blockIdx.x) ++e;
  const WsDesc d = g.d[e];
  const int lb = blockIdx.x - g.start[e];
  const int EB = 256 / d.G;
  const int t = threadIdx.x, el = t % EB, grp = t / EB;
  const float4* ws = reinterpret_cast<const float4*>(d.ws);
  for (long long base = (long long)lb * EB; base < d.n4; base += (long long)d.blocks * EB) {
    const long long i = base + el;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < d.n4) {
#pragma unroll 4
      for (int s = grp; s < d.splits; s += d.G) {
        const float4 v = ld16fn<NT_WS_LD>(ws + (long long)s * d.n4 + i);
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
      }
    }
    part[t] = acc;
    __syncthreads();
    if (grp == 0 && i < d.n4) {
      float4 tot = part[el];
      for (int q = 1; q < d.G; ++q) {
        const float4 v = part[q * EB + el];
        tot.x += v.x;
        tot.y += v.y;
        tot.z += v.z;
        tot.w += v.w;
      }
      float4 o = reinterpret_cast<float4*>(d.dw)[i];
      o.x += tot.x;
      o.y += tot.y;
      o.z += tot.z;
      o.w += tot.w;
      reinterpret_cast<float4*>(d.dw)[i] = o;
    }
    __syncthreads();
  }
}

static WsDesc ws_desc(const float* ws, float* dw, long long n4, int splits) {
  WsDesc d;
  d.ws = ws;
  d.dw = dw;
  d.n4 = n4;
  d.splits = splits;
  d.G = splits >= 64 ? 8 : (splits >= 16 ? 4 : (splits >= 4 ? 2 : 1));
  const int EB = 256 / d.G;
  long long b = (n4 + EB - 1) / EB;
  d.blocks = (int)(b > 2048 ? 2048 : b);
  return d;
}

static void ws_group_launch(const std::vector<WsDesc>& v, hipStream_t st) {
  for (size_t i0 = 0; i0 < v.size(); i0 += kWsGroupMax) {
    WsGroup g{};
    g.n = 0;
    int tot = 0;
    for (size_t i = i0; i < v.size() && g.n < kWsGroupMax; ++i) {
      g.d[g.n] = v[i];
      g.start[g.n] = tot;
      tot += v[i].blocks;
      ++g.n;
    }
    g.start[g.n] = tot;
    hipLaunchKernelGGL(wgrad_reduce_grouped_kernel, dim3(tot), dim3(256), 0, st, g);
  }
}

// Deferred mode (per thread, set around the weight gradients of one block backward on the
// side stream): the split reductions are queued and launched by wgrad_flush as ONE grouped
// launch, instead of one (or two) launches per weight gradient.
static thread_local bool t_ws_defer = false;
static thread_local std::vector<WsDesc> t_ws_pending;
static thread_local hipStream_t t_ws_stream = nullptr;
void wgrad_set_defer(bool on) { t_ws_defer = on; }
bool wgrad_defer() { return t_ws_defer; }
int wgrad_pending() { return (int)t_ws_pending.size(); }
int wgrad_flush(hipStream_t st) {
  if (t_ws_pending.empty()) return 0;
  if (st != t_ws_stream) return 1;  // must run on the stream that wrote the partial slices
  ws_group_launch(t_ws_pending, st);
  t_ws_pending.clear();
  return 0;
}

static void ws_reduce(const float* ws, float* dw, long long n4, int splits, hipStream_t st) {
  const WsDesc d = ws_desc(ws, dw, n4, splits);
  if (t_ws_defer) {
    if (!t_ws_pending.empty() && t_ws_stream != st) {
      ws_group_launch(t_ws_pending, t_ws_stream);  // never mix streams in one group
      t_ws_pending.clear();
    }
    t_ws_stream = st;
    t_ws_pending.push_back(d);
    return;
  }
  ws_group_launch(std::vector<WsDesc>{d}, st);
}

static void wgrad_reduce_launch(const WgradArgs& a, int splits, hipStream_t st) {
  ws_reduce(a.ws, a.dw, (long long)a.K * a.Kg / 4, splits, st);
}

// FP8 wgrad split plan: 128-row chunks, the bf16 kernels' block targets, workspace <= 96 MiB
static void plan_fp8(const WgradF8Args& a, int BM, int BN, int* splits_out, int* cps_out) {
  const int tiles = ((a.K + BM - 1) / BM) * ((a.Kg + BN - 1) / BN);
  const int chunks = (a.M + 127) / 128;
  int splits = (wgrad_target_blocks_f8(a.R) + tiles - 1) / tiles;
  const int max_splits = (chunks + 1) / 2;
  if (splits > max_splits) splits = max_splits;
  const long long per = (long long)a.K * a.Kg * 4;
  while (splits > 1 && per * splits > (96ll << 20)) --splits;
  if (splits < 1) splits = 1;
  const int cps = (chunks + splits - 1) / splits;
  *cps_out = cps;
  *splits_out = (chunks + cps - 1) / cps;
}

static void fill_f8(WgradF8Args& a, int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride,
                    int pad) {
  a.N = N; a.H = H; a.W = W; a.C = C; a.log2C = ilog2w(C);
  a.P = P; a.Q = Q; a.K = K; a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  a.M = (int)((long long)N * P * Q);
  a.Kg = R * S * C;
}

int conv_wgrad_fp8_splits(int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride, int pad) {
  WgradF8Args a;
  fill_f8(a, N, H, W, C, P, Q, K, R, S, stride, pad);
  int splits, cps;
  plan_fp8(a, K == 64 ? 64 : 128, 128, &splits, &cps);
  return splits;
}

int conv_wgrad_fp8_launch(const uint8_t* dyq, const uint8_t* xq, const float* sdy, const float* sx, float* dw,
                          float* ws, int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride,
                          int pad, hipStream_t st) {
  if (C % 16 != 0 || (C & (C - 1)) != 0) return 1;  // a 16-B chunk = 16 channels of one tap
  if (K % 64 != 0) return 2;
  if ((long long)N * P * Q >= (1ll << 31)) return 4;
  WgradF8Args a;
  fill_f8(a, N, H, W, C, P, Q, K, R, S, stride, pad);
  a.dy = dyq;
  a.x = xq;
  a.sdy = sdy;
  a.sx = sx;
  a.dw = dw;
  const int BM = K == 64 ? 64 : 128;
  int splits, cps;
  plan_fp8(a, BM, 128, &splits, &cps);
  if (splits > 1 && !ws) return 5;
  a.ws = splits > 1 ? ws : nullptr;
  a.chunks_per_split = cps;
  const int tiles = ((a.K + BM - 1) / BM) * ((a.Kg + 127) / 128);
  if (BM == 64)
    hipLaunchKernelGGL((conv_wgrad_fp8_kernel<64, 128>), dim3(tiles * splits), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_wgrad_fp8_kernel<128, 128>), dim3(tiles * splits), dim3(256), 0, st, a);
  if (splits > 1) {
    WgradArgs r;
    r.K = a.K;
    r.Kg = a.Kg;
    r.ws = ws;
    r.dw = dw;
    wgrad_reduce_launch(r, splits, st);
  }
  return 0;
}

static int wgrad_tune(const WgradArgs& a0, float* ws, hipStream_t st) {
  WgradArgs a = a0;
  struct NoDefer {  // the timed candidates include their own (immediate) reduction
    bool prev = t_ws_defer;
    NoDefer() { t_ws_defer = false; }
    ~NoDefer() { t_ws_defer = prev; }
  } nodefer;
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
  for (int c : {0, 1, 4, 5, 6}) {
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
  HaloArgs h;
  int ni;
  if (halo_cfg(a, &h, &ni)) best = halo_splits(h) > best ? halo_splits(h) : best;
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
    // A tuned choice is timed alone, but it runs next to the main stream: one 8-wave 256x256
    // block per CU holds 128 KB of LDS for the whole kernel (~150 us at l3/l4), so no main-stream
    // conv block (>= 34 KB) -- nor, with its VGPRs, a 5-us statistics collapse -- fits next to it
    // until it retires.  Tuned 256x256 choices therefore run as the 128x128 tile (64 KB):
    // +0.4% step (13,506 / 13,540 vs 13,460 / 13,467 img/s, profiles/wgrad_lds_r05.txt).
    // (the 256x128 / halo tiles as 128x128 measured slower, so they keep their tuned choice;
    // a forced variant -- PMD_WGRAD_IMPL, conv_wgrad_set_impl -- is never remapped)
    if (impl == 4 && wgrad_cfg_ok(1, a)) impl = 1;
  }
  wgrad_run(impl, a, ws, st);
  return 0;
}


// Fused stem backward (stem_wgrad_fused_kernel): the stem conv's weight gradient from the pooled
// gradient, with its dY produced in-kernel.  Geometry of the stem conv as for conv_wgrad_launch
// (x = the space-to-depth input [N,H,W,16], P x Q = the conv output = the BN input y); returns
// the split count through *splits (query with dw == nullptr), nonzero when the halo plan does not
// give 2-row bands of the pooled grid (the caller then runs the unfused passes).
int stem_wgrad_fused_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y, const float* params,
                            const float* gamma, const float* red, const float* count, float count_h,
                            const bf16_t* x, float* dw, float* ws, int N, int H, int W, int C, int P, int Q,
                            int K, int R, int S, int pad, int P2, int Q2, int* splits, hipStream_t st) {
  if (K != 64 || C != 16 || R != 4 || S != 4) return 1;
  if ((long long)N * P * Q >= (1ll << 31)) return 4;
  WgradArgs a;
  a.dy = nullptr;
  a.x = x;
  a.dw = dw;
  fill_args(a, N, H, W, C, P, Q, K, R, S, 1, pad);
  HaloArgs h;
  int ni;
  if (!halo_cfg(a, &h, &ni) || ni != 4 || h.PB != 2 || h.PB * a.Q != kHaloRows || P % 2 || P2 * 2 != P ||
      h.bands_img != P2 || Q2 > kStemPoolMaxQ || (Q + 1) / 2 != Q2)
    return 2;
  const int sp = halo_splits(h);
  if (splits) *splits = sp;
  if (!dw) return 0;
  if (sp > 1 && !ws) return 3;
  a.ws = sp > 1 ? ws : nullptr;
  StemDyArgs s{dout, arg, y, params, gamma, red, count, count_h, P2, Q2};
  hipLaunchKernelGGL(stem_wgrad_fused_kernel, dim3(sp), dim3(512), 0, st, a, h, s);
  if (sp > 1) wgrad_reduce_launch(a, sp, st);
  return 0;
}

}  // namespace pmd
