// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
// Pure HIP: no torch headers here, so each kernel TU compiles in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "launchers.h"

namespace pmd {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef unsigned short bf16_t;  // storage type of one bf16

constexpr int kWave = 64;  // CDNA wavefront
// Per-channel statistics are accumulated into kStatSlots copies ([slot][2][C])
// picked by block index, so thousands of blocks do not serialise their fp32
// atomics on the same 2C addresses; stats_collapse sums the slots.
constexpr int kStatSlots = 64;

// Slot of a producer block's statistics partial: row block rb -> rb % nslots of the
// [nslots][2][C] slot copies.  nslots = kStatSlots in production: several blocks' fp32 atomics
// land in one slot, so the low bits of a sum depend on their order.  The deterministic mode
// (kernels/det.hip) hands the launch one private slot per row block of a zeroed scratch: every
// address then receives exactly one atomic (0 + v: exact), and det_fold sums the slots in a
// fixed order, so two identical steps are bit-identical.
__device__ __forceinline__ size_t stat_slot(int rb, int nslots) { return (size_t)(rb % nslots); }

// amax of a quantised tensor (fp8 delayed scaling): kAmaxSlots copies per site,
// one per (block % kAmaxSlots), so thousands of blocks do not serialise on one
// address; the host-side update takes the max over the slots.
constexpr int kAmaxSlots = 64;

// block-wide max of a non-negative value -> one atomicMax into slot blockIdx % kAmaxSlots
// (all threads of the block must call it; blockDim.x <= 1024, multiple of 64)
__device__ __forceinline__ void block_amax_update(float* slots, float v) {
  __shared__ float red[16];
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
    atomicMax(reinterpret_cast<unsigned int*>(slots + (blockIdx.x % kAmaxSlots)), __float_as_uint(m));
  }
}

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

// round-to-nearest-even; hipcc lowers the cast to v_cvt_pk_bf16_f32 (NaN-safe)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// 8 bf16 <-> uint4 helpers
// ---- cache policy of the streamed activation traffic (gfx950 "nt" = early eviction).
// Memory-bound passes next to the kernels of the OTHER stream: every line a streaming
// pass leaves in the XCD's L2 pushes out a re-read operand of the concurrent kernel
// (conv weight images, im2col tiles, wgrad operand rows).  Each stream below is
// non-temporal iff its bit is set in PMD_NT_MASK (compile time; A/B builds via
// PMD_EXTRA_CFLAGS=-DPMD_NT_MASK=...).  Full-step A/B on one lease
// (profiles/ab_r03_nt_loads.txt): BN-pass + dgrad-epilogue loads +2.9%, conv epilogue
// stores a further +1.2%, split-K partial / stem loads +0.2%; elementwise stores neutral.
enum NtStream {
  NT_BNA_Y = 1,      // bn_apply: BN input y
  NT_BNA_R = 2,      // bn_apply: residual / second BN input
  NT_BNB_D = 4,      // bn_bwd_elemt: dz
  NT_BNB_Y = 8,      // bn_bwd_elemt: BN input y
  NT_EPI_A = 16,     // dgrad epilogue: addend (identity-path gradient)
  NT_EPI_Y = 32,     // dgrad epilogue: BN inputs of the fused BN-backward reduce
  NT_CONV_ST = 64,   // conv / fp8-conv epilogue output stores
  NT_EW_ST = 128,    // elementwise BN outputs (bn_apply out, bn_bwd_elemt dy / dzm)
  NT_WS_LD = 256,    // wgrad_reduce: split-K partials
  NT_STEM = 512,     // stem pool passes: stem conv output
  NT_WS_ST = 1024,   // wgrad split-K partial stores
};
#ifndef PMD_NT_MASK
#define PMD_NT_MASK (NT_BNA_Y | NT_BNA_R | NT_BNB_D | NT_BNB_Y | NT_EPI_A | NT_EPI_Y | NT_CONV_ST | NT_WS_LD | NT_STEM)
#endif
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
typedef float f32x4_nt __attribute__((ext_vector_type(4)));
template <int S>
__device__ __forceinline__ uint4 ld16n(const void* p) {
  if constexpr ((PMD_NT_MASK & S) != 0) {
    const u32x4_nt w = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}
template <int S>
__device__ __forceinline__ float4 ld16fn(const void* p) {
  if constexpr ((PMD_NT_MASK & S) != 0) {
    const f32x4_nt w = __builtin_nontemporal_load(reinterpret_cast<const f32x4_nt*>(p));
    return make_float4(w[0], w[1], w[2], w[3]);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}
template <int S>
__device__ __forceinline__ void st16n(void* p, const uint4& v) {
  if constexpr ((PMD_NT_MASK & S) != 0) {
    const u32x4_nt w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_nt*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}
template <int S>
__device__ __forceinline__ void stfn(float* p, float v) {
  if constexpr ((PMD_NT_MASK & S) != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// LDS-DMA / register 16-B operand loads of the conv and wgrad mainloops, non-temporal
// when `nt` (wave-uniform: the operand rows no other block of the grid reads) AND the
// operand's bit is set in PMD_DMA_NT: 1 = conv A rows of a 1x1 conv whose single column
// tile covers every output channel, 2 = wgrad dY read by one tile column, 4 = wgrad X of a
// 1x1 conv read by one tile row.  All three (7) measured -1.9% on the full step (12,920 /
// 12,909 vs 13,175 / 13,173 img/s): a dgrad's dY rows are re-read by the weight gradient
// on the other stream, so evicting them early turns its L2/MALL hits into HBM reads.
#ifndef PMD_DMA_NT
#define PMD_DMA_NT 0
#endif
template <int OP>
__device__ __forceinline__ void glds16(const void* src, void* dst, bool nt) {
  if ((PMD_DMA_NT & OP) && nt)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 2);
  else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}
template <int OP>
__device__ __forceinline__ uint4 ld16c(const void* p, bool nt) {
  if ((PMD_DMA_NT & OP) && nt) {
    const u32x4_nt w = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  return *reinterpret_cast<const uint4*>(p);
}

__device__ __forceinline__ void unpack8(const uint4& v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// fp8 operand rows (128 B = 128 e4m3/e5m2 reduction elements): lane l of a
// 16x16x128 fragment read takes row l & 15 and the 16-B chunk PAIR 2 (l >> 4) + {0, 1}.
// A ds_read_b128 lane group (MI355X_MICROARCH.md §LDS: {0-3,12-15,20-27}, ...) then holds
// rows {0-3,12-15} at chunk x and rows 4-11 at chunk x ^ 2; the bf16 swizzles give those
// two row sets the same bank slots (2-way).  Map row pairs {0,1,6,7} (row >> 1) to odd and
// {2,3,4,5} to even XOR values: the x ^ 2 half then lands on the complementary slots,
// conflict-free for both chunks of the pair (brute-force check:
// tests/test_host_logic.py::test_fp8_fragment_swizzle_conflict_free).
__device__ __forceinline__ int swz_f8(int row) {
  constexpr unsigned kPerm = 0x75642031u;  // nibble p = XOR of row pair p
  return (kPerm >> (4 * ((row >> 1) & 7))) & 7;
}

// Bijective XCD-aware block remap (MI355X: 8 XCDs, blocks dispatched
// round-robin).  Blocks that share an XCD (same id % 8) get consecutive
// logical tile ids so neighbouring tiles reuse operand panels in that XCD's
// L2.  Speed-only: correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  constexpr int NX = 8;
  if (nwg < NX) return bid;
  const int q = nwg / NX, r = nwg % NX;
  const int x = bid % NX, j = bid / NX;
  const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + j;
}

// BatchNorm statistics are accumulated about a per-channel SHIFT K -- the
// previous training step's batch mean of the same BN site (0 before the first):
//   s1 = sum (v - K),  s2 = sum (v - K)^2,   mean = K + s1/n,  var = s2/n - (s1/n)^2
// Plain (sum v, sum v^2) cancels catastrophically once |mean| >> std (the fp32
// sum of squares loses (mean/std)^2 of its relative precision); with K within a
// few std of the mean the subtraction is benign ("shifted data" algorithm).
__device__ __forceinline__ void bn_moments(float s1, float s2, float n, float K, float& mean,
                                           float& var) {
  const float d = s1 / n;
  mean = K + d;
  var = fmaxf(s2 / n - d * d, 0.f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace pmd
