// Persistent streaming 1x1 convolution (stride 1, pad 0) for the short-reduction
// layers whose cost is the bytes around the GEMM, not the GEMM: the bottleneck
// conv1 / conv3 / stride-1 shortcut data gradients with the fused block-backward
// epilogue (addend [+ ReLU mask], BN-backward reduce over 1-2 BN inputs) and the
// same convolutions' forwards with the BN-statistics epilogue.
//
//   out[m][n] = sum_k A[m][k] * W[n][k]      (fwd: A = x, W = the KRSC image;
//                                             dgrad: A = dY, W = the transposed image)
//
// Why a different kernel: the tiled implicit-GEMM kernel (conv_igemm.hip) runs one
// output tile per workgroup and then its epilogue, so each workgroup's HBM traffic
// comes in serial phases (operand tiles, then addend / BN inputs, then stores) with a
// full memory latency between them, and ~12 workgroup generations per CU pay that
// chain again and again; the epilogue's fused reductions end in per-workgroup fp32
// atomics (thousands of workgroups x 2-4 x BN channels).  Here:
//   * ONE 256-thread workgroup per CU for the whole launch (persistent); it owns one
//     BN-channel column tile, whose weight slab [BN][KR] is loaded into LDS once;
//   * each wave streams its own 16-row M tiles through a private D-stage LDS ring:
//     the A rows AND every epilogue operand (addend, BN inputs, ReLU masks) of tile
//     k+D-1..k+1 are in flight by LDS-DMA (global_load_lds, no VGPRs) while tile k
//     is multiplied and its epilogue runs -- the HBM queue never drains between
//     tiles, and no workgroup barrier exists inside the loop (a wave reads only the
//     LDS its own DMAs wrote: its counted vmcnt is the only synchronisation);
//   * the MFMA tile is C^T (weights first): lane (p, g) holds output pixel p and,
//     because the slab rows of each 32-channel pair of 16x16 tiles are loaded in a
//     permuted order, 8 CONTIGUOUS channels 8g..8g+7 -- so the epilogue reads its
//     operands as 16-B LDS chunks, computes in registers and stores 16 B per lane,
//     without staging the C tile through LDS;
//   * the fused reductions (BN statistics / BN-backward sums) accumulate per lane in
//     registers across ALL tiles of the workgroup and are combined once at the end:
//     2 x BN (x sets) atomics per workgroup instead of per tile.
// Every LDS image is written lane-linearly by LDS-DMA with the XOR swizzle applied to
// the per-lane SOURCE address, chosen so every ds_read_b128 lane group of 16 touches
// 16 distinct 16-B bank slots (MI355X_MICROARCH.md §LDS lane groups):
//   128-B rows: chunk ^ ((row >> 1) & 7);   >= 256-B rows: chunk ^ (row & 15).
#include "common.h"

#include <stdio.h>
#include <stdlib.h>

namespace pmd {

struct Stream1x1Args {
  const bf16_t* a;   // [M][KR]
  const bf16_t* w;   // [Nout][KR] (channels_last image rows)
  bf16_t* out;       // [M][Nout]
  // forward: BN statistics slots [kStatSlots][2][Nout] about shift (nullable)
  float* stats;
  const float* shift;
  // dgrad epilogue
  const bf16_t* addend;       // [M][Nout] or null
  const uint8_t* amask;       // ReLU bitmask gating the addend [M][Nout/8] or null
  const uint8_t* bnmask;      // ReLU bitmask of the reduced BN output [M][Nout/8] or null
  const bf16_t* y[2];         // BN inputs of the fused reduce
  const float* p[2];          // their params [4][Nout] (mean, invstd, scale, shift)
  float* red[2];              // [kStatSlots][2][Nout] slots
  int M, Nout;
  int tilesN;                 // column tiles (Nout / BN)
  int mgroups;                // gridDim.x / tilesN
  int tiles64;                // 64-row block tiles ((M + 63) / 64)
  int D;                      // ring stages per wave
  int stage;                  // bytes of one wave stage
  int nE, nM;                 // epilogue operand tensors / masks streamed per tile
  int eoff[3];                // byte offsets of the E tensors inside a stage (addend, y0, y1)
  int moff[2];                // byte offsets of the masks (amask, bnmask)
  int slab;                   // slab bytes (ring base)
};

__device__ __attribute__((aligned(16))) unsigned char g_s1_zero[64];
__device__ __attribute__((aligned(16))) unsigned char g_s1_trash[4096];  // stores of rows past M

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (0..63)
__device__ __forceinline__ void wait_vm(int n) {
#define PMD_W1(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define PMD_W8(B) PMD_W1(B) PMD_W1(B + 1) PMD_W1(B + 2) PMD_W1(B + 3) PMD_W1(B + 4) PMD_W1(B + 5) PMD_W1(B + 6) PMD_W1(B + 7)
  switch (n) {
    PMD_W8(0) PMD_W8(8) PMD_W8(16) PMD_W8(24) PMD_W8(32) PMD_W8(40) PMD_W8(48) PMD_W8(56)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef PMD_W8
#undef PMD_W1
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// 32-bit LDS address of a pointer into the workgroup's LDS
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// LDS reads of the ring / slab: each statement issues its ds_reads AND waits for them
// (lgkmcnt(0)) inside ONE asm block.  Separate read and wait statements are not enough:
// the compiler believes an asm output is ready at once and may copy it (v_mov, AGPR
// moves) between the two -- copying registers the ds_read has not written yet.
#define PMD_RD "ds_read_b128 "
__device__ __forceinline__ void rdw1(u32x4& o0, uint32_t a0) {
  asm volatile(PMD_RD "%0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(o0) : "v"(a0) : "memory");
}
__device__ __forceinline__ void rdw2(u32x4& o0, u32x4& o1, uint32_t a0, uint32_t a1) {
  asm volatile(PMD_RD "%0, %2\n\t" PMD_RD "%1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o0), "=&v"(o1) : "v"(a0), "v"(a1) : "memory");
}
__device__ __forceinline__ void rdw3(u32x4& o0, u32x4& o1, u32x4& o2, uint32_t a0, uint32_t a1, uint32_t a2) {
  asm volatile(PMD_RD "%0, %3\n\t" PMD_RD "%1, %4\n\t" PMD_RD "%2, %5\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o0), "=&v"(o1), "=&v"(o2) : "v"(a0), "v"(a1), "v"(a2) : "memory");
}
__device__ __forceinline__ void rdw5(u32x4 (&o)[5], const uint32_t (&a)[5]) {
  asm volatile(PMD_RD "%0, %5\n\t" PMD_RD "%1, %6\n\t" PMD_RD "%2, %7\n\t" PMD_RD "%3, %8\n\t" PMD_RD
               "%4, %9\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]) : "memory");
}
__device__ __forceinline__ void rdw9(u32x4 (&o)[9], const uint32_t (&a)[9]) {
  asm volatile(PMD_RD "%0, %9\n\t" PMD_RD "%1, %10\n\t" PMD_RD "%2, %11\n\t" PMD_RD "%3, %12\n\t" PMD_RD
               "%4, %13\n\t" PMD_RD "%5, %14\n\t" PMD_RD "%6, %15\n\t" PMD_RD "%7, %16\n\t" PMD_RD
               "%8, %17\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]),
                 "=&v"(o[7]), "=&v"(o[8])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
                 "v"(a[8]) : "memory");
}
__device__ __forceinline__ void rdw4(u32x4 (&o)[4], const uint32_t (&a)[4]) {
  asm volatile(PMD_RD "%0, %4\n\t" PMD_RD "%1, %5\n\t" PMD_RD "%2, %6\n\t" PMD_RD "%3, %7\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]) : "memory");
}
__device__ __forceinline__ void rdw8(u32x4 (&o)[8], const uint32_t (&a)[8]) {
  asm volatile(PMD_RD "%0, %8\n\t" PMD_RD "%1, %9\n\t" PMD_RD "%2, %10\n\t" PMD_RD "%3, %11\n\t" PMD_RD
               "%4, %12\n\t" PMD_RD "%5, %13\n\t" PMD_RD "%6, %14\n\t" PMD_RD "%7, %15\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]),
                 "=&v"(o[7])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7])
               : "memory");
}
template <int N>
__device__ __forceinline__ void rdwN(u32x4 (&o)[N], const uint32_t (&a)[N]) {
  static_assert(N == 2 || N == 4 || N == 8, "rdwN");
  if constexpr (N == 2) rdw2(o[0], o[1], a[0], a[1]);
  else if constexpr (N == 4) rdw4(o, a);
  else rdw8(o, a);
}
#undef PMD_RD
// 8-B mask rows (BN = 64): two ds_read_b64, zero-extended to 16 B
__device__ __forceinline__ void rdw2_b64(u32x4& o0, u32x4& o1, uint32_t a0, uint32_t a1) {
  u32x2 x0, x1;
  asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x0), "=&v"(x1) : "v"(a0), "v"(a1) : "memory");
  o0 = u32x4{x0[0], x0[1], 0u, 0u};
  o1 = u32x4{x1[0], x1[1], 0u, 0u};
}

template <int RB>  // row bytes
__device__ __forceinline__ int s1_swz(int row) {
  if constexpr (RB == 128) return (row >> 1) & 7;
  else return row & 15;
}

__device__ __forceinline__ void dma16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// KR: reduction length (= A row length), BN: channels per workgroup column tile,
// NB: BN-input sets of the fused reduce (dgrad), FWD: forward (statistics epilogue)
template <int KR, int BN, int NB, bool FWD>
__global__ __launch_bounds__(256, 1) void conv1x1_stream_kernel(Stream1x1Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int NI = BN / 16;            // 16-channel MFMA tiles
  constexpr int NP = BN / 32;            // channel pairs (8 contiguous channels per lane)
  constexpr int KS = KR / 32;            // MFMA k-steps
  constexpr int RA = 2 * KR;             // A / slab row bytes
  constexpr int RE = 2 * BN;             // epilogue operand row bytes
  constexpr int NA = KR / 32;            // A DMA instructions per tile (16 rows x RA / 1 KiB)
  constexpr int NEI = BN / 32;           // DMA instructions per epilogue tensor
  constexpr int NBA = NB > 0 ? NB : 1;
  static_assert(KR == 64 || KR == 128 || KR == 256, "KR");
  static_assert(BN == 64 || BN == 128, "BN");
  static_assert(!(FWD && NB), "fwd has no BN-backward reduce");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p = lane & 15, g = lane >> 4;
  // XCD-aware placement: the workgroups of one XCD get consecutive logical ids, i.e. the
  // tilesN column tiles of the same row group run side by side on one XCD and share
  // their A rows through its L2
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = L % a.tilesN, mg = L / a.tilesN;
  const int n0 = nt * BN;

  // ---- weight slab: row t = 16 j + i of 16x16 tile j holds channel
  //      32 (j / 2) + 8 (i / 4) + 4 (j % 2) + i % 4, so lane (p, g) of the C^T tile pair
  //      (2jp, 2jp+1) holds the 8 contiguous channels 32 jp + 8 g .. + 7
  unsigned char* slab = lds;
  {
    constexpr int SLAB_INSTR = BN * RA / 1024;
#pragma unroll
    for (int ii = 0; ii < (SLAB_INSTR + 3) / 4; ++ii) {
      const int gi = ii * 4 + wave;
      if (gi < SLAB_INSTR) {
        const int off = gi * 1024 + 16 * lane;
        const int t = off / RA, phys = (off % RA) / 16;
        const int lg = phys ^ s1_swz<RA>(t);
        const int j = t >> 4, i = t & 15;
        const int ch = 32 * (j >> 1) + 8 * (i >> 2) + 4 * (j & 1) + (i & 3);
        dma16(a.w + (size_t)(n0 + ch) * KR + lg * 8, slab + gi * 1024);
      }
    }
  }

  // ---- per-lane constants of the streamed operands
  unsigned char* ring = lds + a.slab + wave * a.D * a.stage;
  // A: instruction i, lane -> row ra, logical chunk ca (constant over tiles)
  int a_off[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int off = i * 1024 + 16 * lane;
    const int r = off / RA, ph = (off % RA) / 16;
    a_off[i] = r * KR + ((ph ^ s1_swz<RA>(r)) << 3);   // elements, relative to row m0
  }
  const int a_row0 = (16 * lane) / RA;  // row of instruction 0 (rows of instr i: + i * 1024 / RA)
  // E tensors: instruction i, lane -> row, logical chunk
  int e_row[NEI], e_col[NEI];
#pragma unroll
  for (int i = 0; i < NEI; ++i) {
    const int off = i * 1024 + 16 * lane;
    const int r = off / RE, ph = (off % RE) / 16;
    e_row[i] = r;
    e_col[i] = n0 + ((ph ^ s1_swz<RE>(r)) << 3);
  }
  // masks: BN / 8 bytes per row, 16 rows, one 4-B DMA (a 256-B mask slot):
  //   BN = 128 -> lane -> row l/4, dword l%4;
  //   BN = 64  -> lanes < 32: row l/2, dword l%2; lanes >= 32 read the zero page into the
  //               unused upper half (a 1- or 2-B LDS-DMA still advances the LDS address by
  //               4 B per lane, so it cannot pack 8-B rows)
  const int mk_row = BN == 128 ? lane >> 2 : (lane & 31) >> 1;
  const int mk_col = BN == 128 ? n0 / 8 + (lane & 3) * 4 : n0 / 8 + (lane & 1) * 4;
  const bool mk_lane = BN == 128 || lane < 32;
  const int rowsN8 = a.Nout / 8;

  // fused-reduce / statistics state
  float s_a[NBA][NP][8], s_b[NBA][NP][8], mean[NBA][NP][8];
#pragma unroll
  for (int t = 0; t < NBA; ++t)
#pragma unroll
    for (int jp = 0; jp < NP; ++jp)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s_a[t][jp][e] = s_b[t][jp][e] = 0.f;
        mean[t][jp][e] = 0.f;
      }
  const bool do_stats = FWD && a.stats != nullptr;
  if (FWD && a.shift) {
#pragma unroll
    for (int jp = 0; jp < NP; ++jp)
#pragma unroll
      for (int e = 0; e < 8; ++e) mean[0][jp][e] = a.shift[n0 + 32 * jp + 8 * g + e];
  }
  if constexpr (NB > 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t)
#pragma unroll
      for (int jp = 0; jp < NP; ++jp)
#pragma unroll
        for (int e = 0; e < 8; ++e) mean[t][jp][e] = a.p[t][n0 + 32 * jp + 8 * g + e];
  }

  // this wave's tiles: block tiles mt = mg + k * mgroups, rows mt * 64 + 16 wave ..
  const int ntiles = mg < a.tiles64 ? (a.tiles64 - mg + a.mgroups - 1) / a.mgroups : 0;
  const int n_dma = NA + a.nE * NEI + a.nM;
  constexpr int n_st = NP;
  const bool has_add = !FWD && a.addend != nullptr;
  const bool has_am = has_add && a.amask != nullptr;
  const bool has_bm = NB > 0 && a.bnmask != nullptr;
  const int eo_add = a.eoff[0];
  const int eo_y0 = has_add ? a.eoff[1] : a.eoff[0];
  const int eo_y1 = has_add ? a.eoff[2] : a.eoff[1];
  const int mo_am = a.moff[0];
  const int mo_bm = a.nM == 2 ? a.moff[1] : a.moff[0];

  auto issue = [&](int k, int s) {
    // tile k of this wave into ring stage s; past the last tile: zero-page DMAs, so every
    // iteration issues the same number of vector-memory ops (counted vmcnt below)
    const int mt = mg + k * a.mgroups;
    const bool live = k < ntiles;
    const int m0 = live ? mt * 64 + 16 * wave : 0;
    unsigned char* st = ring + s * a.stage;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int r = a_row0 + i * (1024 / RA);
      const bool ok = live && m0 + r < a.M;
      const void* src = ok ? (const void*)(a.a + (size_t)m0 * KR + a_off[i]) : (const void*)g_s1_zero;
      dma16(src, st + i * 1024);
    }
    // tensor order in the stage: addend (if any), then the BN inputs
    auto dma_e = [&](const bf16_t* base, int eo) {
#pragma unroll
      for (int i = 0; i < NEI; ++i) {
        const int r = e_row[i];
        const bool ok = live && m0 + r < a.M;
        const void* src = ok ? (const void*)(base + (size_t)(m0 + r) * a.Nout + e_col[i]) : (const void*)g_s1_zero;
        dma16(src, st + eo + i * 1024);
      }
    };
    if (has_add) dma_e(a.addend, eo_add);
    if (NB > 0) dma_e(a.y[0], eo_y0);
    if (NB > 1) dma_e(a.y[1], eo_y1);
    auto dma_m = [&](const uint8_t* base, int mo) {
      const bool ok = live && mk_lane && m0 + mk_row < a.M;
      const void* src = ok ? (const void*)(base + (size_t)(m0 + mk_row) * rowsN8 + mk_col) : (const void*)g_s1_zero;
      dma4(src, st + mo);
    };
    if (has_am) dma_m(a.amask, mo_am);
    if (has_bm) dma_m(a.bnmask, mo_bm);
  };

  // slab landed (own DMAs) and visible to every wave; then the ring prologue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int k = 0; k < a.D; ++k) issue(k, k);

  for (int k = 0; k < ntiles; ++k) {
    const int s = k % a.D;
    // tile k's DMAs are complete: per iteration j the wave issues DMA(j + D) and THEN
    // the stores of tile j, so the ops younger than DMA(k) are the stores of the last
    // min(k, D) tiles and the DMAs of the D-1 tiles issued after it
    wait_vm((k < a.D ? k : a.D) * n_st + (a.D - 1) * n_dma);
    const unsigned char* st = ring + s * a.stage;
    const int mt = mg + k * a.mgroups;
    const int m0 = mt * 64 + 16 * wave;

    // All LDS reads of the ring / slab are explicit ds_reads in inline asm (rdw*): the
    // compiler's own waitcnt pass treats a ds_read as possibly aliasing the in-flight
    // LDS-DMA writes of the LATER stages and drains the whole DMA queue (vmcnt(0)) before
    // it -- exactly the serialisation this kernel exists to remove.  A wave reads only its
    // own completed stage (and the slab), so program order is the only ordering needed.
    const uint32_t stl = lds_addr(st), slabl = lds_addr(slab);
    // ---- every read of ring stage s first: the A fragments of all k-steps, the masks,
    //      the addend / BN inputs -- then stage s is refilled with tile k+D at once, so D
    //      tiles (not D-1) are in flight while this one is multiplied and stored
    u32x4 af[KS];
    {
      uint32_t aa[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) aa[ks] = stl + p * RA + (((ks * 4 + g) ^ s1_swz<RA>(p)) << 4);
      rdwN<KS>(af, aa);
    }
    u32x4 am_row = {0, 0, 0, 0}, bm_row = {0, 0, 0, 0};
    if (has_am || has_bm) {
      const uint32_t a0 = stl + (has_am ? mo_am : mo_bm), a1 = stl + mo_bm;
      if constexpr (BN == 128) rdw2(am_row, bm_row, a0 + p * 16, a1 + p * 16);
      else rdw2_b64(am_row, bm_row, a0 + p * 8, a1 + p * 8);
      if (!has_am) bm_row = am_row;
    }
    u32x4 ad[NP], yv[NBA][NP];
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) {
      const uint32_t po = p * RE + ((((jp * 4 + g) ^ s1_swz<RE>(p))) << 4);
      if constexpr (NB == 0) {
        if (has_add) rdw1(ad[jp], stl + eo_add + po);
      } else if constexpr (NB == 1) {
        if (has_add) rdw2(ad[jp], yv[0][jp], stl + eo_add + po, stl + eo_y0 + po);
        else rdw1(yv[0][jp], stl + eo_y0 + po);
      } else {
        if (has_add) rdw3(ad[jp], yv[0][jp], yv[1][jp], stl + eo_add + po, stl + eo_y0 + po, stl + eo_y1 + po);
        else rdw2(yv[0][jp], yv[1][jp], stl + eo_y0 + po, stl + eo_y1 + po);
      }
    }
    issue(k + a.D, s);
    // ---- MFMA: C^T[channel][pixel] = W[channel][k] * A[pixel][k], weights from the slab
    f32x4 acc[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int q = ks * 4 + g;
      u32x4 fr[NI];
      uint32_t ba[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int t = j * 16 + p;
        ba[j] = slabl + t * RA + ((q ^ s1_swz<RA>(t)) << 4);
      }
      rdwN<NI>(fr, ba);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fr[j]),
                                                          __builtin_bit_cast(bf16x8, af[ks]), acc[j], 0, 0, 0);
    }

    // ---- epilogue: lane (p, g) owns pixel m0 + p, channels n0 + 32 jp + 8 g .. + 7
    const bool row_ok = m0 + p < a.M;
    auto mbyte = [&](const u32x4& v, int c) {  // byte c of a 16-B mask row
      const uint32_t w = c < 4 ? v[0] : (c < 8 ? v[1] : (c < 12 ? v[2] : v[3]));
      return (w >> (8 * (c & 3))) & 0xffu;
    };
#pragma unroll
    for (int jp = 0; jp < NP; ++jp) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = acc[2 * jp][e];
        f[4 + e] = acc[2 * jp + 1][e];
      }
      const int ce = jp * 4 + g;                            // logical 16-B chunk of the row
      if (has_add) {
        float ga[8];
        unpack8(make_uint4(ad[jp][0], ad[jp][1], ad[jp][2], ad[jp][3]), ga);
        const uint32_t am = has_am ? mbyte(am_row, ce) : 0xffu;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += ((am >> e) & 1u) ? ga[e] : 0.f;
      }
      uint4 o = pack8(f);
      if (has_bm) {
        const uint32_t mk = mbyte(bm_row, ce);
        o.x &= ((mk & 1u) ? 0x0000ffffu : 0u) | ((mk & 2u) ? 0xffff0000u : 0u);
        o.y &= ((mk & 4u) ? 0x0000ffffu : 0u) | ((mk & 8u) ? 0xffff0000u : 0u);
        o.z &= ((mk & 16u) ? 0x0000ffffu : 0u) | ((mk & 32u) ? 0xffff0000u : 0u);
        o.w &= ((mk & 64u) ? 0x0000ffffu : 0u) | ((mk & 128u) ? 0xffff0000u : 0u);
      }
      // every lane stores (rows past M into the trash page): a fixed store count per tile
      void* dst = row_ok ? (void*)(a.out + (size_t)(m0 + p) * a.Nout + n0 + 32 * jp + 8 * g)
                         : (void*)(g_s1_trash + 16 * lane);
      st16n<NT_CONV_ST>(dst, o);
      if (FWD) {
        if (do_stats && row_ok) {
          float d[8];
          unpack8(o, d);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = d[e] - mean[0][jp][e];
            s_a[0][jp][e] += v;
            s_b[0][jp][e] += v * v;
          }
        }
      } else if constexpr (NB > 0) {
        float d[8];
        unpack8(o, d);
#pragma unroll
        for (int t = 0; t < NB; ++t) {
          float yy[8];
          unpack8(make_uint4(yv[t][jp][0], yv[t][jp][1], yv[t][jp][2], yv[t][jp][3]), yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s_a[t][jp][e] += d[e];
            s_b[t][jp][e] += d[e] * (yy[e] - mean[t][jp][e]);   // * invstd once, at the end
          }
        }
      }
    }
  }
  // no LDS-DMA may still be writing when the workgroup's LDS is reused
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- workgroup combine of the per-lane sums, one atomic per channel per workgroup
  constexpr int NSUM = FWD ? 1 : NB;
  if (NSUM > 0 && (!FWD || do_stats)) {
    // lanes p = 0..15 of a g group hold the same channels: xor-reduce over p
#pragma unroll
    for (int t = 0; t < NBA; ++t)
#pragma unroll
      for (int jp = 0; jp < NP; ++jp)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float u = s_a[t][jp][e], v = s_b[t][jp][e];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            u += __shfl_xor(u, o, 64);
            v += __shfl_xor(v, o, 64);
          }
          s_a[t][jp][e] = u;
          s_b[t][jp][e] = v;
        }
    __syncthreads();   // every wave is done with its ring: reuse it
    float* part = reinterpret_cast<float*>(lds + a.slab);   // [4 waves][NSUM][2][BN]
    if (p == 0) {
#pragma unroll
      for (int t = 0; t < NSUM; ++t)
#pragma unroll
        for (int jp = 0; jp < NP; ++jp)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int c = 32 * jp + 8 * g + e;
            part[((wave * NSUM + t) * 2 + 0) * BN + c] = s_a[t][jp][e];
            part[((wave * NSUM + t) * 2 + 1) * BN + c] = s_b[t][jp][e];
          }
    }
    __syncthreads();
    const int slot = blockIdx.x % kStatSlots;
    for (int i = tid; i < NSUM * 2 * BN; i += 256) {
      const int t = i / (2 * BN), which = (i / BN) & 1, c = i % BN;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += part[((w * NSUM + t) * 2 + which) * BN + c];
      if (FWD) {
        atomicAdd(a.stats + ((size_t)slot * 2 + which) * a.Nout + n0 + c, v);
      } else {
        const float* pt = t == 0 ? a.p[0] : a.p[1];
        float* rt = t == 0 ? a.red[0] : a.red[1];
        if (which) v *= pt[a.Nout + n0 + c];   // sum dz (y - mean) * invstd
        atomicAdd(rt + ((size_t)slot * 2 + which) * a.Nout + n0 + c, v);
      }
    }
  }
}

// ---------------------------------------------------------------- host side
static int g_s1_policy = -1;  // 0 off, 1 dgrad, 2 dgrad + fwd (PMD_CONV1X1 / conv1x1_set_policy)
void conv1x1_set_policy(int p) { g_s1_policy = p; }
int conv1x1_policy() {
  if (g_s1_policy < 0) {
    const char* e = getenv("PMD_CONV1X1");
    g_s1_policy = (e && e[0] >= '0' && e[0] <= '9') ? e[0] - '0' : 0;
  }
  return g_s1_policy;
}
static int g_s1_bn = 0;  // force BN (64 / 128), 0 = auto
void conv1x1_set_bn(int bn) { g_s1_bn = bn; }
static long long g_s1_launches = 0;  // launches taken by this kernel (tests check the path ran)
long long conv1x1_launches() { return g_s1_launches; }

constexpr int kS1Lds = 160 * 1024;

template <int KR, int BN, int NB, bool FWD>
static void s1_launch(const Stream1x1Args& a, int grid, int lds_bytes, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv1x1_stream_kernel<KR, BN, NB, FWD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, kS1Lds);
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_stream_kernel<KR, BN, NB, FWD>), dim3(grid), dim3(256), lds_bytes, st, a);
}

template <int KR, int BN, bool FWD>
static void s1_dispatch_nb(const Stream1x1Args& a, int nb, int grid, int lds, hipStream_t st) {
  if constexpr (FWD) {
    s1_launch<KR, BN, 0, true>(a, grid, lds, st);
  } else {
    if (nb == 2) s1_launch<KR, BN, 2, false>(a, grid, lds, st);
    else if (nb == 1) s1_launch<KR, BN, 1, false>(a, grid, lds, st);
    else s1_launch<KR, BN, 0, false>(a, grid, lds, st);
  }
}

// BN and ring depth: keep >= ~96 KiB of DMA in flight per CU (4 waves x D stages;
// MI355X_MICROARCH.md: 72 KiB/CU in flight reads HBM at ~6 TB/s) with the slab resident.
// nE: bf16 epilogue tensors per tile, nM: bit masks per tile, force_bn: 0 (auto) / 64 / 128.
// Returns 0 with the plan, nonzero when no plan fits (LDS or the 63-op vmcnt window).
static int s1_plan(int KR, int Nout, int nE, int nM, int force_bn, int* bn_out, int* D_out, int* stage_out,
                   int* slab_out) {
  if (KR != 64 && KR != 128 && KR != 256) return 1;
  if (Nout % 64 != 0) return 2;
  auto plan = [&](int bn, int* D, int* stage, int* slab) {
    *slab = bn * 2 * KR;
    *stage = 16 * (2 * KR + nE * 2 * bn) + nM * 256;   // 256-B mask slots (one 4-B DMA)
    *stage = (*stage + 15) & ~15;
    int d = (kS1Lds - *slab) / (4 * *stage);
    if (d > 8) d = 8;
    const int n_dma = KR / 32 + nE * (bn / 32) + nM, n_st = bn / 32;
    while (d > 2 && d * n_st + (d - 1) * n_dma > 63) --d;
    *D = d;
    // the final cross-wave combine reuses the ring as scratch
    return d >= 2 && d * n_st + (d - 1) * n_dma <= 63 && 4 * d * *stage >= 4 * 2 * 2 * bn * 4;
  };
  int bn = force_bn;
  if (bn == 128 || bn == 64) {
    if (Nout % bn || !plan(bn, D_out, stage_out, slab_out)) return 3;
  } else {
    bn = 0;
    if (Nout % 128 == 0 && plan(128, D_out, stage_out, slab_out) && 4 * *D_out * *stage_out >= 96 * 1024) bn = 128;
    else if (plan(64, D_out, stage_out, slab_out)) bn = 64;
    else return 3;
  }
  *bn_out = bn;
  return 0;
}

// Column tile the launcher would pick for this problem under the current conv1x1_set_bn
// (0 = not eligible): the tests' and the autotuner's eligibility oracle.
int conv1x1_stream_bn(int KR, int Nout, int nE, int nM) {
  int bn = 0, D = 0, stage = 0, slab = 0;
  return s1_plan(KR, Nout, nE, nM, g_s1_bn, &bn, &D, &stage, &slab) ? 0 : bn;
}

// Returns 0 when launched, nonzero when the shape / options are outside this kernel.
int conv1x1_stream_launch(const bf16_t* src, const bf16_t* wt, bf16_t* out, int M, int KR, int Nout, bool dgrad,
                          float* stats, const float* shift, const bf16_t* addend, const uint8_t* addend_mask,
                          const BnReduceArgs* bnr, hipStream_t st, int cus) {
  if (M <= 0) return 2;
  const int nb = (dgrad && bnr) ? (bnr->red[1] ? 2 : 1) : 0;
  Stream1x1Args a{};
  a.a = src;
  a.w = wt;
  a.out = out;
  a.stats = dgrad ? nullptr : stats;
  a.shift = dgrad ? nullptr : shift;
  a.addend = dgrad ? addend : nullptr;
  a.amask = (dgrad && addend) ? addend_mask : nullptr;
  a.bnmask = nb ? bnr->mask : nullptr;
  for (int t = 0; t < 2; ++t) {
    a.y[t] = (nb > t) ? bnr->y[t] : nullptr;
    a.p[t] = (nb > t) ? bnr->p[t] : nullptr;
    a.red[t] = (nb > t) ? bnr->red[t] : nullptr;
  }
  a.M = M;
  a.Nout = Nout;
  a.nE = (a.addend ? 1 : 0) + nb;
  a.nM = (a.amask ? 1 : 0) + (a.bnmask ? 1 : 0);
  int bn = 0, D = 0, stage = 0, slab = 0;
  const int rc = s1_plan(KR, Nout, a.nE, a.nM, g_s1_bn, &bn, &D, &stage, &slab);
  if (rc) return rc;
  a.D = D;
  a.stage = stage;
  a.slab = slab;
  int off = 16 * 2 * KR;
  for (int t = 0; t < 3; ++t) {
    a.eoff[t] = off;
    if (t < a.nE) off += 16 * 2 * bn;
  }
  for (int t = 0; t < 2; ++t) {
    a.moff[t] = off;
    if (t < a.nM) off += 256;
  }
  a.tilesN = Nout / bn;
  a.tiles64 = (M + 63) / 64;
  // persistent grid: one workgroup per CU, a whole number of column tiles, no more row
  // groups than there are 64-row tiles
  int mgroups = cus / a.tilesN;
  if (mgroups < 1) mgroups = 1;
  if (mgroups > a.tiles64) mgroups = a.tiles64;
  a.mgroups = mgroups;
  const int grid = mgroups * a.tilesN;
  const int lds = slab + 4 * D * stage;
#define S1K(KRV)                                                           \
  if (bn == 128) {                                                         \
    if (dgrad) s1_dispatch_nb<KRV, 128, false>(a, nb, grid, lds, st);     \
    else s1_dispatch_nb<KRV, 128, true>(a, nb, grid, lds, st);            \
  } else {                                                                 \
    if (dgrad) s1_dispatch_nb<KRV, 64, false>(a, nb, grid, lds, st);      \
    else s1_dispatch_nb<KRV, 64, true>(a, nb, grid, lds, st);             \
  }
  if (KR == 64) { S1K(64) }
  else if (KR == 128) { S1K(128) }
  else { S1K(256) }
#undef S1K
  ++g_s1_launches;
  return 0;
}

}  // namespace pmd
