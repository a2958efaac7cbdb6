// Implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
//   FWD  : Y[m = (n,p,q)][k]  = sum_{r,s,c} X[n, p*st-pad+r, q*st-pad+s, c] * W[k,r,s,c]
//   DGRAD: dX[m = (n,h,w)][c] = sum_{r,s,k} dY[n, (h+pad-r)/st, (w+pad-s)/st, k] * W[k,r,s,c]
//                                (taps whose numerator is not divisible by st are skipped)
//
// Both are the same GEMM  C[M][Nout] = A[M][Kg] * B[Kg][Nout]  where A is the
// on-the-fly im2col gather of an NHWC activation (Kg ordered (r, s, c)) and
// B^T is a [Nout][Kg] row-major bf16 weight image (KRSC for fwd, CRSK for
// dgrad).  Because NHWC keeps the channel contiguous, every 16-byte (8 x bf16)
// chunk of an A row is one contiguous load for any C % 8 == 0 -- no im2col
// buffer, and the 3-channel stem only needs zero-padding to C = 8.
//
// Tile: BM x BN x BK (128x128, 128x64, 256x256, 256x128; 4 or 8 waves, each wave
// owning a sub-tile of 16x16x32 (or 32x32x16) MFMA accumulators).  Operands are
// copied global->LDS by LDS-DMA into an NST-stage ring (XOR-swizzled rows, one
// barrier per K-tile, counted vmcnt so later tiles stay in flight); a register-
// staged variant and the P8 register-resident-fragment pipeline are kept for
// A/B.  A per-shape autotuner picks the variant (the framework's
// cudnn.benchmark), persisted / broadcast as a tuning table (ops/tuning.py).
//
// Epilogue: fwd -- optional per-output-channel (sum, sum^2) of the bf16-rounded
// outputs about the BN shift K (combined across the block's waves in LDS, one
// fp32 atomic per channel per block into 64 slot copies); dgrad -- optional
// addend (+ReLU-mask gate) and the fused BN-backward reduce over 1-2 BN inputs.
// The tile is staged through LDS (C^T layout with 8-byte writes when no
// statistics are taken) and written with coalesced 16-byte row stores.
#include "common.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <vector>
#include <mutex>
#include <type_traits>

namespace pmd {

struct ConvArgs {
  const bf16_t* src;  // gathered operand, NHWC [N, H, W, Cs]
  const bf16_t* wt;   // B^T image [Nout][Kg]
  bf16_t* out;        // [M][Nout]
  float* stats;       // [kStatSlots][2][Nout] or nullptr: (sum (y-K), sum (y-K)^2) per channel
  const float* shift;  // K = the BN statistics shift [Nout] (nullable: 0), see bn_moments
  const bf16_t* addend;  // optional [M][Nout] tensor added to the output (grad accumulation)
  const uint8_t* addend_mask;  // optional ReLU bitmask gating the addend (identity-path dz = dout*mask)
  const float* addend_bias;    // optional fp32 [Nout] added with the addend (dgrad only)
  // optional fused BatchNorm-backward reduce over the (final, bf16) output tile
  // (dgrad of the conv that CONSUMED a BN+ReLU output): per channel n
  //   red[slot][0][n] += sum dz,  red[slot][1][n] += sum dz * (y - mean) * invstd
  // with dz = out * relu_bit(mask) -- for up to two BNs sharing the ReLU mask
  // (block-final BN + projection-shortcut BN).  Replaces a bn_bwd_reduce pass.
  const uint8_t* bn_mask;
  const bf16_t* bn_y[2];
  const float* bn_p[2];  // [4][Nout] (mean, invstd, scale, shift)
  float* bn_red[2];      // [kStatSlots][2][Nout]
  int N, H, W, Cs, log2Cs;
  int OH, OW;
  int Nout, R, S, stride, log2stride, pad;
  int M, Kg;
  // grid.z batch of independent problems (Winograd's 16 transformed-domain GEMMs):
  // problem z reads src + z * bs_src, wt + z * bs_wt and writes out + z * bs_out
  int batch;
  long long bs_src, bs_wt, bs_out;
  // F8 (fp8 dgrad, BASELINE config 5): src is e5m2 dY and wt an e4m3 [Nout][Kg] image
  // (byte pointers behind the bf16_t* fields); acc is scaled by 1 / (f8_sa * f8_sb)
  const float* f8_sa;
  const float* f8_sb;
  // statistics slots of stats / bn_red: a block of row tile rb adds into slot rb % nslots
  // (kStatSlots; the deterministic mode's private scratch slots: det_begin, kernels/det.hip)
  int nslots = kStatSlots;
};
typedef __attribute__((ext_vector_type(8))) int i32x8_c;

constexpr int LDA_REG = 64 + 8;  // padded LDS row of the register-staged path (elements)

// 16 zero bytes: the LDS-DMA source for padded / out-of-range im2col chunks
__device__ __attribute__((aligned(16))) unsigned char g_zero16[64];

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// DMA=true : operands are copied global->LDS by LDS-DMA (global_load_lds_dwordx4,
//            no VGPR round trip, no ds_write) into unpadded BK-element rows.  The
//            DMA writes lane-linearly (lane l -> LDS base + 16 l), so one wave
//            instruction fills 64/(BK/8) whole rows; the 16-B chunk is
//            XOR-swizzled on the per-lane SOURCE address so the fragment reads
//            (ds_read_b128, 16 rows x one chunk per lane group) are conflict-free:
//              BK=64 (8 chunks/row): phys = chunk ^ (row & 7)
//              BK=32 (4 chunks/row): phys = chunk ^ ((row >> 2) & 2)
//            NST-stage ring: NST-1 K-tiles of DMA in flight while one is consumed,
//            ONE barrier per K-tile (it both publishes tile kt and retires the
//            reads of the buffer the next DMA overwrites).
// DMA=false: register staging into 144-B padded rows, 2 stages (BK=64 only).
// PMD_CONV_SWZ=1: swizzles that make the 16 rows of one ds_read_b128 lane group
// hit 16 distinct 16-B bank slots (64 banks x 4 B): 128-B rows (BK=64) pair up
// rows by bit 0 (the two halves of the bank row), so the chunk XOR uses row
// bits 1..3; 64-B rows (BK=32) put 4 rows in one bank row, so it uses bits 2..3.
// Both are periodic in 16 rows, so a DMA instruction's rows (a multiple-of-16
// slab base + RPI i + lane / CH) get their chunk from the in-slab row alone.
#ifndef PMD_CONV_SWZ
#define PMD_CONV_SWZ 0
#endif
#ifndef PMD_CONV_SWAPC
#define PMD_CONV_SWAPC 1
#endif
#ifndef PMD_CONV_ST_PASS
#define PMD_CONV_ST_PASS 0
#endif
#ifndef PMD_F8_NB2_MINB4
#define PMD_F8_NB2_MINB4 0  // 1: the 2-set single-stage fp8 dgrad under the PMD_F8_MINB cap too
#endif
#ifndef PMD_TIMING_NO_ATOMICS
#define PMD_TIMING_NO_ATOMICS 0  // bit 0 / 1: drop the forward BN statistics / the dgrad fused-reduce atomics
                                 // (WRONG numerics; timing A/B only)
#endif
// PMD_DGRAD_PROBE=1 (timing-only variant build, bench/dgrad_probe.py): every data-gradient
// block's wave 0 stamps its sections -- entry, main loop done, C tile staged (+ the first
// epilogue row group's operand prefetch), epilogue rows done, fused BN-reduce done -- and
// appends one 16-word record to a device buffer (conv_probe_set).
#ifndef PMD_DGRAD_PROBE
#define PMD_DGRAD_PROBE 0
#endif
#if PMD_DGRAD_PROBE
__device__ unsigned long long* g_probe_buf;
// 256 counters, each owning cap/256 records (one counter for the whole grid serialised every
// block's append on one L2 line: ~1 ms per 12k-block launch)
__device__ unsigned int g_probe_ctr[256 * 32];  // one 128-B line per counter
__device__ unsigned int g_probe_cap;
#endif
#ifndef PMD_F8_MINB
// min blocks per CU of the single-stage fp8 dgrad with 0 / 1 fused BN-reduce sets: 4 = the
// 128-VGPR cap (4 waves/SIMD; no spills with one B fragment held, NJ = 1); the 2-set
// instantiation spills at that cap and keeps 2 (158 VGPRs, 3 waves/SIMD, NJ = NI)
#define PMD_F8_MINB 4
#endif
#ifndef PMD_CONV_SETPRIO
#define PMD_CONV_SETPRIO 0
#endif
#ifndef PMD_CONV_MINB4
#define PMD_CONV_MINB4 2  // __launch_bounds__ min blocks per CU of the 4-wave tiles (VGPR cap A/B knob)
#endif
template <int BK>
__device__ __forceinline__ int swz(int row) {
  if constexpr (PMD_CONV_SWZ) {
    if constexpr (BK == 64) return (row >> 1) & 7;
    else return (row >> 2) & 3;
  } else {
    if constexpr (BK == 64) return row & 7;
    else return (row >> 2) & 2;
  }
}

// MF32: v_mfma_f32_32x32x16_bf16 instead of 16x16x32 (same FLOPs in half the
// instructions, so the MFMA holds the SIMD's issue port 8 of every 32 cycles
// instead of 8 of 16 -- more room for the gather math and LDS reads).  Needs
// the LDS-DMA uniform-tap path with BK=64; chunk swizzle phys = q ^ ((row>>1)&7)
// keeps the 32-row ds_read_b128 lane groups conflict-free.
// WM x WN waves (NT = 64 WM WN threads): 2x2 = the 128-row tiles at 2 blocks/CU;
// 4x2 / 2x4 = 256-row tiles at one 8-wave block per CU, i.e. half the operand
// bytes per MFMA FLOP from L2 (128x128: 64 FLOP/B -> 256x128: 85, 256x256: 128),
// for the layers whose grid still fills the chip with the bigger tile.
//
// P8: register-resident fragment pipeline (LDS-DMA, BK=64, 2 LDS buffers, uniform-tap
// loader): a whole K-tile's A/B fragments live in VGPRs, so the LDS buffer they came
// from is re-filled (tile kt+2) right after ONE barrier while the tile's MFMAs run from
// registers; the DMA queue never drains to zero inside the loop (counted vmcnt leaves
// the next tile's loads in flight across both barriers of a K-tile), and the next
// tile's fragments are read into each register set as soon as its MFMAs retire
// (cdna_hip_programming.md §5 "Pipelining across barriers", T3/T4, T5).
//
// HALO: 3x3 / stride 1 / pad 1 (fwd, or dgrad with flipped taps), Cs % 64 == 0, 7 <= W <= 56.
// A tile of BM output pixels of ONE image needs a few input rows: those rows (+1-pixel
// halo, zero borders) are copied to LDS once per 64-channel block and all 9 taps read
// their A fragments from that halo image at a wave-uniform pixel offset, instead of
// gathering every input pixel 9 times from L2 (the 64/128-channel 3x3 layers are
// bound by that L2->LDS gather traffic); only the weight tiles stream per K-tile.
template <int BM, int BN, int BK, int NST, bool DGRAD, bool STATS, bool DMA, bool MF32 = false,
          int WM = 2, int WN = 2, bool P8 = false, bool HALO = false, int NB = 2, bool F8 = false,
          int NST1 = 0>
__global__ __launch_bounds__(64 * WM * WN,
                             (F8 && NST1 && (NB < 2 || PMD_F8_NB2_MINB4)) ? PMD_F8_MINB
                                                                          : (WM * WN == 4 ? PMD_CONV_MINB4 : 2))
    void conv_igemm_kernel(ConvArgs a) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  static_assert(DMA || (BK == 64 && NST == 2 && NW == 4), "register staging: BK=64, 2 stages, 4 waves");
  // F8: fp8 operands (1 B per element) in the same 128-B LDS rows (BK = 64 bf16 slots =
  // 128 fp8 reduction elements per K-tile), one v_mfma_scale_f32_16x16x128_f8f6f4 per
  // fragment pair and K-tile; NST1: a single LDS stage (load, wait, compute) for the
  // one- or two-K-tile reductions of the epilogue-bound dgrads (occupancy of the bf16 BK=32
  // tiles: 4 blocks per CU)
  static_assert(!F8 || (DMA && BK == 64 && !MF32 && !P8 && !HALO), "F8: LDS-DMA, 128-B rows, plain pipeline");
  static_assert(!NST1 || (F8 && NST == 2), "NST1: fp8 only");
  static_assert(!MF32 || (DMA && BK == 64), "32x32 MFMA path: LDS-DMA, BK=64");
  static_assert(!P8 || (DMA && BK == 64 && NST == 2 && !MF32), "P8: LDS-DMA, BK=64, 2 buffers, 16x16 MFMA");
  static_assert(!HALO || (DMA && BK == 64 && (NST == 2 || NST == 3) && !MF32 && !P8),
                "HALO: LDS-DMA, BK=64, 2- or 3-deep weight ring");
  // SWAPC: without the BN-statistics epilogue the 16x16 MFMAs compute C^T (weights as
  // the first operand): a lane then holds 4 consecutive output CHANNELS of one pixel,
  // so the C tile is staged with one ds_write_b64 per accumulator instead of four
  // ds_write_b16 (the statistics epilogue keeps the channel-per-lane layout, whose
  // per-channel sums need 4x fewer cross-lane steps)
  constexpr bool SWAPC = PMD_CONV_SWAPC && !STATS && !MF32;
  constexpr int CH = BK / 8;                      // 16-B chunks per LDS row
  constexpr int CE = F8 ? 16 : 8;                 // reduction elements per 16-B chunk
  constexpr int BKE = F8 ? 2 * BK : BK;           // reduction elements per K-tile
  using ET = typename std::conditional<F8, uint8_t, bf16_t>::type;
  constexpr int RPI = DMA ? 64 / CH : 32;         // rows per load instruction (wave / block)
  constexpr int PA = DMA ? BM / (NW * RPI) : BM / 32;  // A load instructions per thread per tile
  constexpr int PB = DMA ? BN / (NW * RPI) : BN / 32;
  static_assert(PA >= 1 && PB >= 1, "tile too small for this BK");
  static_assert(!DMA || ((BM / NW) % RPI == 0 && (BN / NW) % RPI == 0), "wave row slabs");
  constexpr int LPT = PA + PB;
  constexpr int MI = BM / (16 * WM);  // 16-row MFMA tiles per wave
  constexpr int NI = BN / (16 * WN);  // 16-col MFMA tiles per wave
  constexpr int LDR = DMA ? BK : BK + 8;  // LDS row length (elements)
  constexpr int A_ELEMS = BM * LDR;
  constexpr int B_ELEMS = BN * LDR;
  constexpr int STAGE = A_ELEMS + B_ELEMS;
  // C tile staged with 8 elements of row padding (an unpadded XOR-swizzled staging, 32 instead of
  // 34 KB, measured -0.3% on the step: profiles/epi_x_r05.txt)
  constexpr int LDC = BN + 8;
  // epilogue C-staging layout (SWAPC only): EPI_SW = 8-B half swap in rows with bit 3
  // set (conflict-free ds_write_b64); EPI_RM = row order of the ds_read_b128 row reads
  // for 16-chunk rows read by 16 thread rows (BN = 128, 4 waves): the two 16-lane
  // halves of a 32-lane read group take rows 16 apart (64 dwords = the same bank
  // phase) instead of adjacent rows, whose 4-dword skew overlapped two chunks
#ifndef PMD_EPI_SW
#define PMD_EPI_SW 1
#endif
  constexpr bool EPI_SW = PMD_EPI_SW && SWAPC;
  constexpr bool EPI_RM = PMD_EPI_SW && SWAPC && BN == 128 && NT == 256;
  constexpr bool EPI_RM64 = PMD_EPI_SW >= 2 && SWAPC && BN == 64 && NT == 256;
  // HALO image: at most ceil(BM / W) + 3 input rows of W + 2 pixels (a tile spans
  // ceil(BM / W) + 1 rows, plus the two halo rows), 8 chunks each, rounded up to whole
  // block-wide DMA rounds (NT chunks).  For BM = 128 and 7 <= W <= 56 (launcher
  // guard) the maximum is 348 pixels (W = 56): 45 KB, 2 blocks per CU with the B ring.
  static_assert(!HALO || BM == 128, "HALO sized for 128-pixel tiles");
  constexpr int HALO_PIX = 348;
  constexpr int HALO_CHUNKS = ((HALO_PIX * 8 + NT - 1) / NT) * NT;
  constexpr int HALO_BYTES = HALO ? HALO_CHUNKS * 16 : 0;
  constexpr int SMEM_MAIN = HALO ? HALO_BYTES + NST * B_ELEMS * 2 : (NST1 ? 1 : NST) * STAGE * 2;
  constexpr int SMEM_EPI = BM * LDC * 2;
  constexpr int PSTR = 17;                          // fused BN-reduce partials [NT][17] (odd stride)
  constexpr int SMEM_PART = DGRAD ? NT * PSTR * 4 : 0;
  constexpr int SMEM0 = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  constexpr int SMEM = SMEM0 > SMEM_PART ? SMEM0 : SMEM_PART;
  static_assert(SMEM + (STATS ? WM * 2 * BN * 4 : 0) <= 160 * 1024, "exceeds the 160 KiB LDS of a CU");
  constexpr int SMEM_ST = STATS ? WM * 2 * BN * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[SMEM + SMEM_ST];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem);

  if (blockIdx.z) {  // batched launch (no statistics / addend / fused reduce: launcher contract)
    a.src += blockIdx.z * a.bs_src;
    a.wt += blockIdx.z * a.bs_wt;
    a.out += blockIdx.z * a.bs_out;
  }
  // operand base pointers in elements of the operand type (F8: bytes behind the bf16_t* fields)
  const ET* const srcE = reinterpret_cast<const ET*>(a.src);
  const ET* const wtE = reinterpret_cast<const ET*>(a.wt);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // Strided dgrad is split into stride^2 output phases (blockIdx.y): in phase
  // (ph, pw) only taps r == (ph+pad) mod 2 (resp. s) contribute, so every
  // gathered tap is real work (no 3/4-masked MFMAs); rows of the phase GEMM
  // are the output pixels (n, 2*hh+ph, 2*ww+pw).
  int ph = 0, pw = 0, OHp = a.OH, OWp = a.OW, r0 = 0, s0 = 0, rstep = 1, ns = a.S, Mp = a.M,
      Kgp = a.Kg;
  if (DGRAD && a.stride == 2) {
    ph = blockIdx.y >> 1;
    pw = blockIdx.y & 1;
    OHp = (a.OH - ph + 1) >> 1;
    OWp = (a.OW - pw + 1) >> 1;
    r0 = (ph + a.pad) & 1;
    s0 = (pw + a.pad) & 1;
    rstep = 2;
    const int nr = (a.R - r0 + 1) >> 1;
    ns = (a.S - s0 + 1) >> 1;
    Mp = a.N * OHp * OWp;
    Kgp = nr * ns * a.Cs;
  }
  const int tilesN = (a.Nout + BN - 1) / BN;
  // the A rows of a 1x1 conv are read by this block alone when one column tile covers
  // every output channel (no L2 reuse to protect: non-temporal DMA, glds16)
  const bool a_once = tilesN == 1 && a.R == 1 && a.S == 1;
  const int Mgrid = (DGRAD && a.stride == 2) ? a.N * ((a.OH + 1) >> 1) * ((a.OW + 1) >> 1) : a.M;
  const int hw_out = a.OH * a.OW;
  const int halo_T = HALO ? (hw_out + BM - 1) / BM : 1;  // HALO: M tiles never straddle images
  const int tilesM = HALO ? a.N * halo_T : (Mgrid + BM - 1) / BM;  // grid.x sized for the largest phase
  const int L = xcd_remap(blockIdx.x, tilesM * tilesN);
  const int mt = L / tilesN;
  const int halo_img = HALO ? mt / halo_T : 0, halo_t = HALO ? mt - (mt / halo_T) * halo_T : 0;
  const int m0 = HALO ? halo_img * hw_out + halo_t * BM : mt * BM;
  const int n0 = (L % tilesN) * BN;
  if (HALO) Mp = m0 + min(BM, hw_out - halo_t * BM);  // rows of this image only
  if (m0 >= Mp) return;  // uniform per block, before any barrier
#if PMD_DGRAD_PROBE
  unsigned long long pt[5] = {0, 0, 0, 0, 0};
  const unsigned long long pwc0 = wall_clock64();
  pt[0] = clock64();
#define PMD_PROBE_AT(k) \
  do {                  \
    pt[k] = clock64();  \
  } while (0)
#else
#define PMD_PROBE_AT(k) \
  do {                  \
  } while (0)
#endif

  // ---- per-thread A-row precompute
  // register staging: thread -> (row rsub + 32 i, chunk tid & 7)
  // DMA: wave w, instruction i, lane l -> row w*(BM/4) + RPI i + l/CH, LDS chunk l%CH
  //      holding logical chunk (l%CH) ^ swz(row)
  // DMA: LDS chunk lane % CH of A (B) instruction i's tile row holds logical chunk
  // achunk(i) (bchunk(i)); the swizzle is taken of the absolute tile row
  auto swzk = [](int row) { return F8 ? swz_f8(row) : swz<BK>(row); };
  auto achunk = [&](int i) { return DMA ? ((lane % CH) ^ swzk(wid * (BM / NW) + RPI * i + lane / CH)) : (tid & 7); };
  auto bchunk = [&](int i) { return DMA ? ((lane % CH) ^ swzk(wid * (BN / NW) + RPI * i + lane / CH)) : (tid & 7); };
  const int chunk = tid & 7;  // register staging
  const int rsub = tid >> 3;  // 0..31
  auto a_row_of = [&](int i) { return DMA ? wid * (BM / NW) + RPI * i + lane / CH : rsub + 32 * i; };
  auto b_row_of = [&](int i) { return DMA ? wid * (BN / NW) + RPI * i + lane / CH : rsub + 32 * i; };
  int a_base[PA], a_h[PA], a_w[PA];
  bool a_ok[PA];
  const int ohw = OHp * OWp;
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int m = m0 + a_row_of(i);
    a_ok[i] = m < Mp;
    const int mm = a_ok[i] ? m : 0;
    const int n = mm / ohw;
    const int rem = mm - n * ohw;
    const int oh = (rem / OWp) * rstep + ph;
    const int ow = (rem - (rem / OWp) * OWp) * rstep + pw;
    a_base[i] = n * a.H * a.W;  // pixel index base
    if (DGRAD) {
      a_h[i] = oh + a.pad;
      a_w[i] = ow + a.pad;
    } else {
      a_h[i] = oh * a.stride - a.pad;
      a_w[i] = ow * a.stride - a.pad;
    }
  }
  const ET* b_row[PB];
  bool b_ok[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int nn = n0 + b_row_of(i);
    b_ok[i] = nn < a.Nout;
    b_row[i] = wtE + (size_t)(b_ok[i] ? nn : 0) * a.Kg;
  }
  // Uniform-tap fast path (LDS-DMA, Cs % BK == 0 -- every layer but the stem):
  // a K-tile then lies inside ONE filter tap, so the tap (r, s) and its pixel
  // offset are wave-uniform scalars; per row the gather needs only
  //   ih = u_h + dr, iw = u_w + ds, pix = u_p + dr*W + ds   (dr, ds scalars)
  // with (dr, ds) = (r, s) fwd, (-r, -s) stride-1 dgrad, (-tr, -ts) stride-2
  // dgrad (the phase fixes r = r0 + 2 tr, so (h + pad - r) / 2 = u_h - tr).
  const bool uni = DMA && a.Cs >= BKE;
  int u_h[PA], u_w[PA], u_p[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    int hh = a_h[i], ww = a_w[i];
    if (DGRAD && a.stride == 2) {
      hh = (a_h[i] - r0) >> 1;
      ww = (a_w[i] - s0) >> 1;
    }
    u_h[i] = hh;
    u_w[i] = ww;
    u_p[i] = a_base[i] + hh * a.W + ww;
  }
  // MF32 swizzle depends on row bits 1..3: instruction i covers rows base + 8i + l/8 with
  // base % 32 == 0 (BM/4, BN/4 multiples of 16 -> (base >> 1) % 8 == 0)
  const int lane_c32[2] = {((lane & 7) ^ (((lane >> 3) >> 1) & 7)) * 8,
                           ((lane & 7) ^ ((4 + ((lane >> 3) >> 1)) & 7)) * 8};
  const int wid_s = __builtin_amdgcn_readfirstlane(wid);

  uint4 ra[DMA ? 1 : PA], rb[DMA ? 1 : PB];
  const int nk = (Kgp + BKE - 1) / BKE;

  // Tap state of the NEXT K-tile the uniform loader issues.  K-tiles are issued
  // strictly in order (prologue 0..NST-2, then kt+NST-1), and with Cs >= BK a
  // K-tile lies inside one filter tap, so (channel block, tap row, tap col) is
  // advanced incrementally in scalar registers -- no per-tile integer division.
  int u_cb = 0, u_tr = 0, u_ts = 0, u_kt = 0;
  // per-row source pointers at tap (0,0) channel 0 (+ this lane's chunk); a tile
  // then only adds the wave-uniform offset (dr*W + ds)*Cs + cb
  const ET* a_ptr[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int ci = MF32 ? lane_c32[i & 1] : achunk(i) * CE;
    // signed: u_p is -1.. at padded borders (never dereferenced there: `ok` masks it)
    a_ptr[i] = srcE + ((long long)u_p[i] << a.log2Cs) + ci;
  }
  auto load_tile_uni = [&](int kt, int dbuf) {
    (void)kt;
    const bool kok = u_kt < nk;
    const int r = r0 + rstep * u_tr, sx = s0 + rstep * u_ts;
    int dr, ds;
    if (!DGRAD) {
      dr = r;
      ds = sx;
    } else if (a.stride == 2) {
      dr = -u_tr;
      ds = -u_ts;
    } else {
      dr = -r;
      ds = -sx;
    }
    const long long aoff = ((long long)(dr * a.W + ds) << a.log2Cs) + u_cb;  // scalar
    const int tapo = ((r * a.S + sx) << a.log2Cs) + u_cb;
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const bool ok = kok && a_ok[i] && (unsigned)(u_h[i] + dr) < (unsigned)a.H &&
                      (unsigned)(u_w[i] + ds) < (unsigned)a.W;
      const void* src = ok ? (const void*)(a_ptr[i] + aoff) : (const void*)g_zero16;
      bf16_t* dst = lds + dbuf * STAGE + (wid_s * (BM / NW) + RPI * i) * LDR;
      glds16<1>(src, dst, a_once);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int boff = tapo + (MF32 ? lane_c32[i & 1] : bchunk(i) * CE);
      const void* src = (b_ok[i] && kok) ? (const void*)(b_row[i] + boff) : (const void*)g_zero16;
      bf16_t* dst = lds + dbuf * STAGE + A_ELEMS + (wid_s * (BN / NW) + RPI * i) * LDR;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
    // advance to the next K-tile: channel block, then tap column, then tap row
    ++u_kt;
    u_cb += BKE;
    if (u_cb == a.Cs) {
      u_cb = 0;
      if (++u_ts == ns) {
        u_ts = 0;
        ++u_tr;
      }
    }
  };

  // tap -> (tap row, tap col) of the general loader: a shift when the (phase) filter width
  // is a power of two (the 4x4 space-to-depth stem, 1x1, 2-tap phases) instead of a
  // runtime integer division per chunk per K-tile (the stem conv's gather was VALU-bound)
  const bool ns_pow2 = (ns & (ns - 1)) == 0;
  const int log2ns = ns_pow2 ? __builtin_ctz(ns) : 0;
  auto tap_row = [&](int tap) { return ns_pow2 ? (tap >> log2ns) : tap / ns; };
  auto load_tile = [&](int kt, int dbuf) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int k0 = kt * BKE + achunk(i) * CE;
      const bool kok = k0 < Kgp;
      const int tap = k0 >> a.log2Cs;
      const int c = k0 & (a.Cs - 1);
      const int tr = tap_row(tap);
      const int r = r0 + rstep * tr;
      const int s = s0 + rstep * (tap - tr * ns);
      int ih, iw;
      bool ok = a_ok[i] && kok;
      if (DGRAD) {
        const int th = a_h[i] - r, tw = a_w[i] - s;
        ok = ok && th >= 0 && tw >= 0 && ((th | tw) & (a.stride - 1)) == 0;
        ih = th >> a.log2stride;
        iw = tw >> a.log2stride;
      } else {
        ih = a_h[i] + r;
        iw = a_w[i] + s;
      }
      ok = ok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      if constexpr (DMA) {
        const void* src = g_zero16;
        if (ok) src = srcE + (((size_t)(a_base[i] + ih * a.W + iw)) << a.log2Cs) + c;
        bf16_t* dst = lds + dbuf * STAGE + (wid * (BM / NW) + RPI * i) * LDR;
        glds16<1>(src, dst, a_once);
      } else {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ok) {
          const size_t pix = (size_t)(a_base[i] + ih * a.W + iw);
          v = *reinterpret_cast<const uint4*>(a.src + (pix << a.log2Cs) + c);
        }
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int k0 = kt * BKE + bchunk(i) * CE;
      const bool kok = k0 < Kgp;
      const int tap = k0 >> a.log2Cs;
      const int tr = tap_row(tap);
      const int r = r0 + rstep * tr;
      const int s = s0 + rstep * (tap - tr * ns);
      const int boff = ((r * a.S + s) << a.log2Cs) + (k0 & (a.Cs - 1));
      if constexpr (DMA) {
        const void* src = (b_ok[i] && kok) ? (const void*)(b_row[i] + boff) : (const void*)g_zero16;
        bf16_t* dst = lds + dbuf * STAGE + A_ELEMS + (wid * (BN / NW) + RPI * i) * LDR;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      } else {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (b_ok[i] && kok) v = *reinterpret_cast<const uint4*>(b_row[i] + boff);
        rb[i] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
    if constexpr (!DMA) {
      bf16_t* As = lds + buf * STAGE;
      bf16_t* Bs = As + A_ELEMS;
#pragma unroll
      for (int i = 0; i < PA; ++i)
        *reinterpret_cast<uint4*>(As + (rsub + 32 * i) * LDA_REG + chunk * 8) = ra[i];
#pragma unroll
      for (int i = 0; i < PB; ++i)
        *reinterpret_cast<uint4*>(Bs + (rsub + 32 * i) * LDA_REG + chunk * 8) = rb[i];
    }
  };

  constexpr int MI2 = MF32 ? BM / (32 * WM) : 1, NI2 = MF32 ? BN / (32 * WN) : 1;  // 32x32 tiles per wave
  f32x4 acc[MF32 ? 1 : MI][MF32 ? 1 : NI];
  f32x16 acc2[MI2][NI2];
  if constexpr (MF32) {
#pragma unroll
    for (int i = 0; i < MI2; ++i)
#pragma unroll
      for (int j = 0; j < NI2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc2[i][j][e] = 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int frow = lane & 15;
  // fragment read: row r, logical 16-B chunk q of the current K-step
  auto frag = [&](const bf16_t* base, int r, int q) {
    if constexpr (DMA)
      return *reinterpret_cast<const bf16x8*>(base + r * LDR + ((q ^ swz<BK>(r)) << 3));
    else
      return *reinterpret_cast<const bf16x8*>(base + r * LDR + (q << 3));
  };
  auto compute = [&](int buf, int kt) {
    (void)kt;
    const bf16_t* As = lds + buf * STAGE;
    const bf16_t* Bs = lds + buf * STAGE + A_ELEMS;
    if constexpr (F8) {
      // lane l holds row l & 15, reduction bytes 32 (l >> 4) .. +31 = logical chunks q0, q0+1
      const int q0 = 2 * (lane >> 4);
      auto frag8 = [&](const bf16_t* base, int r) {
        const uint4 lo = *reinterpret_cast<const uint4*>(base + r * LDR + ((q0 ^ swz_f8(r)) << 3));
        const uint4 hi = *reinterpret_cast<const uint4*>(base + r * LDR + (((q0 + 1) ^ swz_f8(r)) << 3));
        i32x8_c v;
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        return v;
      };
      // the B fragments stay in registers, the A fragments stream one at a time: a 32-B
      // fragment is 8 VGPRs, and holding all MI + NI of them (64) would cost the fused-
      // epilogue dgrads a wave per SIMD (154 VGPRs -> 3 waves; the epilogue needs 4)
      // formats: the gathered operand is e5m2 (bf8) in dgrad (dY), e4m3 in fwd; weights e4m3
      constexpr int FA = DGRAD ? 1 : 0;
      if constexpr (NST1) {
        // single-stage (short-reduction, epilogue-bound) variant: NJ B fragments and ONE A
        // fragment live at a time, i.e. every A fragment is read NI / NJ times from LDS.
        // With 2 fused BN sets the 128x128 instantiation compiles to 152 VGPRs at NJ = 1 or 2
        // and 158 at NJ = 4 -- 3 waves per SIMD in every case (the epilogue sets the peak), so
        // it reads each fragment once (NJ = NI).  With 0 / 1 sets NJ = 1 fits the 128-VGPR cap
        // of 4 waves per SIMD without spills (PMD_F8_MINB, at the kernel template)
#ifndef PMD_F8_NJ
#define PMD_F8_NJ 4
#endif
        constexpr int NJW = ((NB < 2 || PMD_F8_NB2_MINB4) && PMD_F8_MINB >= 4) ? 1 : PMD_F8_NJ;
        constexpr int NJ = NJW < NI ? NJW : NI;
        static_assert(NI % NJ == 0, "NJ divides NI");
#pragma unroll
        for (int j0 = 0; j0 < NI; j0 += NJ) {
          i32x8_c bf[NJ];
#pragma unroll
          for (int jj = 0; jj < NJ; ++jj) bf[jj] = frag8(Bs, wn * (BN / WN) + (j0 + jj) * 16 + frow);
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const i32x8_c af = frag8(As, wm * (BM / WM) + i * 16 + frow);
#pragma unroll
            for (int jj = 0; jj < NJ; ++jj) {
              const int j = j0 + jj;
              acc[i][j] = SWAPC ? __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bf[jj], af, acc[i][j], 0, FA, 0,
                                                                                  127, 0, 127)
                                : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf[jj], acc[i][j], FA, 0, 0,
                                                                                  127, 0, 127);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        return;
      }
      i32x8_c bfg[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bfg[j] = frag8(Bs, wn * (BN / WN) + j * 16 + frow);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const i32x8_c af = frag8(As, wm * (BM / WM) + i * 16 + frow);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = SWAPC ? __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfg[j], af, acc[i][j], 0, FA, 0,
                                                                              127, 0, 127)
                            : __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfg[j], acc[i][j], FA, 0, 0,
                                                                              127, 0, 127);
        // keep the scheduler from hoisting the next A fragment's reads above these MFMAs
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
    if constexpr (MF32) {
      const int r32 = lane & 31;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 af[MI2], bfg[NI2];
        const int q = ks * 2 + (lane >> 5);
#pragma unroll
        for (int i = 0; i < MI2; ++i) {
          const int r = wm * (BM / WM) + i * 32 + r32;
          af[i] = *reinterpret_cast<const bf16x8*>(As + r * LDR + ((q ^ ((r >> 1) & 7)) << 3));
        }
#pragma unroll
        for (int j = 0; j < NI2; ++j) {
          const int r = wn * (BN / WN) + j * 32 + r32;
          bfg[j] = *reinterpret_cast<const bf16x8*>(Bs + r * LDR + ((q ^ ((r >> 1) & 7)) << 3));
        }
#pragma unroll
        for (int i = 0; i < MI2; ++i)
#pragma unroll
          for (int j = 0; j < NI2; ++j)
            acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc2[i][j], 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[MI], bfg[NI];
      const int q = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = frag(As, wm * (BM / WM) + i * 16 + frow, q);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfg[j] = frag(Bs, wn * (BN / WN) + j * 16 + frow, q);
      // PMD_CONV_SETPRIO (A/B knob): raise the wave's issue priority around the MFMA cluster
      // (cdna_hip_programming.md T5: keeps hipcc from moving MFMAs in among the loads)
      if constexpr (PMD_CONV_SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = SWAPC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      if constexpr (PMD_CONV_SETPRIO) __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (DMA) {
    // the loader choice is hoisted out of the K loop: one loop instance per loader
    auto pipeline = [&](auto&& load) {
    if constexpr (NST1) {
      // one LDS stage: load, wait, publish, compute, retire the reads before the next load
      for (int kt = 0; kt < nk; ++kt) {
        if (kt) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        load(kt, 0);
        wait_vmcnt<0>();
        asm volatile("s_barrier" ::: "memory");
        compute(0, kt);
      }
      return;
    }
    // prologue: tiles 0 .. NST-2 in flight
#pragma unroll
    for (int t = 0; t < NST - 1; ++t)
      if (t < nk) load(t, t);
    for (int kt = 0; kt < nk; ++kt) {
      // own DMAs of tile kt done; later tiles (at most NST-2 of them) may still fly
      const int rem = min(NST - 2, nk - 1 - kt);
      if constexpr (NST >= 4) {
        if (rem >= 2) wait_vmcnt<2 * LPT>();
        else if (rem == 1) wait_vmcnt<LPT>();
        else wait_vmcnt<0>();
      } else if constexpr (NST == 3) {
        if (rem >= 1) wait_vmcnt<LPT>();
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
      // publishes tile kt to all waves AND retires every wave's reads of tile kt-1,
      // whose buffer the DMA below overwrites
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + NST - 1 < nk) load(kt + NST - 1, (kt + NST - 1) % NST);
      compute(kt % NST, kt);
    }
    };
    if constexpr (HALO) {
      // ---- halo image of this tile (see the HALO note at the kernel template)
      const int Wd = a.W + 2;
      const int p0 = halo_t * BM;  // first output pixel of the tile (image-local)
      const int hf = p0 / a.W;
      const int hl = (min(p0 + BM, hw_out) - 1) / a.W;
      const int HP = (hl - hf + 3) * Wd;  // input rows hf-1 .. hl+1, columns -1 .. W
      bf16_t* halo = lds;                                  // [pixel][8 chunks], chunk ^= pixel & 7
      bf16_t* Bring = lds + HALO_BYTES / 2;                // NST x [BN][64]
      const bf16_t* img = a.src + (size_t)halo_img * a.H * a.W * a.Cs;
      int hbase[MI];  // halo pixel of each of this lane's A-fragment rows at tap (0, 0)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int p = min(p0 + wm * (BM / WM) + i * 16 + frow, hw_out - 1);  // rows past the image: clamped, masked
        const int h = p / a.W, w = p - (p / a.W) * a.W;
        hbase[i] = (h - hf) * Wd + w;
      }
      auto load_halo = [&](int cb) {
#pragma unroll
        for (int j = 0; j < HALO_CHUNKS / NT; ++j) {
          const int ci = (j * NW + wid_s) * 64 + lane;  // chunk index: lane-linear within the wave
          const int hp = ci >> 3, c = ci & 7;
          const int hr = hp / Wd, hc = hp - hr * Wd;
          const int ih = hf - 1 + hr, iw = hc - 1;
          const bool ok = hp < HP && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          const void* src = ok ? (const void*)(img + ((size_t)(ih * a.W + iw) << a.log2Cs) + cb + ((c ^ (hp & 7)) << 3))
                               : (const void*)g_zero16;
          bf16_t* dst = halo + (size_t)(j * NW + wid_s) * 64 * 8;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
      };
      auto load_b = [&](int kt, int buf) {
        const int cbi = kt / 9, tap = kt - cbi * 9;
        const int tapo = (tap << a.log2Cs) + cbi * 64;  // tap == r * 3 + s
#pragma unroll
        for (int i = 0; i < PB; ++i) {
          const void* src = b_ok[i] ? (const void*)(b_row[i] + tapo + bchunk(i) * 8) : (const void*)g_zero16;
          bf16_t* dst = Bring + buf * B_ELEMS + (wid_s * (BN / NW) + RPI * i) * LDR;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
      };
      auto compute_halo = [&](int buf, int kt) {
        const int tap = kt % 9;
        int r = tap / 3, sx = tap - (tap / 3) * 3;
        if (DGRAD) {  // dX(h, w) gathers dY(h + 1 - r, w + 1 - s)
          r = 2 - r;
          sx = 2 - sx;
        }
        const int toff = r * Wd + sx;
        const bf16_t* Bs = Bring + buf * B_ELEMS;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int q = ks * 4 + (lane >> 4);
          bf16x8 af[MI], bfg[NI];
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int hp = hbase[i] + toff;
            af[i] = *reinterpret_cast<const bf16x8*>(halo + hp * 64 + ((q ^ (hp & 7)) << 3));
          }
#pragma unroll
          for (int j = 0; j < NI; ++j) bfg[j] = frag(Bs, wn * (BN / WN) + j * 16 + frow, q);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc[i][j] = SWAPC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
        }
      };
      const int nkt = (a.Cs >> 6) * 9;
      if constexpr (NST == 3) {
        // 3-deep weight ring: B(kt+1) stays in flight across the barrier (counted vmcnt);
        // only a channel-block switch (halo refill) drains the queue
        load_halo(0);
        load_b(0, 0);
        if (nkt > 1) load_b(1, 1);
        bool drain = true;
        for (int kt = 0; kt < nkt; ++kt) {
          if (drain || kt + 1 >= nkt) wait_vmcnt<0>();
          else wait_vmcnt<PB>();
          // publishes B(kt) (+ the halo) and retires every wave's reads of B(kt-1)
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          drain = false;
          if (kt + 2 < nkt) load_b(kt + 2, (kt + 2) % 3);
          compute_halo(kt % 3, kt);
          if (kt + 1 < nkt && (kt + 1) % 9 == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            load_halo((kt + 1) / 9 * 64);
            drain = true;
          }
        }
      } else {
      load_halo(0);
      load_b(0, 0);
      wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      for (int kt = 0; kt < nkt; ++kt) {
        const bool next = kt + 1 < nkt;
        const bool newcb = next && (kt + 1) % 9 == 0;
        // B(kt+1) into the buffer B(kt-1) used: its reads were retired by the last barrier
        if (next && !newcb) load_b(kt + 1, (kt + 1) & 1);
        compute_halo(kt & 1, kt);
        if (next) {
          if (newcb) {
            // every wave is done with this channel block's halo image: refill it
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            load_halo((kt + 1) / 9 * 64);
            load_b(kt + 1, (kt + 1) & 1);
          }
          wait_vmcnt<0>();
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
      }
      }
    } else if constexpr (P8) {
      if (uni) {
        static_assert(MI % 2 == 0, "P8 splits the wave's row tiles in two halves");
        bf16x8 fa[MI][2], fb[NI][2];
        auto rd_a = [&](int buf, int i) {
          const bf16_t* As = lds + buf * STAGE;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) fa[i][kh] = frag(As, wm * (BM / WM) + i * 16 + frow, kh * 4 + (lane >> 4));
        };
        auto rd_b = [&](int buf) {
          const bf16_t* Bs = lds + buf * STAGE + A_ELEMS;
#pragma unroll
          for (int j = 0; j < NI; ++j)
#pragma unroll
            for (int kh = 0; kh < 2; ++kh)
              fb[j][kh] = frag(Bs, wn * (BN / WN) + j * 16 + frow, kh * 4 + (lane >> 4));
        };
        auto mma = [&](int i) {
#pragma unroll
          for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc[i][j] = SWAPC ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kh], fa[i][kh], acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kh], fb[j][kh], acc[i][j], 0, 0, 0);
        };
        // prologue: tiles 0 and 1 in flight, tile 0's fragments in registers
        load_tile_uni(0, 0);
        if (nk > 1) {
          load_tile_uni(1, 1);
          wait_vmcnt<LPT>();
        } else {
          wait_vmcnt<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int i = 0; i < MI; ++i) rd_a(0, i);
        rd_b(0);
        for (int kt = 0; kt < nk; ++kt) {
          const int cur = kt & 1;
          // every wave's fragment reads of buffer `cur` have retired: re-fill it
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          if (kt + 2 < nk) load_tile_uni(kt + 2, cur);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < MI / 2; ++i) mma(i);
          __builtin_amdgcn_s_setprio(0);
          const bool more = kt + 1 < nk;
          if (more) {
            // tile kt+1 landed (only tile kt+2's loads may still fly) and is visible
            if (kt + 2 < nk) wait_vmcnt<LPT>();
            else wait_vmcnt<0>();
            asm volatile("s_barrier" ::: "memory");
#pragma unroll
            for (int i = 0; i < MI / 2; ++i) rd_a(cur ^ 1, i);
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = MI / 2; i < MI; ++i) mma(i);
          __builtin_amdgcn_s_setprio(0);
          if (more) {
#pragma unroll
            for (int i = MI / 2; i < MI; ++i) rd_a(cur ^ 1, i);
            rd_b(cur ^ 1);
          }
        }
      } else {
        pipeline(load_tile);
      }
    } else {
      if (uni) pipeline(load_tile_uni);
      else pipeline(load_tile);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (F8) {
      const float dsc = 1.f / (a.f8_sa[0] * a.f8_sb[0]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] *= dsc;
    }
  } else {
    if (nk > 0) {
      load_tile(0, 0);
      store_tile(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load_tile(kt + 1, buf ^ 1);
      compute(buf, kt);
      if (kt + 1 < nk) store_tile(buf ^ 1);
      __syncthreads();
    }
  }
  PMD_PROBE_AT(1);

  // ---- epilogue
  constexpr int CPR = BN / 8;  // 16-B chunks per output row
  // fused BN-backward reduce: each thread owns one 8-channel chunk column (NT % CPR == 0)
  static_assert(NT % CPR == 0, "chunk column per thread");
  // NB = the BN-input sets this instantiation handles (launch_k instantiates 0 / 1 / 2
  // to the call's count): the per-set reduce state is the epilogue's register peak,
  // so a one-set dgrad (the common case) carries half of it.  The invstd is applied
  // once after the loop, loaded there, for the same reason.
  constexpr int NBA = NB > 0 ? NB : 1;
  const int nbn = (DGRAD && NB > 0 && a.bn_red[0]) ? (NB > 1 && a.bn_red[1] ? 2 : 1) : 0;
  float bsum[NBA][8], bdot[NBA][8], bmean[NBA][8];
  {
    const int n = n0 + (tid % CPR) * 8;
#pragma unroll
    for (int t = 0; t < NBA; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bsum[t][e] = bdot[t][e] = 0.f;
        bmean[t][e] = 0.f;
      }
    if (nbn && n < a.Nout) {
#pragma unroll
      for (int t = 0; t < NBA; ++t)
        if (t < nbn)
#pragma unroll
          for (int e = 0; e < 8; ++e) bmean[t][e] = a.bn_p[t][n + e];
    }
  }
  // Output rows in groups of G per thread: every global load of a group (addend,
  // masks, BN inputs) is issued before the group's first store (the stores may
  // alias nothing the group reads), so a thread has G x (1-3) HBM reads in
  // flight instead of one dependent load->store chain per row.  Full-step A/B
  // (bench/ab_so.sh): G=2 +0.6% over the serial loop, G=4 -3.6% with default-policy
  // loads (the 4-deep register tile of activation chunks cost more than the extra
  // latency hiding) -- but +0.5% once the epilogue operands stream non-temporal (round 3:
  // 13,440 / 13,435 vs 13,348 / 13,386 img/s, profiles/ab_r03_nt_loads.txt).
  constexpr int ITERS = BM * CPR / NT;
  static_assert((BM * CPR) % NT == 0, "whole epilogue iterations");
#ifndef PMD_EPI_G
#define PMD_EPI_G 4
#endif
#ifndef PMD_F8_NB2_G
#define PMD_F8_NB2_G PMD_EPI_G  // rows in flight of the 2-set single-stage fp8 dgrad epilogue
#endif
  constexpr int GW = (F8 && NST1 && NB == 2) ? PMD_F8_NB2_G : PMD_EPI_G;
  constexpr int G = ITERS < GW ? ITERS : GW;
  static_assert(ITERS % G == 0, "epilogue groups");
  const bool has_add = DGRAD && a.addend, has_amask = DGRAD && a.addend_mask;
  // per-channel addend bias (the linear-BN backward's constant term, ops/functional.py
  // _bnlin_backward): this thread's 8 output channels are fixed for the whole epilogue
  float abias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) abias[e] = 0.f;
  if (DGRAD && a.addend_bias && n0 + (tid % (BN / 8)) * 8 < a.Nout) {
#pragma unroll
    for (int e = 0; e < 8; ++e) abias[e] = a.addend_bias[n0 + (tid % (BN / 8)) * 8 + e];
  }
  // Per thread the chunk column (cc, n) is fixed and the tile row advances by
  // RSTEP per iteration, so for every layer but the strided dgrads the global
  // element offset is one base plus a uniform stride: no per-row integer
  // division / 64-bit multiply in the loop (they were ~1/3 of its VALU issue).
  // EPI_RM: thread row group q reads rows (q >> 1) + 16 (q & 1) + 8 (it & 1) + 32 (it >> 1)
  constexpr int RSTEP = NT / CPR;
  static_assert(!EPI_RM || (RSTEP == 16 && ITERS % 2 == 0), "EPI_RM row order: 16 thread rows");
  auto row_delta = [](int it) { return EPI_RM ? 8 * (it & 1) + 32 * (it >> 1) : it * RSTEP; };
  // EPI_RM64 (8-chunk rows, 36-dword row skew): the 4 thread rows of a 32-lane read
  // group take rows {0, 16, 24, 8} + (q >> 2), which puts both 16-lane halves of every
  // ds_read_b128 group on 4 disjoint 16-dword bank ranges
  const int qr = tid / CPR;
  const int row0 = EPI_RM ? (qr >> 1) + 16 * (qr & 1)
                          : EPI_RM64 ? (qr >> 2) + 8 * ((0x1320 >> (4 * (qr & 3))) & 0xF) : qr;
  const int cc = tid % CPR;
  const int n = n0 + cc * 8;
  const bool n_ok = n < a.Nout;
  const bool phased = DGRAD && a.stride == 2;
  const size_t off0 = (size_t)(m0 + row0) * a.Nout + (n_ok ? n : 0);
  const size_t ostep = (size_t)a.Nout;
  // Prefetch (dgrad): the first row group's global epilogue operands (addend, masks, BN
  // inputs) are issued before the C tile is staged through LDS, so their latency overlaps
  // the staging instead of following it: +0.6% on the full step (profiles/epi_pf_r05.txt).
  // Not for the 4-wave 128-column tiles with <= 1 BN set, which it would cost their 4th
  // wave per SIMD (125 -> 144 VGPRs).
  constexpr bool PF = DGRAD && !(NW == 4 && BN == 128 && NB < 2);
  uint4 pf_ad[PF ? G : 1], pf_yy[NBA][PF ? G : 1];
  uint32_t pf_am[PF ? G : 1], pf_mb[PF ? G : 1];
  if constexpr (PF) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int row = row0 + row_delta(g);
      const int m = m0 + row;
      const bool okg = m < Mp && n_ok;
      size_t o = off0 + (size_t)row_delta(g) * ostep;
      if (phased) {
        const int mm = okg ? m : 0;
        const int nb = mm / ohw, rem = mm - nb * ohw;
        const int hh = rem / OWp, ww = rem - hh * OWp;
        o = (((size_t)nb * a.OH + 2 * hh + ph) * a.OW + 2 * ww + pw) * a.Nout + (n_ok ? n : 0);
      }
      if (!okg) o = 0;
      if (has_add && okg) {
        pf_ad[g] = ld16n<NT_EPI_A>(a.addend + o);
        pf_am[g] = has_amask ? a.addend_mask[o >> 3] : 0xffu;
      }
      if (nbn && okg) {
        pf_mb[g] = a.bn_mask ? a.bn_mask[o >> 3] : 0xffu;
#pragma unroll
        for (int t = 0; t < NBA; ++t)
          if (t < nbn) pf_yy[t][g] = a.bn_y[t] ? ld16n<NT_EPI_Y>(a.bn_y[t] + o) : make_uint4(0, 0, 0, 0);
      }
    }
  }
  bf16_t* Cs = lds;
  const int crow0 = wm * (BM / WM) + (lane >> 4) * 4;
  const int ccol0 = wn * (BN / WN) + (lane & 15);
  float csum[NI], csq[NI], cshift[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    csum[j] = 0.f;
    csq[j] = 0.f;
    cshift[j] = 0.f;
    if (STATS && a.shift) {
      const int col = n0 + (MF32 ? wn * (BN / WN) + j * 32 + (lane & 31) : ccol0 + j * 16);
      if ((!MF32 || j < NI2) && col < a.Nout) cshift[j] = a.shift[col];
    }
  }
  if constexpr (MF32) {
    // 32x32 C layout: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < MI2; ++i)
#pragma unroll
      for (int j = 0; j < NI2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const bf16_t h = f2bf(acc2[i][j][e]);
          const int row = wm * (BM / WM) + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          Cs[row * LDC + wn * (BN / WN) + j * 32 + (lane & 31)] = h;
          if (STATS) {
            // rows past M (zero accumulators) must not contribute (0 - K) to the shifted sums
            const float v = m0 + row < Mp ? bf2f(h) - cshift[j] : 0.f;
            csum[j] += v;
            csq[j] += v * v;
          }
        }
  } else if constexpr (SWAPC) {
    // C^T layout: pixel = lane & 15, channels (lane >> 4) * 4 + 0..3 (8-B aligned:
    // LDC * 2 = 2 BN + 16 bytes per row).  A ds_write_b64 is served in groups of 16
    // lanes on 32 banks: the 16 rows of a group, 4 dwords apart, would pair up rows
    // r and r + 8 on the same two banks, so rows with bit 3 set store their two 8-B
    // halves of every 16-B chunk swapped (EPI_SW; the row reads swap them back).
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wm * (BM / WM) + i * 16 + (lane & 15);
        const int colw = wn * (BN / WN) + j * 16 + (lane >> 4) * 4;   // logical channel (4 per lane)
        const int col = colw ^ (EPI_SW ? ((lane >> 1) & 4) : 0);
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        *reinterpret_cast<uint2*>(Cs + row * LDC + col) = make_uint2(lo, hi);
      }
  } else {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16_t h = f2bf(acc[i][j][e]);
          Cs[(crow0 + i * 16 + e) * LDC + ccol0 + j * 16] = h;
          if (STATS) {
            const float v = m0 + crow0 + i * 16 + e < Mp ? bf2f(h) - cshift[j] : 0.f;
            csum[j] += v;
            csq[j] += v * v;
          }
        }
  }
  if (STATS && MF32) {
    // column sums: lanes l and l+32 hold the two row halves of column l & 31
    float* st = reinterpret_cast<float*>(smem + SMEM);  // [WM][2][BN]
#pragma unroll
    for (int j = 0; j < NI2; ++j) {
      float s1 = csum[j], s2 = csq[j];
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 32) {
        st[(wm * 2 + 0) * BN + wn * (BN / WN) + j * 32 + lane] = s1;
        st[(wm * 2 + 1) * BN + wn * (BN / WN) + j * 32 + lane] = s2;
      }
    }
  }
  if (STATS && !MF32) {
    float* st = reinterpret_cast<float*>(smem + SMEM);  // [WM][2][BN]
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
  PMD_PROBE_AT(2);
  if (STATS) {
    const float* st = reinterpret_cast<const float*>(smem + SMEM);
    for (int c = tid; c < 2 * BN; c += NT) {
      const int which = c / BN, col = c % BN;
      if (n0 + col < a.Nout) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) v += st[(w * 2 + which) * BN + col];
        if constexpr (!(PMD_TIMING_NO_ATOMICS & 1))  // timing-only A/B knob: what the statistics atomics cost
          atomicAdd(a.stats + (stat_slot(blockIdx.y * tilesM + mt, a.nslots) * 2 + which) * a.Nout + n0 + col, v);
      }
    }
  }
  // fully unrolled (A/B: +0.8% step over the rolled loop with per-row index
  // math; an LDS lookup table expanding the ReLU mask bytes measured -2.7%).
  // Skipped by a statistics-only forward (out == nullptr: the stats are complete).
  if (a.out || nbn)
#pragma unroll
  for (int it0 = 0; it0 < ITERS; it0 += G) {
    size_t off[G];
    bool ok[G];
    uint4 v[G], ad[G], yy[NBA][G];
    uint32_t am[G], mb[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int row = row0 + row_delta(it0 + g);
      const int m = m0 + row;
      ok[g] = m < Mp && n_ok;
      off[g] = off0 + (size_t)row_delta(it0 + g) * ostep;
      if (phased) {
        const int mm = ok[g] ? m : 0;
        const int nb = mm / ohw, rem = mm - nb * ohw;
        const int hh = rem / OWp, ww = rem - hh * OWp;
        off[g] = (((size_t)nb * a.OH + 2 * hh + ph) * a.OW + 2 * ww + pw) * a.Nout + (n_ok ? n : 0);
      }
      if (!ok[g]) off[g] = 0;
      v[g] = *reinterpret_cast<const uint4*>(Cs + row * LDC + cc * 8);
      if constexpr (EPI_SW) {
        // rows with bit 3 set hold their 8-B halves swapped (compile-time under EPI_RM)
        const bool sw = EPI_RM ? ((it0 + g) & 1) != 0 : ((row >> 3) & 1) != 0;
        if (sw) v[g] = make_uint4(v[g].z, v[g].w, v[g].x, v[g].y);
      }
      if (PF && it0 == 0) {
        ad[g] = pf_ad[g];
        am[g] = pf_am[g];
        mb[g] = pf_mb[g];
#pragma unroll
        for (int t = 0; t < NBA; ++t) yy[t][g] = pf_yy[t][g];
      } else {
        if (has_add && ok[g]) {
          ad[g] = ld16n<NT_EPI_A>(a.addend + off[g]);
          am[g] = has_amask ? a.addend_mask[off[g] >> 3] : 0xffu;
        }
        if (nbn && ok[g]) {
          mb[g] = a.bn_mask ? a.bn_mask[off[g] >> 3] : 0xffu;
#pragma unroll
          for (int t = 0; t < NBA; ++t)
            if (t < nbn) yy[t][g] = a.bn_y[t] ? ld16n<NT_EPI_Y>(a.bn_y[t] + off[g]) : make_uint4(0, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!ok[g]) continue;
      uint4 o = v[g];
      if (has_add) {
        float f[8], ga[8];
        unpack8(o, f);
        unpack8(ad[g], ga);
#pragma unroll
        for (int e = 0; e < 8; ++e) ga[e] = ((am[g] >> e) & 1u) ? ga[e] : 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += ga[e] + abias[e];
        o = pack8(f);
      }
      if (nbn) {
        // the output IS a BN site's dz; every consumer gates it with this same ReLU
        // mask (BN backward, identity-path addend), so store dzm = dz * mask (bit-exact
        // zeroing; the fused reduce below sums exactly what is stored)
        const uint32_t mk = mb[g];
        o.x &= ((mk & 1u) ? 0x0000ffffu : 0u) | ((mk & 2u) ? 0xffff0000u : 0u);
        o.y &= ((mk & 4u) ? 0x0000ffffu : 0u) | ((mk & 8u) ? 0xffff0000u : 0u);
        o.z &= ((mk & 16u) ? 0x0000ffffu : 0u) | ((mk & 32u) ? 0xffff0000u : 0u);
        o.w &= ((mk & 64u) ? 0x0000ffffu : 0u) | ((mk & 128u) ? 0xffff0000u : 0u);
      }
      // PMD_CONV_ST_PASS (A/B): 0 = both passes as PMD_NT_MASK says, 1 = forward outputs only,
      // 2 = data-gradient outputs only
      if (a.out) {
        if constexpr (PMD_CONV_ST_PASS == 0 || (PMD_CONV_ST_PASS == 1) == !DGRAD)
          st16n<NT_CONV_ST>(a.out + off[g], o);
        else
          *reinterpret_cast<uint4*>(a.out + off[g]) = o;
      }
      if (nbn) {
        float d[8];
        unpack8(o, d);
#pragma unroll
        for (int t = 0; t < NBA; ++t) {
          if (t < nbn) {
            float yv[8];
            unpack8(yy[t][g], yv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              bsum[t][e] += d[e];
              bdot[t][e] += d[e] * (yv[e] - bmean[t][e]);  // * invstd once, after the loop
            }
          }
        }
      }
    }
  }
#if PMD_DGRAD_PROBE
  if constexpr (DGRAD) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's epilogue stores have landed
    __syncthreads();
  }
#endif
  PMD_PROBE_AT(3);
  if (nbn && n_ok) {
#pragma unroll
    for (int t = 0; t < NBA; ++t)
      if (t < nbn)
#pragma unroll
        for (int e = 0; e < 8; ++e) bdot[t][e] *= a.bn_p[t][a.Nout + n + e];
  }
  if (nbn) {
    // block-level combine of the 256/CPR threads sharing a chunk column, then one
    // fp32 atomic per channel per block into a kStatSlots slot (like conv_fwd stats)
    __syncthreads();  // everyone is done reading Cs
    float* part = reinterpret_cast<float*>(smem);  // [NT][PSTR]
#pragma unroll
    for (int t = 0; t < NBA; ++t) {
      if (t >= nbn) break;  // uniform
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        part[tid * PSTR + e] = bsum[t][e];
        part[tid * PSTR + 8 + e] = bdot[t][e];
      }
      __syncthreads();
      for (int q = tid; q < CPR * 16; q += NT) {
        const int col = q >> 4, k = q & 15;
        float acc2 = 0.f;
        for (int r = col; r < NT; r += CPR) acc2 += part[r * PSTR + k];
        const int n = n0 + col * 8 + (k & 7);
        if (n < a.Nout && !(PMD_TIMING_NO_ATOMICS & 2))
          atomicAdd(a.bn_red[t] + (stat_slot(blockIdx.y * tilesM + mt, a.nslots) * 2 + (k >> 3)) * a.Nout + n, acc2);
      }
      __syncthreads();
    }
  }
#if PMD_DGRAD_PROBE
  if constexpr (DGRAD) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PMD_PROBE_AT(4);
    const unsigned long long pwc1 = wall_clock64();
    if (tid == 0 && g_probe_buf) {
      const unsigned int q = (blockIdx.x + 7u * blockIdx.y) & 255u, per = g_probe_cap >> 8;
      const unsigned int slot = atomicAdd(&g_probe_ctr[q * 32], 1u);
      if (slot < per) {
        unsigned long long* r = g_probe_buf + ((size_t)q * per + slot) * 16;
        r[0] = pwc0;
        r[1] = pwc1;
#pragma unroll
        for (int k = 0; k < 5; ++k) r[2 + k] = pt[k];
        r[7] = ((unsigned long long)a.M << 32) | ((unsigned long long)a.Nout << 16) | (unsigned)a.Kg;
        r[8] = ((unsigned long long)BM << 48) | ((unsigned long long)BN << 32) | ((unsigned long long)BK << 16) |
               (NST << 8) | (F8 ? 16 : 0) | (NST1 ? 32 : 0) | (HALO ? 64 : 0) | (P8 ? 128 : 0);
        r[9] = ((unsigned long long)a.stride << 32) | (nbn << 8) | (has_add ? 1 : 0) | (NW << 16);
        r[10] = blockIdx.x | ((unsigned long long)blockIdx.y << 32);
        r[11] = (unsigned long long)(size_t)a.out;
      }
    }
  }
#endif
}

#if PMD_DGRAD_PROBE
// probe buffer (cap records of 16 words, cap/256 per counter; nullptr: off); returns 1 in a probe build
int conv_probe_set(void* buf, int cap) {
  unsigned long long* p = reinterpret_cast<unsigned long long*>(buf);
  static const unsigned int zero[256 * 32] = {0};
  const unsigned int c = (unsigned int)cap;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_probe_buf), &p, sizeof(p)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_probe_cap), &c, sizeof(c)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_probe_ctr), zero, sizeof(zero)) != hipSuccess) return -1;
  return 1;
}
int conv_probe_count() {  // the largest per-counter fill (records beyond cap/256 were dropped)
  static unsigned int c[256 * 32];
  if (hipMemcpyFromSymbol(c, HIP_SYMBOL(g_probe_ctr), sizeof(c)) != hipSuccess) return -1;
  unsigned int m = 0;
  for (int i = 0; i < 256; ++i) m = c[32 * i] > m ? c[32 * i] : m;
  return (int)m;
}
#else
int conv_probe_set(void*, int) { return 0; }
int conv_probe_count() { return 0; }
#endif

// fp32 param (physical K,R,S,C = channels_last [K,C,R,S]) -> bf16 images:
//   wk  [K][R][S][Cp]   (B^T of the forward GEMM, zero-padded channels)
//   wkt [Cp][R][S][K]   (B^T of the dgrad GEMM), optional
__global__ void conv_weight_prep_kernel(const float* __restrict__ w, bf16_t* __restrict__ wk,
                                        bf16_t* __restrict__ wkt, int K, int RS, int C, int Cp) {
  const int total = K * RS * Cp;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % Cp;
    const int rs = (i / Cp) % RS;
    const int k = i / (Cp * RS);
    const float v = c < C ? w[((size_t)k * RS + rs) * C + c] : 0.f;
    const bf16_t h = f2bf(v);
    wk[i] = h;
    if (wkt) wkt[((size_t)c * RS + rs) * K + k] = h;
  }
}

// All conv weight images of a model in ONE launch (instead of one small launch
// per conv per step): block b finds its descriptor by scanning the block-start
// table (<= a few dozen entries) once, then grid-strides inside that weight.
// mode bit 0: forward images wk (8 channels per thread: two float4 reads, one 16-B
// write); bit 1: dgrad images wkt.  The training step refreshes wk on the main
// stream (the stem needs it at once) and wkt on the idle side stream during the
// forward (the first dgrad is milliseconds later).
__global__ __launch_bounds__(256) void conv_weight_prep_grouped_kernel(const WeightPrepDesc* __restrict__ descs,
                                                                      const int* __restrict__ block_start, int n,
                                                                      int mode) {
  __shared__ int e_sh;
  __shared__ float tile[64][65];   // pass 2: one 64 (k) x 64 (c) slice of a tap, odd row pitch
  if (threadIdx.x == 0) {
    int e = 0;
    while (e + 1 < n && block_start[e + 1] <= (int)blockIdx.x) ++e;
    e_sh = e;
  }
  __syncthreads();
  const WeightPrepDesc d = descs[e_sh];
  const int lb = blockIdx.x - block_start[e_sh];
  const int nb = block_start[e_sh + 1] - block_start[e_sh];
  // pass 1: wk [K][RS][Cp] in its own order, 8 channels (16 B) per thread (Cp % 8 == 0)
  if (mode & 1) {
    const int total8 = d.K * d.RS * d.Cp / 8;
    for (int i = lb * blockDim.x + threadIdx.x; i < total8; i += nb * blockDim.x) {
      const int e0 = i * 8;
      const int c0 = e0 % d.Cp;
      const int krs = e0 / d.Cp;  // k * RS + rs
      const float* src = d.w + (size_t)krs * d.C + c0;
      float v[8];
      if (d.C == d.Cp && (d.C & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(src);
        const float4 b = *reinterpret_cast<const float4*>(src + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = c0 + e < d.C ? src[e] : 0.f;
      }
      uint4 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
      o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
      *reinterpret_cast<uint4*>(d.wk + e0) = o;
    }
  }
  // pass 2: wkt [Cp][RS][K], the per-tap [K][C] -> [C][K] transpose through LDS in 64 x 64 tiles:
  // reads along c and writes along k both coalesced (the element-per-thread version read one
  // fp32 per 64-B line: 141 -> 61 us per step, profiles/weight_prep_tile_r05.txt; one walk
  // writing both images in mode 3 measured slower, 70 us: fewer bytes but latency-bound)
  if ((mode & 2) && d.wkt) {
    const int kt = (d.K + 63) / 64, ct = (d.Cp + 63) / 64;
    const int ntiles = d.RS * kt * ct;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 columns x 4 rows per pass
    for (int t = lb; t < ntiles; t += nb) {
      const int rs = t / (kt * ct);
      const int rem = t - rs * kt * ct;
      const int k0 = (rem / ct) * 64, c0 = (rem % ct) * 64;
#pragma unroll 4
      for (int r = ty; r < 64; r += 4) {
        const int k = k0 + r, c = c0 + tx;
        tile[r][tx] = (k < d.K && c < d.C) ? d.w[((size_t)k * d.RS + rs) * d.C + c] : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int r = ty; r < 64; r += 4) {
        const int c = c0 + r, k = k0 + tx;
        if (c < d.Cp && k < d.K) d.wkt[((size_t)c * d.RS + rs) * d.K + k] = f2bf(tile[tx][r]);
      }
      __syncthreads();
    }
  }
}

void conv_weight_prep_grouped_launch(const WeightPrepDesc* d_descs, const int* d_block_start, int n,
                                     int total_blocks, hipStream_t st, int mode) {
  hipLaunchKernelGGL(conv_weight_prep_grouped_kernel, dim3(total_blocks), dim3(256), 0, st, d_descs,
                     d_block_start, n, mode);
}

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// Operand staging / pipeline variant (conv_set_impl or PMD_CONV_IMPL):
//   0 register staging, BK=64, 2 stages
//   1 LDS-DMA BK=64, 2 stages      2 LDS-DMA BK=32, 4 stages
//   3 LDS-DMA BK=64, 3 stages      4 LDS-DMA BK=32, 3 stages
//   6 LDS-DMA BK=64, 2 stages, 32x32x16 MFMA
//   7 LDS-DMA BK=32, 2 stages (128x128 tiles; 128x64 -> 4)
//   5 (default) per shape: BK=32/3 stages for short reductions (Kg <= 512: the
//     prologue/epilogue dominate, a shallower K-tile fills the pipe sooner),
//     BK=64/2 stages otherwise (fewer barriers per MFMA) -- measured on all 23
//     ResNet-50 layer shapes x {fwd, dgrad} (profiles/conv_bench_r01_v5_impls.txt).
static int g_conv_impl = -1;

void conv_set_impl(int impl) { g_conv_impl = impl; }

static int conv_impl() {
  if (g_conv_impl < 0) {
    const char* e = getenv("PMD_CONV_IMPL");
    g_conv_impl = (e && e[0] >= '0' && e[0] <= '7') ? e[0] - '0' : 5;
  }
  return g_conv_impl;
}

template <int BM, int BN, int BK, int NST, bool DGRAD, bool STATS, bool DMA, bool MF32 = false,
          int WM = 2, int WN = 2, bool P8 = false, bool HALO = false>
static void launch_k(const ConvArgs& a, hipStream_t st) {
  const bool ph2 = DGRAD && a.stride == 2;
  const int Mgrid = ph2 ? a.N * ((a.OH + 1) >> 1) * ((a.OW + 1) >> 1) : a.M;
  const int mtiles = HALO ? a.N * ((a.OH * a.OW + BM - 1) / BM) : (Mgrid + BM - 1) / BM;
  const int tiles = mtiles * ((a.Nout + BN - 1) / BN);
  const int phases = ph2 ? 4 : 1;
  const dim3 grid(tiles, phases, a.batch), block(64 * WM * WN);
  if constexpr (DGRAD) {  // instantiation per count of fused BN-reduce input sets (register peak)
    const int nb = a.bn_red[0] ? (a.bn_red[1] ? 2 : 1) : 0;
    if (nb == 2)
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, NST, DGRAD, STATS, DMA, MF32, WM, WN, P8, HALO, 2>), grid,
                         block, 0, st, a);
    else if (nb == 1)
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, NST, DGRAD, STATS, DMA, MF32, WM, WN, P8, HALO, 1>), grid,
                         block, 0, st, a);
    else
      hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, NST, DGRAD, STATS, DMA, MF32, WM, WN, P8, HALO, 0>), grid,
                         block, 0, st, a);
  } else {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, BK, NST, DGRAD, STATS, DMA, MF32, WM, WN, P8, HALO, 0>), grid,
                       block, 0, st, a);
  }
}

// HALO conv (see the kernel): 3x3, stride 1, pad 1, Cs % 64 == 0, 7 <= W <= 56
static bool halo_ok(const ConvArgs& a) {
  return a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.Cs % 64 == 0 && a.W >= 7 && a.W <= 56 &&
         a.OH == a.H && a.OW == a.W;
}
template <bool DGRAD, bool STATS>
static void launch_halo(const ConvArgs& a, hipStream_t st, int depth) {
  if (a.Nout <= 64) {
    if (depth == 3) launch_k<128, 64, 64, 3, DGRAD, STATS, true, false, 2, 2, false, true>(a, st);
    else launch_k<128, 64, 64, 2, DGRAD, STATS, true, false, 2, 2, false, true>(a, st);
  } else {
    if (depth == 3) launch_k<128, 128, 64, 3, DGRAD, STATS, true, false, 2, 2, false, true>(a, st);
    else launch_k<128, 128, 64, 2, DGRAD, STATS, true, false, 2, 2, false, true>(a, st);
  }
}

// P8 register-resident fragment pipeline (see the kernel): 0 = 256x256 (8 waves 2x4),
// 1 = 256x128 (8 waves 4x2), 2 = 128x128 (4 waves 2x2), 3 = 128x128 (8 waves 4x2)
template <bool DGRAD, bool STATS>
static void launch_p8(const ConvArgs& a, hipStream_t st, int shape) {
  switch (shape) {
    case 0: launch_k<256, 256, 64, 2, DGRAD, STATS, true, false, 2, 4, true>(a, st); break;
    case 1: launch_k<256, 128, 64, 2, DGRAD, STATS, true, false, 4, 2, true>(a, st); break;
    case 3: launch_k<128, 128, 64, 2, DGRAD, STATS, true, false, 4, 2, true>(a, st); break;
    default: launch_k<128, 128, 64, 2, DGRAD, STATS, true, false, 2, 2, true>(a, st); break;
  }
}

template <int BM, int BN, bool DGRAD, bool STATS>
static void launch_t(const ConvArgs& a, hipStream_t st, int impl) {
  if (impl == 5) impl = a.Kg <= 512 ? 4 : 1;
  switch (impl) {
    case 0: launch_k<BM, BN, 64, 2, DGRAD, STATS, false>(a, st); break;
    case 1: launch_k<BM, BN, 64, 2, DGRAD, STATS, true>(a, st); break;
    case 2: launch_k<BM, BN, 32, 4, DGRAD, STATS, true>(a, st); break;
    case 3: launch_k<BM, BN, 64, 3, DGRAD, STATS, true>(a, st); break;
    case 7:  // BK=32 x2 stages (4 blocks/CU); the 64-column tile is too small for it
      if constexpr (BN >= 128) launch_k<BM, BN, 32, 2, DGRAD, STATS, true>(a, st);
      else launch_k<BM, BN, 32, 3, DGRAD, STATS, true>(a, st);
      break;
    case 6:  // 32x32x16 MFMA: needs the uniform-tap loader (Cs % 64 == 0)
      if (a.Cs % 64 == 0) launch_k<BM, BN, 64, 2, DGRAD, STATS, true, true>(a, st);
      else launch_k<BM, BN, 64, 2, DGRAD, STATS, true>(a, st);
      break;
    default: launch_k<BM, BN, 32, 3, DGRAD, STATS, true>(a, st); break;
  }
}

// 8-wave 256-row tiles (LDS-DMA only; one block per CU).  Pipeline by
// PMD_CONV_BIGPIPE: 0 (default) BK=64 x2 stages, 1 BK=64 x3, 2 BK=32 x4, 3 BK=64 x2 on
// the 32x32x16 MFMA.
static int g_big_pipe = -1;
void conv_set_big_pipe(int p) { g_big_pipe = p; }
static int big_pipe() {
  if (g_big_pipe < 0) {
    const char* e = getenv("PMD_CONV_BIGPIPE");
    g_big_pipe = (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : 0;
  }
  return g_big_pipe;
}

template <int BM, int BN, int WM, int WN, bool DGRAD, bool STATS>
static void launch_big(const ConvArgs& a, hipStream_t st) {
  switch (big_pipe()) {
    case 1:  // 3 x (256+BN) x 64 x 2 B: fits the CU's LDS only at BN = 128
      if constexpr (BN <= 128) launch_k<BM, BN, 64, 3, DGRAD, STATS, true, false, WM, WN>(a, st);
      else launch_k<BM, BN, 64, 2, DGRAD, STATS, true, false, WM, WN>(a, st);
      break;
    case 2: launch_k<BM, BN, 32, 4, DGRAD, STATS, true, false, WM, WN>(a, st); break;
    case 3:  // 32x32x16 MFMA (half the MFMA instructions per FLOP); needs the uniform-tap loader
      if (a.Cs % 64 == 0) launch_k<BM, BN, 64, 2, DGRAD, STATS, true, true, WM, WN>(a, st);
      else launch_k<BM, BN, 64, 2, DGRAD, STATS, true, false, WM, WN>(a, st);
      break;
    default: launch_k<BM, BN, 64, 2, DGRAD, STATS, true, false, WM, WN>(a, st); break;
  }
}

// Tile policy (conv_set_tile or PMD_CONV_TILE): 0 auto (autotuned per shape, else
// 128-row tiles), 1 128-row tiles only, 2 256x128 wherever legal, 3 256x256
// wherever legal (Nout >= 256), 4/5 8-wave 128-row tiles (see launch_w8),
// 6..9 the P8 pipeline shapes 0..3 (see launch_p8) wherever legal, 10 the 64x128 tile, 11 / 12
// the halo-image 3x3 kernel, 14 the fused Winograd forward (kernels/winograd.hip) wherever legal.
static int g_conv_tile = -1;
void conv_set_tile(int t) { g_conv_tile = t; }
static int conv_tile() {
  if (g_conv_tile < 0) {
    const char* e = getenv("PMD_CONV_TILE");
    const int v = e ? atoi(e) : 0;
    g_conv_tile = (v >= 0 && v <= 14) ? v : 0;
  }
  return g_conv_tile;
}

// 8-wave 128-row tiles (4 waves per SIMD at 2 blocks/CU, half the MFMA work per
// wave): 128x128 as 2x4 (policy 4) or 4x2 (policy 5) waves, 128x64 as 4x2
template <bool DGRAD, bool STATS>
static void launch_w8(const ConvArgs& a, hipStream_t st, int shape) {
  if (a.Nout <= 64) launch_k<128, 64, 64, 2, DGRAD, STATS, true, false, 4, 2>(a, st);
  else if (shape == 0) launch_k<128, 128, 64, 2, DGRAD, STATS, true, false, 2, 4>(a, st);
  else launch_k<128, 128, 64, 2, DGRAD, STATS, true, false, 4, 2>(a, st);
}

static bool big_ok(const ConvArgs& a) {
  // 256-row tiles need the uniform-tap DMA loader (Cs >= 64) and >= 128 output channels
  return a.Cs >= 64 && a.Nout >= 128;
}

// One candidate kernel configuration of the autotuner:
//   0  128-row tile, LDS-DMA BK=32 x3 stages      1  128-row tile, LDS-DMA BK=64 x2
//   2  256x256 tile (8 waves), BK=64 x2            3  256x128 tile (8 waves), BK=64 x2
//   4  128x128 tile, LDS-DMA BK=32 x2 stages: 34 KB of LDS -> 4 blocks (16 waves) per
//      CU, for the short-reduction dgrads whose fused epilogue (addend, BN-backward
//      reduce over 1-2 BN inputs) streams 3-4 activation tensors and needs the
//      extra waves to hide HBM latency
//   5  8-wave 128-row tile (launch_w8): 4 waves per SIMD at the LDS of a 4-wave
//      block (measured +3..7% on several forward 3x3 / 1x1 layers, slower dgrads)
//   6..9 P8 pipeline shapes 0..3 (launch_p8): needs the uniform-tap loader (Cs % 64 == 0);
//      256-row shapes need >= 128 output channels (256x256: >= 256)
static bool p8_ok(int shape, const ConvArgs& a) {
  if (a.Cs % 64 != 0) return false;
  if (shape == 0) return a.Nout >= 256;
  if (shape == 1) return a.Nout >= 128;
  return a.Nout > 64;
}
//   10 64x128 tile, LDS-DMA BK=32 x2 stages (Nout > 64): half the rows per block, so
//      an epilogue-bound short-reduction dgrad gets twice the blocks (and half the
//      serial epilogue rows per thread) in flight
//   14 fused Winograd F(2x2,3x3) forward (kernels/winograd.hip: filter transform + one kernel with
//      the input transform, 16 MFMA GEMMs, output transform and the statistics epilogue)
static bool wino_ok(const ConvArgs& a) {
  return a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.OH == a.H && a.OW == a.W &&
         a.Cs % 64 == 0 && a.Nout % 64 == 0 && a.batch == 1 && a.out && !a.addend && !a.f8_sa;
}
template <bool DGRAD, bool STATS>
static void launch_choice(int c, const ConvArgs& a, hipStream_t st) {
  if constexpr (!DGRAD) {
    if (c == 14 && wino_ok(a) &&
        winograd_conv_fwd_run(a.src, a.wt, a.out, STATS ? a.stats : nullptr, STATS ? a.shift : nullptr, a.N, a.H,
                              a.W, a.Cs, a.Nout, a.nslots, st) == 0)
      return;   // (a failed launch -- e.g. its scratch cannot grow inside a capture -- runs the GEMM)
  }
  if ((c == 11 || c == 12) && halo_ok(a)) {
    launch_halo<DGRAD, STATS>(a, st, c == 12 ? 3 : 2);
  } else if (c == 10 && a.Nout > 64) {
    launch_k<64, 128, 32, 2, DGRAD, STATS, true>(a, st);
  } else if (c >= 6 && c <= 9 && p8_ok(c - 6, a)) {
    launch_p8<DGRAD, STATS>(a, st, c - 6);
  } else if (c == 5 && a.Cs >= 64) {
    launch_w8<DGRAD, STATS>(a, st, 0);
  } else if (c == 4 && a.Nout > 64) {
    launch_k<128, 128, 32, 2, DGRAD, STATS, true>(a, st);
  } else if (c == 2 && big_ok(a) && a.Nout >= 256) {
    launch_k<256, 256, 64, 2, DGRAD, STATS, true, false, 2, 4>(a, st);
  } else if (c == 3 && big_ok(a)) {
    launch_k<256, 128, 64, 2, DGRAD, STATS, true, false, 4, 2>(a, st);
  } else {
    const int impl = c == 0 ? 4 : 1;
    if (a.Nout <= 64) launch_t<128, 64, DGRAD, STATS>(a, st, impl);
    else launch_t<128, 128, DGRAD, STATS>(a, st, impl);
  }
}

// ---- per-shape autotuner: the framework's cudnn.benchmark (reference main.py:45).
// The first launch of every (shape, pass) outside HIP-graph capture times each
// legal candidate on the live operands (best of 3 after one warm launch, HIP
// events on the caller's stream) and caches the winner; later launches go
// straight to it.  Candidates write the real output (every candidate overwrites
// all of it, and the chosen kernel runs last), but BN statistics go to a
// scratch slot buffer and the fused BN-backward reduce into scratch sums, so
// nothing accumulates twice.  PMD_CONV_AUTOTUNE=0 disables it
// (then: 128-row tiles, BK by reduction depth); PMD_CONV_AUTOTUNE_LOG=1 prints
// every decision.
struct TuneKey {
  int v[13];
  bool operator<(const TuneKey& o) const {
    for (int i = 0; i < 13; ++i)
      if (v[i] != o.v[i]) return v[i] < o.v[i];
    return false;
  }
};
static std::map<TuneKey, int> g_tune;
static std::mutex g_tune_mu;
static int g_autotune = -1;
void conv_set_autotune(int on) { g_autotune = on; }
static bool autotune_on() {
  if (g_autotune < 0) {
    const char* e = getenv("PMD_CONV_AUTOTUNE");
    g_autotune = (e && e[0] == '0') ? 0 : 1;
  }
  return g_autotune == 1;
}
int conv_autotune_entries() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  return (int)g_tune.size();
}
void conv_autotune_clear() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tune.clear();
}
// flat table export/import (persisted tuning table, rank-0 broadcast): each entry
// is the 13 key fields followed by the chosen candidate
std::vector<int> conv_autotune_export() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::vector<int> out;
  for (const auto& kv : g_tune) {
    out.insert(out.end(), kv.first.v, kv.first.v + 13);
    out.push_back(kv.second);
  }
  return out;
}
int conv_autotune_import(const std::vector<int>& flat) {
  if (flat.size() % 14) return -1;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  for (size_t i = 0; i < flat.size(); i += 14) {
    TuneKey k;
    for (int j = 0; j < 13; ++j) k.v[j] = flat[i + j];
    g_tune[k] = flat[i + 13];
  }
  return (int)(flat.size() / 14);
}

template <bool DGRAD, bool STATS>
static int tune(const ConvArgs& a0, hipStream_t st) {
  ConvArgs a = a0;
  a.nslots = kStatSlots;  // the scratch sums below have kStatSlots slots (deterministic mode too)
  // the fused BN-backward reduce is part of the cost being compared (it decides
  // the epilogue-bound dgrads), so the timing runs keep it, aimed at scratch sums
  static float* scratch_red = nullptr;
  static int scratch_red_n = 0;
  if (a.bn_red[0]) {
    const int need = 2 * kStatSlots * 2 * a.Nout;
    if (need > scratch_red_n) {
      if (scratch_red) (void)hipFree(scratch_red);
      if (hipMalloc(&scratch_red, sizeof(float) * need) != hipSuccess) return -1;
      scratch_red_n = need;
    }
    a.bn_red[0] = scratch_red;
    if (a.bn_red[1]) a.bn_red[1] = scratch_red + kStatSlots * 2 * a.Nout;
  }
  static float* scratch_stats = nullptr;
  static int scratch_n = 0;
  if (STATS) {
    const int need = kStatSlots * 2 * a.Nout;
    if (need > scratch_n) {
      if (scratch_stats) (void)hipFree(scratch_stats);
      if (hipMalloc(&scratch_stats, sizeof(float) * need) != hipSuccess) return -1;
      scratch_n = need;
    }
    a.stats = scratch_stats;
  }
  static hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!e0) {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
  }
  int best = -1;
  float best_ms = 1e30f;
  char all[256];   // PMD_CONV_AUTOTUNE_LOG=2: every candidate's time
  int alln = 0;
  all[0] = 0;
  // the P8 shapes (6..9) measured equal or slower than 0..5 on every R50 layer
  // (profiles/conv_p8_r02.txt): forced-policy only, not timed by the tuner
  // (10, the 64x128 tile, measured slower than 0..5 on every short-K dgrad --
  // profiles/dgrad_epi_r02_tile10.txt -- so it is a forced policy only)
  // (the 32x32x16-MFMA 128-row tile measured slower than 0..5 on every ResNet-50 shape: not a
  // candidate; PMD_CONV_IMPL=6 forces it)
  for (int c : {0, 1, 2, 3, 4, 5, 14}) {
    if ((c == 2 && !(big_ok(a) && a.Nout >= 256)) || (c == 3 && !big_ok(a)) || (c == 4 && a.Nout <= 64) ||
        (c == 5 && (DGRAD || a.Cs < 64)) || (c == 14 && (DGRAD || !wino_ok(a))))
      continue;
    launch_choice<DGRAD, STATS>(c, a, st);  // warm (code object load, caches)
    float t = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(e0, st);
      launch_choice<DGRAD, STATS>(c, a, st);
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
    if (alln < 200) alln += snprintf(all + alln, sizeof(all) - alln, " %d:%.1f", c, t * 1e3f);
  }
  const char* lg = getenv("PMD_CONV_AUTOTUNE_LOG");
  if (lg && (lg[0] == '1' || lg[0] == '2'))
    fprintf(stderr, "[pmd autotune] %s N=%d H=%d W=%d C=%d -> %dx%d K=%d R=%d s=%d: choice %d (%.1f us)%s%s\n",
            DGRAD ? "dgrad" : "fwd", a.N, a.H, a.W, a.Cs, a.OH, a.OW, a.Nout, a.R, a.stride, best,
            best_ms * 1e3f, lg[0] == '2' ? " | us per candidate:" : "", lg[0] == '2' ? all : "");
  return best;
}

template <bool DGRAD, bool STATS>
static void launch_sel(const ConvArgs& a, hipStream_t st) {
  if (conv_impl() == 5 && conv_tile() == 0 && autotune_on()) {
    const TuneKey k{{a.N, a.H, a.W, a.Cs, a.OH, a.OW, a.Nout, a.R, a.S, a.stride, a.pad, (int)DGRAD,
                     (int)STATS}};
    int c = -1;
    {
      std::lock_guard<std::mutex> lk(g_tune_mu);
      auto it = g_tune.find(k);
      if (it != g_tune.end()) c = it->second;
    }
    if (c < 0) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(st, &cs);
      if (cs == hipStreamCaptureStatusNone) {
        c = tune<DGRAD, STATS>(a, st);
        if (c >= 0) {
          std::lock_guard<std::mutex> lk(g_tune_mu);
          g_tune[k] = c;
        }
      }
    }
    if (c >= 0) {
      launch_choice<DGRAD, STATS>(c, a, st);
      return;
    }
  }
  const int t = conv_tile();
  if (t == 14 && !DGRAD) {
    launch_choice<DGRAD, STATS>(14, a, st);   // fused Winograd wherever eligible (forced policy)
  } else if ((t == 11 || t == 12) && halo_ok(a)) {
    launch_choice<DGRAD, STATS>(t, a, st);
  } else if (t == 10 && a.Nout > 64) {
    launch_choice<DGRAD, STATS>(10, a, st);
  } else if (t >= 6 && t <= 9 && p8_ok(t - 6, a)) {
    launch_p8<DGRAD, STATS>(a, st, t - 6);
  } else if ((t == 4 || t == 5) && a.Cs >= 64) {
    launch_w8<DGRAD, STATS>(a, st, t - 4);
  } else if (big_ok(a) && t == 3 && a.Nout >= 256) {
    launch_big<256, 256, 2, 4, DGRAD, STATS>(a, st);
  } else if (big_ok(a) && t == 2) {
    launch_big<256, 128, 4, 2, DGRAD, STATS>(a, st);
  } else if (a.Nout <= 64) {
    launch_t<128, 64, DGRAD, STATS>(a, st, conv_impl());
  } else {
    launch_t<128, 128, DGRAD, STATS>(a, st, conv_impl());
  }
}

// per-channel fp32 bias added with the addend by the NEXT dgrad launch on this thread
// (conv_dgrad in bind.cpp sets it around one launch; the linear-BN backward's constant term)
static thread_local const float* g_addend_bias = nullptr;
void conv_set_addend_bias(const float* b) { g_addend_bias = b; }

// deterministic mode: an upper bound of the launch's row-tile count over every tile choice
// (BM >= 64; stride-2 dgrads run 4 phase grids of Mgrid rows; HALO tiles never straddle images)
static int det_slot_bound(const ConvArgs& a) {
  const bool ph2 = a.stride == 2;
  const long long Mgrid = ph2 ? (long long)a.N * ((a.OH + 1) >> 1) * ((a.OW + 1) >> 1) : a.M;
  return (int)((ph2 ? 4 : 1) * ((Mgrid + 63) / 64) + a.N);
}

static int conv_igemm_launch_b(const bf16_t* src, const bf16_t* wt, bf16_t* out, float* stats, int N, int H,
                               int W, int Cs, int OH, int OW, int Nout, int R, int S, int stride, int pad,
                               bool dgrad, const bf16_t* addend, const uint8_t* addend_mask,
                               const BnReduceArgs* bnr, hipStream_t st, const float* shift, int batch,
                               long long bs_src, long long bs_wt, long long bs_out) {
  if (Cs % 8 != 0 || (Cs & (Cs - 1)) != 0) return 1;  // power-of-two channels (>= 8)
  if (Nout % 8 != 0) return 2;
  if (stride != 1 && stride != 2) return 3;
  if (batch < 1 || batch > 65535 || (batch > 1 && (dgrad || stats || addend || bnr))) return 6;
  ConvArgs a{};
  if (!out && !stats) return 9;   // no store only for a statistics-only pass
  a.batch = batch;
  a.bs_src = bs_src;
  a.bs_wt = bs_wt;
  a.bs_out = bs_out;
  a.src = src;
  a.wt = wt;
  a.out = out;
  a.stats = stats;
  a.shift = stats ? shift : nullptr;
  a.addend = addend;
  a.addend_mask = addend ? addend_mask : nullptr;
  a.addend_bias = (dgrad && addend) ? g_addend_bias : nullptr;
  a.bn_mask = nullptr;
  for (int t = 0; t < 2; ++t) {
    a.bn_y[t] = nullptr;
    a.bn_p[t] = nullptr;
    a.bn_red[t] = nullptr;
  }
  if (bnr) {
    // y[t] may be null: a sum-only reduce (row 1 gets -mean * invstd * sum dz; the linear-BN
    // backward adds the y-dependent part from the weight gradient, ops/functional.py)
    if (!dgrad || !bnr->p[0] || !bnr->red[0]) return 5;
    a.bn_mask = bnr->mask;
    for (int t = 0; t < 2; ++t) {
      a.bn_y[t] = bnr->y[t];
      a.bn_p[t] = bnr->p[t];
      a.bn_red[t] = bnr->red[t];
    }
  }
  a.N = N;
  a.H = H;
  a.W = W;
  a.Cs = Cs;
  a.log2Cs = ilog2(Cs);
  a.OH = OH;
  a.OW = OW;
  a.Nout = Nout;
  a.R = R;
  a.S = S;
  a.stride = stride;
  a.log2stride = ilog2(stride);
  a.pad = pad;
  const long long M = (long long)N * OH * OW;
  if (M >= (1ll << 31) || (long long)N * H * W >= (1ll << 31)) return 4;
  a.M = (int)M;
  a.Kg = R * S * Cs;
  a.f8_sa = nullptr;
  a.f8_sb = nullptr;
  DetStats det;
  if (stats && a.bn_red[0] && det_stats_on()) return 10;  // one slot count per launch
  if (stats || a.bn_red[0]) {
    a.nslots = det_begin(det, stats ? &a.stats : &a.bn_red[0], stats ? nullptr : &a.bn_red[1],
                         det_slot_bound(a), 2 * Nout, st);
    if (a.nslots < 1) return 10;
  }
  if (dgrad) {
    if (stats) launch_sel<true, true>(a, st);
    else launch_sel<true, false>(a, st);
  } else {
    if (stats) launch_sel<false, true>(a, st);
    else launch_sel<false, false>(a, st);
  }
  det_end(det, st);
  return 0;
}

// ---- FP8 dgrad (config 5): e5m2 dY x e4m3 [Cp][R][S][K] weight image, the bf16 kernel's
// dgrad epilogue (addend + mask, fused BN-backward reduce), fixed tile policy (no tuner):
// 128x64 for 64-channel outputs, 128x128 otherwise, a single LDS stage when the whole
// reduction is <= 4 K-tiles (the epilogue-bound short-reduction dgrads keep 4 blocks / CU)
template <int BM, int BN, bool ONE>
static void launch_f8(const ConvArgs& a, hipStream_t st) {
  const bool ph2 = a.stride == 2;
  const int Mgrid = ph2 ? a.N * ((a.OH + 1) >> 1) * ((a.OW + 1) >> 1) : a.M;
  const int tiles = ((Mgrid + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
  const dim3 grid(tiles, ph2 ? 4 : 1, 1), block(256);
  const int nb = a.bn_red[0] ? (a.bn_red[1] ? 2 : 1) : 0;
#define F8K(NBV) \
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 64, 2, true, false, true, false, 2, 2, false, false, NBV, true, \
                                        ONE ? 1 : 0>), grid, block, 0, st, a)
  if (nb == 2) F8K(2);
  else if (nb == 1) F8K(1);
  else F8K(0);
#undef F8K
}

// fp8 FORWARD on the same implicit-GEMM kernel (the e4m3 x e4m3 path of conv_igemm_kernel<...,
// F8>: swz_f8 LDS layout, XCD remap, the bf16 kernel's statistics epilogue) -- an alternative
// to conv_fp8_fwd_kernel (fp8.hip) selected by conv_fp8_fwd_set_impl / PMD_FP8_FWD_IMPL.
template <int BM, int BN, bool ONE, bool STATS>
static void launch_f8_fwd(const ConvArgs& a, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
  hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, 64, 2, false, STATS, true, false, 2, 2, false, false, 0, true,
                                        ONE ? 1 : 0>), dim3(tiles, 1, 1), dim3(256), 0, st, a);
}
int conv_fwd_fp8_igemm_launch(const uint8_t* xq, const uint8_t* wq, bf16_t* out, float* stats, const float* sx,
                              const float* sw, int N, int H, int W, int Cs, int OH, int OW, int Nout, int R, int S,
                              int stride, int pad, hipStream_t st, const float* shift) {
  if (Cs % 16 != 0 || (Cs & (Cs - 1)) != 0) return 1;  // a 16-B chunk = 16 channels of one tap
  if (Nout % 8 != 0) return 2;
  if (stride != 1 && stride != 2) return 3;
  ConvArgs a{};
  a.batch = 1;
  a.src = reinterpret_cast<const bf16_t*>(xq);
  a.wt = reinterpret_cast<const bf16_t*>(wq);
  a.out = out;
  a.stats = stats;
  a.shift = stats ? shift : nullptr;
  a.N = N; a.H = H; a.W = W; a.Cs = Cs; a.log2Cs = ilog2(Cs);
  a.OH = OH; a.OW = OW; a.Nout = Nout; a.R = R; a.S = S;
  a.stride = stride; a.log2stride = ilog2(stride); a.pad = pad;
  const long long M = (long long)N * OH * OW;
  if (M >= (1ll << 31) || (long long)N * H * W >= (1ll << 31)) return 4;
  a.M = (int)M;
  a.Kg = R * S * Cs;
  a.f8_sa = sx;
  a.f8_sb = sw;
  const bool one = a.Kg <= 512;
  DetStats det;
  if (stats) {
    a.nslots = det_begin(det, &a.stats, nullptr, det_slot_bound(a), 2 * Nout, st);
    if (a.nslots < 1) return 10;
  }
#define F8F(BMV, BNV)                                              \
  do {                                                             \
    if (one) {                                                     \
      if (stats) launch_f8_fwd<BMV, BNV, true, true>(a, st);       \
      else launch_f8_fwd<BMV, BNV, true, false>(a, st);            \
    } else {                                                       \
      if (stats) launch_f8_fwd<BMV, BNV, false, true>(a, st);      \
      else launch_f8_fwd<BMV, BNV, false, false>(a, st);           \
    }                                                              \
  } while (0)
  if (a.Nout <= 64) F8F(128, 64);
  else F8F(128, 128);
#undef F8F
  det_end(det, st);
  return 0;
}

int conv_dgrad_fp8_launch(const uint8_t* dyq, const uint8_t* wtq, const float* sdy, const float* sw, bf16_t* out,
                          int N, int H, int W, int Cs, int OH, int OW, int Nout, int R, int S, int stride, int pad,
                          const bf16_t* addend, const uint8_t* addend_mask, const BnReduceArgs* bnr,
                          hipStream_t st) {
  // dgrad view: gathered operand dY [N, H, W, Cs] (H x W = the conv's output grid), output [N, OH, OW, Nout]
  if (Cs % 16 != 0 || (Cs & (Cs - 1)) != 0) return 1;  // a 16-B chunk = 16 channels of one tap
  if (Nout % 8 != 0) return 2;
  if (stride != 1 && stride != 2) return 3;
  ConvArgs a{};
  a.batch = 1;
  a.src = reinterpret_cast<const bf16_t*>(dyq);
  a.wt = reinterpret_cast<const bf16_t*>(wtq);
  a.out = out;
  a.addend = addend;
  a.addend_mask = addend ? addend_mask : nullptr;
  if (bnr) {
    if (!bnr->y[0] || !bnr->p[0] || !bnr->red[0]) return 5;
    a.bn_mask = bnr->mask;
    for (int t = 0; t < 2; ++t) {
      a.bn_y[t] = bnr->y[t];
      a.bn_p[t] = bnr->p[t];
      a.bn_red[t] = bnr->red[t];
    }
  }
  a.N = N; a.H = H; a.W = W; a.Cs = Cs; a.log2Cs = ilog2(Cs);
  a.OH = OH; a.OW = OW; a.Nout = Nout; a.R = R; a.S = S;
  a.stride = stride; a.log2stride = ilog2(stride); a.pad = pad;
  const long long M = (long long)N * OH * OW;
  if (M >= (1ll << 31) || (long long)N * H * W >= (1ll << 31)) return 4;
  a.M = (int)M;
  a.Kg = R * S * Cs;
  a.f8_sa = sdy;
  a.f8_sb = sw;
  const bool one = a.Kg <= 512;  // <= 4 K-tiles: the short-reduction, epilogue-bound dgrads
  DetStats det;
  if (a.bn_red[0]) {
    a.nslots = det_begin(det, &a.bn_red[0], &a.bn_red[1], det_slot_bound(a), 2 * Nout, st);
    if (a.nslots < 1) return 10;
  }
  if (a.Nout <= 64) {
    if (one) launch_f8<128, 64, true>(a, st);
    else launch_f8<128, 64, false>(a, st);
  } else {
    if (one) launch_f8<128, 128, true>(a, st);
    else launch_f8<128, 128, false>(a, st);
  }
  det_end(det, st);
  return 0;
}

// Returns 0 on success, nonzero on unsupported shape.
int conv_igemm_launch(const bf16_t* src, const bf16_t* wt, bf16_t* out, float* stats, int N, int H,
                      int W, int Cs, int OH, int OW, int Nout, int R, int S, int stride, int pad,
                      bool dgrad, const bf16_t* addend, const uint8_t* addend_mask,
                      const BnReduceArgs* bnr, hipStream_t st, const float* shift) {
  return conv_igemm_launch_b(src, wt, out, stats, N, H, W, Cs, OH, OW, Nout, R, S, stride, pad, dgrad, addend,
                             addend_mask, bnr, st, shift, 1, 0, 0, 0);
}

// `batch` independent forward convolutions of one shape in ONE launch (grid.z), no
// epilogue fusions: problem z = (src + z bs_src, wt + z bs_wt) -> out + z bs_out.
int conv_igemm_batched_launch(const bf16_t* src, const bf16_t* wt, bf16_t* out, int batch, long long bs_src,
                              long long bs_wt, long long bs_out, int N, int H, int W, int Cs, int OH, int OW,
                              int Nout, int R, int S, int stride, int pad, hipStream_t st) {
  return conv_igemm_launch_b(src, wt, out, nullptr, N, H, W, Cs, OH, OW, Nout, R, S, stride, pad, false, nullptr,
                             nullptr, nullptr, st, nullptr, batch, bs_src, bs_wt, bs_out);
}

void conv_weight_prep_launch(const float* w, bf16_t* wk, bf16_t* wkt, int K, int RS, int C, int Cp,
                             hipStream_t st) {
  const int total = K * RS * Cp;
  const int blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
  hipLaunchKernelGGL(conv_weight_prep_kernel, dim3(blocks), dim3(256), 0, st, w, wk, wkt, K, RS, C,
                     Cp);
}

}  // namespace pmd
