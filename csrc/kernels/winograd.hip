// Winograd F(2x2, 3x3) convolution for stride-1, pad-1, 3x3 layers (SURVEY
// §2.4.3 K4), NHWC bf16 in/out, fp32 transform arithmetic:
//
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A      per 2x2 output tile, per channel pair
//
//   B^T = | 1  0 -1  0 |   G = | 1    0    0  |   A^T = | 1  1  1  0 |
//         | 0  1  1  0 |       | 1/2  1/2  1/2|         | 0  1 -1 -1 |
//         | 0 -1  1  0 |       | 1/2 -1/2  1/2|
//         | 0  1  0 -1 |       | 0    0    1  |
//
// Three memory-bound transform kernels around 16 independent GEMMs
//   M[xi][t][k] = sum_c V[xi][t][c] * U[xi][k][c]     (xi = 4x4 transform position)
// which run as one grid.z-batched launch of the implicit-GEMM MFMA conv kernel
// (conv_igemm_batched_launch: each is a 1x1 conv of T tiles by the K x C slice).  The output
// transform fuses the BatchNorm statistics epilogue of conv_fwd (same [slot][2][K]
// contract), so the Winograd path is a drop-in forward for a BN-followed conv.
// Dgrad of the same layer is the forward of dY with the spatially flipped,
// channel-transposed filter (flip=true in the filter transform).
//
// On MI355X this path is NOT the default (see docs/ARCHITECTURE.md, "Winograd"):
// it trades 2.25x fewer multiplies for 16/(2x2)=4x larger transformed operands;
// with bf16 MFMA at ~2.5 PFLOP/s against ~8 TB/s HBM the implicit GEMM is already
// near the bandwidth roofline for these layers, so the transformed-tensor
// traffic costs more than the MFMA work saved.  Not on the training path (round 3):
// an explicit API (ops/winograd.py::conv_fwd / conv_dgrad); bench/winograd_bench.py
// measures it against the implicit GEMM.
#include "common.h"

#include <map>
#include <mutex>

namespace pmd {

// U[xi][k][c] (bf16) from the forward weight image wk[K][3][3][Cp].
// flip: build the dgrad filter instead, g'[c][r][s][k] = wk[k][2-r][2-s][c],
// i.e. U[xi][c][k] over an "output channel" axis of size Cp.
__global__ __launch_bounds__(256) void winograd_filter_kernel(const bf16_t* __restrict__ wk,
                                                              bf16_t* __restrict__ U, int K, int Cp,
                                                              int flip) {
  const int KO = flip ? Cp : K, CI = flip ? K : Cp;  // transformed filter is [16][KO][CI]
  const long long total = (long long)KO * CI;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % CI), ko = (int)(i / CI);
    float g[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        // fwd: g[r][s] = wk[ko][r][s][ci];  dgrad: g[r][s] = wk[ci][2-r][2-s][ko]
        const size_t idx = flip ? (((size_t)ci * 3 + (2 - r)) * 3 + (2 - s)) * Cp + ko
                                : (((size_t)ko * 3 + r) * 3 + s) * Cp + ci;
        g[r][s] = bf2f(wk[idx]);
      }
    float t[4][3];  // G g
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      t[0][s] = g[0][s];
      t[1][s] = 0.5f * (g[0][s] + g[1][s] + g[2][s]);
      t[2][s] = 0.5f * (g[0][s] - g[1][s] + g[2][s]);
      t[3][s] = g[2][s];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const float u[4] = {t[a][0], 0.5f * (t[a][0] + t[a][1] + t[a][2]),
                          0.5f * (t[a][0] - t[a][1] + t[a][2]), t[a][2]};
#pragma unroll
      for (int b = 0; b < 4; ++b) U[((size_t)(a * 4 + b) * KO + ko) * CI + ci] = f2bf(u[b]);
    }
  }
}

// V[xi][t][c] = (B^T d B)[xi] for every 2x2 output tile t = (n, th, tw) and 8-channel
// chunk; d is the 4x4 input patch at rows 2 th - 1 .. 2 th + 2 (zero outside).
__global__ __launch_bounds__(256) void winograd_input_kernel(const bf16_t* __restrict__ x,
                                                             bf16_t* __restrict__ V, int N, int H,
                                                             int W, int C, int TH, int TW) {
  const int C8 = C >> 3;
  const long long T = (long long)N * TH * TW;
  const long long total = T * C8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const long long t = i / C8;
    const int tw = (int)(t % TW), th = (int)((t / TW) % TH), n = (int)(t / ((long long)TW * TH));
    uint4 raw[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int h = 2 * th - 1 + a, w = 2 * tw - 1 + b;
        const bool ok = h >= 0 && h < H && w >= 0 && w < W;
        raw[a][b] = ok ? *reinterpret_cast<const uint4*>(x + (((size_t)n * H + h) * W + w) * C + c8 * 8)
                       : make_uint4(0, 0, 0, 0);
      }
    float d[4][4][8];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) unpack8(raw[a][b], d[a][b]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t4[4][4];  // B^T d
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        t4[0][b] = d[0][b][e] - d[2][b][e];
        t4[1][b] = d[1][b][e] + d[2][b][e];
        t4[2][b] = d[2][b][e] - d[1][b][e];
        t4[3][b] = d[1][b][e] - d[3][b][e];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {  // (B^T d) B, written back into d[a][*][e]
        d[a][0][e] = t4[a][0] - t4[a][2];
        d[a][1][e] = t4[a][1] + t4[a][2];
        d[a][2][e] = t4[a][2] - t4[a][1];
        d[a][3][e] = t4[a][1] - t4[a][3];
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        *reinterpret_cast<uint4*>(V + ((size_t)(a * 4 + b) * T + t) * C + c8 * 8) = pack8(d[a][b]);
  }
}

// y[n, 2th+i, 2tw+j, k] = (A^T M A)[i][j] from M[xi][t][K]; optional BN statistics
// (sum (v-K), sum (v-K)^2 of the bf16-rounded outputs v about the shift K, bn_moments)
// into stats[slot][2][K], slot = block % 64.
// Grid stride is a multiple of K/8, so each thread keeps ONE 8-channel chunk.
__global__ __launch_bounds__(256) void winograd_output_kernel(const bf16_t* __restrict__ M,
                                                              bf16_t* __restrict__ y,
                                                              float* __restrict__ stats,
                                                              const float* __restrict__ shift, int N,
                                                              int H, int W, int K, int TH, int TW,
                                                              int nslots) {
  const int K8 = K >> 3;
  const long long T = (long long)N * TH * TW;
  const long long total = T * K8;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  const long long start = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int k8 = (int)(start % K8);
  float sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sh[e] = (stats && shift) ? shift[k8 * 8 + e] : 0.f;
  for (long long i = start; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long t = i / K8;
    const int tw = (int)(t % TW), th = (int)((t / TW) % TH), n = (int)(t / ((long long)TW * TH));
    uint4 raw[16];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
      raw[xi] = *reinterpret_cast<const uint4*>(M + ((size_t)xi * T + t) * K + k8 * 8);
    float mm[16][8];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) unpack8(raw[xi], mm[xi]);
    float o[2][2][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float m[4][4];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) m[xi >> 2][xi & 3] = mm[xi][e];
      float t2[2][4];  // A^T M
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        t2[0][b] = m[0][b] + m[1][b] + m[2][b];
        t2[1][b] = m[1][b] - m[2][b] - m[3][b];
      }
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        o[a][0][e] = t2[a][0] + t2[a][1] + t2[a][2];
        o[a][1][e] = t2[a][1] - t2[a][2] - t2[a][3];
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * th + a, w = 2 * tw + b;
        if (h < H && w < W) {
          const uint4 pk = pack8(o[a][b]);
          *reinterpret_cast<uint4*>(y + (((size_t)n * H + h) * W + w) * K + k8 * 8) = pk;
          if (stats) {
            float r[8];
            unpack8(pk, r);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = r[e] - sh[e];
              s1[e] += d;
              s2[e] += d * d;
            }
          }
        }
      }
  }
  if (!stats) return;
  // block combine of the threads sharing a chunk (tid % K8), one atomic per channel
  __shared__ float part[256][17];
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    part[tid][e] = s1[e];
    part[tid][8 + e] = s2[e];
  }
  __syncthreads();
  // K8 divides 256, so thread r of every block holds chunk r % K8
  for (int q = tid; q < K8 * 16; q += 256) {
    const int col = q >> 4, j = q & 15;
    float acc = 0.f;
    for (int r = col; r < 256; r += K8) acc += part[r][j];
    atomicAdd(stats + (stat_slot(blockIdx.x, nslots) * 2 + (j >> 3)) * K + col * 8 + (j & 7), acc);
  }
}

static int ew_blocks(long long work) {
  long long b = (work + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

int winograd_filter_launch(const bf16_t* wk, bf16_t* U, int K, int Cp, bool flip, hipStream_t st) {
  if (K % 8 || Cp % 8) return 1;
  hipLaunchKernelGGL(winograd_filter_kernel, dim3(ew_blocks((long long)K * Cp)), dim3(256), 0, st, wk,
                     U, K, Cp, flip ? 1 : 0);
  return 0;
}

int winograd_input_launch(const bf16_t* x, bf16_t* V, int N, int H, int W, int C, hipStream_t st) {
  const int C8 = C >> 3;
  if (C % 8 || C8 > 256 || (C8 & (C8 - 1))) return 1;  // grid stride must stay chunk-aligned
  const int TH = (H + 1) / 2, TW = (W + 1) / 2;
  hipLaunchKernelGGL(winograd_input_kernel, dim3(ew_blocks((long long)N * TH * TW * C8)), dim3(256), 0,
                     st, x, V, N, H, W, C, TH, TW);
  return 0;
}

int winograd_output_launch(const bf16_t* M, bf16_t* y, float* stats, int N, int H, int W, int K,
                           hipStream_t st, const float* shift) {
  const int K8 = K >> 3;
  if (K % 8 || K8 > 256 || (K8 & (K8 - 1))) return 1;  // 256-thread blocks: stride % K8 == 0
  const int TH = (H + 1) / 2, TW = (W + 1) / 2;
  const int blocks = ew_blocks((long long)N * TH * TW * K8);
  DetStats det;
  const int ns = det_begin(det, &stats, nullptr, blocks, 2 * K, st);
  if (ns < 1) return 2;
  hipLaunchKernelGGL(winograd_output_kernel, dim3(blocks), dim3(256), 0, st, M, y, stats, shift, N, H, W, K,
                     TH, TW, ns);
  det_end(det, st);
  return 0;
}


// ---------------------------------------------------------------- fused forward
// F(2x2,3x3) forward as ONE kernel: the input transform, the 16
// transformed-domain GEMMs and the output transform (+ the BN-statistics epilogue) never
// leave the CU -- no V / M tensors in HBM.  Block: 256 threads (4 waves), 32 output tiles
// (2x2 pixels each, flattened (n, th, tw) order) x 64 output channels; K-steps of 64 input
// channels:
//   1. each thread gathers the 4x4 input patch of one tile for one 8-channel chunk (16 x 16 B
//      loads, issued one K-step ahead), forms V = B^T d B in fp32 and writes the 16 bf16
//      values into LDS V[xi][tile][c] (64 KB; 16-B chunk XOR-swizzled by the tile row, as the
//      implicit-GEMM kernel's BK=64 tiles, so the fragment reads are conflict-free);
//   2. wave w owns positions xi = 4w..4w+3: per xi, 2 x 4 16x16 accumulator tiles over the
//      32 x 64 block tile, 16 v_mfma_f32_16x16x32_bf16 per K-step with the A fragments from
//      LDS and the filter fragments U[xi][k][c] (winograd_filter_kernel, L2-resident) read
//      straight into registers, the next position's fragments in flight during the MFMAs;
//   3. the accumulators are exchanged through the same LDS as fp32 (two halves of 16 tiles,
//      channel index XOR-swizzled by the tile's lane group so the fragment-layout writes are
//      conflict-free); each thread then owns (tile, 4 channels), forms Y = A^T M A, rounds to
//      bf16, stores the 2x2 pixels and accumulates the BN statistics of the stored values.
// Contract: stride 1, pad 1, 3x3, C % 64 == 0, K % 64 == 0 (launcher).
constexpr int kWgT = 32;   // output tiles per block
constexpr int kWgBN = 64;  // output channels per block
constexpr int kWgBK = 64;  // input channels per K-step

template <bool STATS>
__global__ __launch_bounds__(256, 1) void winograd_fused_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ U, bf16_t* __restrict__ y,
    float* __restrict__ stats, const float* __restrict__ shift, int N, int H, int W, int C, int K,
    int TH, int TW, int nslots) {
  __shared__ __attribute__((aligned(16))) char smem[65536];
  bf16_t* Vs = reinterpret_cast<bf16_t*>(smem);
  float* Ms = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int T = N * TH * TW;
  const int ncol = K / kWgBN;
  const int nrow = (T + kWgT - 1) / kWgT;
  // the ncol column blocks of one row block are consecutive logical ids on one XCD (its L2
  // then serves their shared input patches)
  const int L = xcd_remap(blockIdx.x, nrow * ncol);
  const int rb = L / ncol, n0 = (L % ncol) * kWgBN;
  const int t0 = rb * kWgT;

  // ---- input-transform role: tile it, 8-channel chunk ic
  const int it = tid >> 3, ic = tid & 7;
  const int tg = t0 + it;
  unsigned vmask = 0;
  long long pbase = 0;
  if (tg < T) {
    const int pn = tg / (TH * TW), r = tg - pn * (TH * TW), ph = r / TW, pw = r - (r / TW) * TW;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int h = 2 * ph - 1 + a, w = 2 * pw - 1 + b;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) vmask |= 1u << (a * 4 + b);
      }
    pbase = (((long long)pn * H + (2 * ph - 1)) * W + (2 * pw - 1)) * C + ic * 8;
  }
  uint4 raw[16];
  auto load_patch = [&](int c0) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int q = a * 4 + b;
        raw[q] = ((vmask >> q) & 1u)
                     ? *reinterpret_cast<const uint4*>(x + pbase + ((long long)a * W + b) * C + c0)
                     : make_uint4(0, 0, 0, 0);
      }
  };
  // V = B^T d B per channel pair (32 fp32 temporaries), 16 dwords written per pair
  auto write_v = [&]() {
    const int wch = ((ic ^ (it & 7)) << 3);
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) {
      float d0[4][4], d1[4][4];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t w = pr == 0 ? raw[q].x : pr == 1 ? raw[q].y : pr == 2 ? raw[q].z : raw[q].w;
        d0[q >> 2][q & 3] = __uint_as_float(w << 16);
        d1[q >> 2][q & 3] = __uint_as_float(w & 0xffff0000u);
      }
      float v0[4][4], v1[4][4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {  // B^T d (rows)
        const float a0 = d0[0][b] - d0[2][b], a1 = d0[1][b] + d0[2][b], a2 = d0[2][b] - d0[1][b],
                    a3 = d0[1][b] - d0[3][b];
        v0[0][b] = a0; v0[1][b] = a1; v0[2][b] = a2; v0[3][b] = a3;
        const float c0 = d1[0][b] - d1[2][b], c1 = d1[1][b] + d1[2][b], c2 = d1[2][b] - d1[1][b],
                    c3 = d1[1][b] - d1[3][b];
        v1[0][b] = c0; v1[1][b] = c1; v1[2][b] = c2; v1[3][b] = c3;
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {  // (B^T d) B (columns)
        const float o0[4] = {v0[a][0] - v0[a][2], v0[a][1] + v0[a][2], v0[a][2] - v0[a][1], v0[a][1] - v0[a][3]};
        const float o1[4] = {v1[a][0] - v1[a][2], v1[a][1] + v1[a][2], v1[a][2] - v1[a][1], v1[a][1] - v1[a][3]};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t pk = (uint32_t)f2bf(o0[b]) | ((uint32_t)f2bf(o1[b]) << 16);
          *reinterpret_cast<uint32_t*>(Vs + ((a * 4 + b) * kWgT + it) * kWgBK + wch + 2 * pr) = pk;
        }
      }
    }
  };

  // ---- GEMM role: wave wid, positions xi = 4 wid + x4
  f32x4 acc[4][2][4];
#pragma unroll
  for (int x4 = 0; x4 < 4; ++x4)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[x4][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int frow = lane & 15, fq = lane >> 4;
  // U fragment (column n0 + j*16 + frow, reduction c0 + ks*32 + fq*8 .. +7) of position xi
  const bf16_t* ucol = U + (size_t)(n0 + frow) * C + fq * 8;
  auto load_u = [&](bf16x8 (&u)[2][4], int xi, int c0) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        u[ks][j] = *reinterpret_cast<const bf16x8*>(ucol + ((size_t)xi * K + j * 16) * C + c0 + ks * 32);
  };
  const int nks = C / kWgBK;
  load_patch(0);
  for (int ks0 = 0; ks0 < nks; ++ks0) {
    const int c0 = ks0 * kWgBK;
    bf16x8 ua[2][4], ub[2][4];
    load_u(ua, 4 * wid, c0);               // first position's filter fragments: fly during the transform
    __syncthreads();                       // every wave is done reading the previous V
    write_v();
    if (ks0 + 1 < nks) load_patch(c0 + kWgBK);   // next K-step's patch: flies during the MFMAs
    __syncthreads();                       // V published
#pragma unroll
    for (int x4 = 0; x4 < 4; ++x4) {
      const int xi = 4 * wid + x4;
      bf16x8 (&uc)[2][4] = (x4 & 1) ? ub : ua;
      bf16x8 (&un)[2][4] = (x4 & 1) ? ua : ub;
      if (x4 + 1 < 4) load_u(un, xi + 1, c0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = i * 16 + frow;
          const int q = ks * 4 + fq;
          af[i] = *reinterpret_cast<const bf16x8*>(Vs + (xi * kWgT + row) * kWgBK + ((q ^ (row & 7)) << 3));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[x4][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], uc[ks][j], acc[x4][i][j], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: M through LDS (fp32, [xi][16 tiles][64 ch], channel ^= (tile & 3) << 4), two halves
  const int et = tid >> 4, ec = (tid & 15) * 4;  // this thread's tile (within the half) and 4 channels
  float sh[4], s1[4], s2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sh[e] = (STATS && shift) ? shift[n0 + ec + e] : 0.f;
    s1[e] = s2[e] = 0.f;
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // V reads / the previous half's M reads are done
#pragma unroll
    for (int x4 = 0; x4 < 4; ++x4)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int tile = fq * 4 + e;             // within the half (row tile `half`)
          const int ch = (j * 16 + frow) ^ (fq << 4);   // the 4 lane groups on 4 disjoint bank ranges
          Ms[((4 * wid + x4) * 16 + tile) * kWgBN + ch] = acc[x4][half][j][e];
        }
    __syncthreads();
    const int tg2 = t0 + half * 16 + et;
    if (tg2 >= T) continue;
    float m[16][4];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
      const float4 v = *reinterpret_cast<const float4*>(Ms + (xi * 16 + et) * kWgBN + (ec ^ ((et >> 2) << 4)));
      m[xi][0] = v.x; m[xi][1] = v.y; m[xi][2] = v.z; m[xi][3] = v.w;
    }
    const int pn = tg2 / (TH * TW), r = tg2 - pn * (TH * TW), ph = r / TW, pw = r - (r / TW) * TW;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int h = 2 * ph + a, w = 2 * pw + b;
        if (h >= H || w >= W) continue;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // row a of A^T M (rows 0: m0 + m1 + m2, 1: m1 - m2 - m3), then column b likewise
          float t[4];
#pragma unroll
          for (int c = 0; c < 4; ++c)
            t[c] = a == 0 ? m[c][e] + m[4 + c][e] + m[8 + c][e] : m[4 + c][e] - m[8 + c][e] - m[12 + c][e];
          o[e] = b == 0 ? t[0] + t[1] + t[2] : t[1] - t[2] - t[3];
        }
        const uint32_t lo = (uint32_t)f2bf(o[0]) | ((uint32_t)f2bf(o[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(o[2]) | ((uint32_t)f2bf(o[3]) << 16);
        *reinterpret_cast<uint2*>(y + (((size_t)pn * H + h) * W + w) * K + n0 + ec) = make_uint2(lo, hi);
        if (STATS) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = round_bf(o[e]) - sh[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        }
      }
  }
  if (!STATS) return;
  // block combine over the 16 thread rows sharing a channel quad, one atomic per channel
  __syncthreads();
  float* part = Ms;  // [256][8]
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    part[tid * 8 + e] = s1[e];
    part[tid * 8 + 4 + e] = s2[e];
  }
  __syncthreads();
  if (tid < 2 * kWgBN) {
    const int which = tid / kWgBN, ch = tid % kWgBN;
    const int q = ch >> 2, e = ch & 3;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += part[(r * 16 + q) * 8 + which * 4 + e];
    atomicAdd(stats + (stat_slot(rb, nslots) * 2 + which) * K + n0 + ch, v);
  }
}

// U: the transformed filter [16][K][C] (winograd_filter_kernel, flip = false); the statistics slots
// are indexed modulo nslots (kStatSlots, or the deterministic mode's count: the caller's det_begin)
int winograd_fused_fwd_run(const bf16_t* x, const bf16_t* U, bf16_t* y, float* stats, const float* shift, int N,
                           int H, int W, int C, int K, int nslots, hipStream_t st) {
  if (C % kWgBK || K % kWgBN || nslots < 1) return 1;
  const int TH = (H + 1) / 2, TW = (W + 1) / 2;
  const long long T = (long long)N * TH * TW;
  if (T >= (1ll << 30)) return 2;
  const long long blocks = ((T + kWgT - 1) / kWgT) * (K / kWgBN);
  if (blocks >= (1ll << 31)) return 2;
  if (stats)
    hipLaunchKernelGGL(winograd_fused_fwd_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, x, U, y, stats,
                       shift, N, H, W, C, K, TH, TW, nslots);
  else
    hipLaunchKernelGGL(winograd_fused_fwd_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, x, U, y,
                       nullptr, nullptr, N, H, W, C, K, TH, TW, nslots);
  return 0;
}

int winograd_fused_fwd_launch(const bf16_t* x, const bf16_t* U, bf16_t* y, float* stats, const float* shift,
                              int N, int H, int W, int C, int K, hipStream_t st) {
  const int TH = (H + 1) / 2, TW = (W + 1) / 2;
  const long long nrow = ((long long)N * TH * TW + kWgT - 1) / kWgT;
  DetStats det;
  int ns = kStatSlots;
  if (stats) {
    ns = det_begin(det, &stats, nullptr, (int)(nrow < (1 << 30) ? nrow : 1), 2 * K, st);
    if (ns < 1) return 3;
  }
  const int rc = winograd_fused_fwd_run(x, U, y, stats, shift, N, H, W, C, K, ns, st);
  det_end(det, st);
  return rc;
}

// A whole forward from the conv's own weight image wk [K][3][3][C] (the implicit-GEMM kernel's
// B^T image): the filter transform into a per-stream U scratch (stream-ordered reuse; grown
// outside HIP-graph capture only), then the fused kernel.  The autotuner's candidate 14
// (kernels/conv_igemm.hip): timed, and adopted per shape, against the implicit GEMM.
int winograd_conv_fwd_run(const bf16_t* x, const bf16_t* wk, bf16_t* y, float* stats, const float* shift, int N,
                          int H, int W, int C, int K, int nslots, hipStream_t st) {
  static std::mutex mu;
  static std::map<hipStream_t, std::pair<bf16_t*, size_t>> scr;
  const size_t need = (size_t)16 * K * C;
  bf16_t* U = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto& e = scr[st];
    if (e.second < need) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      (void)hipStreamIsCapturing(st, &cs);
      if (cs != hipStreamCaptureStatusNone) return 4;
      // an outgrown buffer is never freed (in-flight launches / captured graphs may use it)
      bf16_t* p = nullptr;
      if (hipMalloc(&p, need * sizeof(bf16_t)) != hipSuccess) return 5;
      e = {p, need};
    }
    U = e.first;
  }
  const int rc = winograd_filter_launch(wk, U, K, C, false, st);
  if (rc) return rc;
  return winograd_fused_fwd_run(x, U, y, stats, shift, N, H, W, C, K, nslots, st);
}

}  // namespace pmd
