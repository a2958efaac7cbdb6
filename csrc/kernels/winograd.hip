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

}  // namespace pmd
