// Linear-BN backward helpers (ops/functional.py _bnlin_final): the final BatchNorm of a
// bottleneck block back-propagated THROUGH the 1x1 conv3 that produced its input,
//   y = z W^T   (W = the bf16 [K][Cp] forward weight image the conv used, z = the conv input),
// so dy is never materialised and the BN-backward elementwise pass disappears (the BN passes
// are a third of the step's bytes, profiles/bytes_budget_r05.txt).  With the per-channel
// affine dy = A dz + B y + Cc (A = gamma * invstd, B = -A * invstd * mean(dz xhat), Cc = ...):
//   dz_in = dz (diag(A) W) + z (W^T diag(B) W) + Cc W       bnlin_dimg_kernel (diag(A) W image,
//           forward-time), bnlin_coeff_kernel (G, bias): the plain dgrad of dz on the scaled
//           image, then the small z G GEMM with it as addend + the bias, with the next BN's
//           fused reduce in its epilogue
//   dW    = diag(A) T + diag(B) W (z^T z) + Cc (x) colsum(z),  T = dz^T z    bnlin_wgrad_kernel
// Reference: the BN backward of /root/reference/model/resnet.py:66-70 (bn3 + shortcut add +
// relu), delegated there to torch's batch_norm_backward_{reduce,elemt}.
#include "common.h"

namespace pmd {

// Coefficients from the global sums, then G = W^T diag(B) W and bias = Cc W.  Block c (one per
// column of W; every block recomputes B, Cc for all K into LDS, block 0 also writes abc [3][K]):
// wc[k] = B_k W[k][c] in LDS, then G[c][q] = sum_k wc[k] W[k][q] with the K loop split over
// S = 256 / C thread slices (C < 256) and 8 independent, coalesced row loads in flight per
// thread (no barrier inside the K loop; this runs on the critical path of the backward,
// where the one-slice loop was a chain of K / 4 dependent L2 round trips: 27 us per call),
// slices combined in LDS; wave 0 reduces bias[c].
constexpr int kLinMaxK = 2048;

__global__ __launch_bounds__(256) void bnlin_coeff_kernel(const float* __restrict__ red, const float* __restrict__ count,
                                                         float count_h, const float* __restrict__ gamma,
                                                         const float* __restrict__ params, const bf16_t* __restrict__ wk,
                                                         bf16_t* __restrict__ g, float* __restrict__ bias,
                                                         float* __restrict__ abc, int K, int C, int Cp) {
  extern __shared__ float lsm[];
  float* wc = lsm;          // [K]  B_k W[k][c]
  float* cc = lsm + K;      // [K]  Cc_k W[k][c]
  float* part = lsm + 2 * K;  // [256] slice partials
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const float inv_cnt = 1.f / (count ? count[0] : count_h);
  for (int k = tid; k < K; k += 256) {
    const float mean = params[k], inv = params[K + k];
    const float a = gamma[k] * inv;
    const float mdy = red[k] * inv_cnt, mdyx = red[K + k] * inv_cnt;
    const float bb = -a * inv * mdyx, c3 = a * (mean * inv * mdyx - mdy);
    const float w = bf2f(wk[(size_t)k * Cp + c]);
    wc[k] = bb * w;
    cc[k] = c3 * w;
    if (c == 0) {
      abc[k] = a;
      abc[K + k] = bb;
      abc[2 * K + k] = c3;
    }
  }
  __syncthreads();
  const int qn = C < 256 ? C : 256;               // threads per slice
  const int S = C < 256 ? 256 / C : 1;            // K slices
  const int q0 = tid % qn, sl = tid / qn;
  const bool active = sl < S;
  const int kb = (int)((long long)sl * K / S), ke = (int)((long long)(sl + 1) * K / S);
  for (int q = q0; q < C; q += qn) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (active) {
      int k = kb;
      for (; k + 8 <= ke; k += 8) {
        float w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = bf2f(wk[(size_t)(k + u) * Cp + q]);
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += wc[k + u] * w[u];
      }
      for (; k < ke; ++k) s[0] += wc[k] * bf2f(wk[(size_t)k * Cp + q]);
    }
    const float t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
    if (S == 1) {
      g[(size_t)c * C + q] = f2bf(t);
    } else {
      part[tid] = t;   // tid = sl * qn + q (C < 256: one q per thread)
    }
  }
  if (S > 1) {
    __syncthreads();
    if (tid < C) {
      float t = 0.f;
      for (int j = 0; j < S; ++j) t += part[j * qn + tid];
      g[(size_t)c * C + tid] = f2bf(t);
    }
  }
  if (tid < 64) {
    float sb = 0.f;
    for (int k = tid; k < K; k += 64) sb += cc[k];
    sb = wave_sum(sb);
    if (tid == 0) bias[c] = sb;
  }
}

int bnlin_coeff_launch(const float* red, const float* count, float count_h, const float* gamma, const float* params,
                       const bf16_t* wk, bf16_t* g, float* bias, float* abc, int K, int C, int Cp, hipStream_t st) {
  if (K < 1 || K > kLinMaxK || C < 1 || Cp < C) return 1;
  hipLaunchKernelGGL(bnlin_coeff_kernel, dim3(C), dim3(256), sizeof(float) * (2 * (size_t)K + 256), st, red, count, count_h,
                     gamma, params, wk, g, bias, abc, K, C, Cp);
  return 0;
}

// The A-scaled, transposed dgrad image wkt_a[c][k] = bf16(gamma_k invstd_k W[k][c]) ([C][1][1][K]):
// A depends on forward quantities only, so the forward prepares it on the side stream.  32x32
// tiles transposed through LDS (coalesced reads along c, writes along k).
__global__ __launch_bounds__(256) void bnlin_dimg_kernel(const float* __restrict__ gamma,
                                                        const float* __restrict__ params,
                                                        const bf16_t* __restrict__ wk, bf16_t* __restrict__ wkt_a,
                                                        int K, int C, int Cp) {
  __shared__ float t[32][33];
  const int tilesC = (C + 31) / 32;
  const int k0 = (blockIdx.x / tilesC) * 32, c0 = (blockIdx.x % tilesC) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int k = k0 + r, c = c0 + tx;
    t[r][tx] = (k < K && c < C) ? gamma[k] * params[K + k] * bf2f(wk[(size_t)k * Cp + c]) : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r, k = k0 + tx;
    if (c < C && k < K) wkt_a[(size_t)c * K + k] = f2bf(t[tx][r]);
  }
}

int bnlin_dimg_launch(const float* gamma, const float* params, const bf16_t* wk, bf16_t* wkt_a, int K, int C, int Cp,
                      hipStream_t st) {
  if (K < 1 || C < 1 || Cp < C) return 1;
  const int grid = ((K + 31) / 32) * ((C + 31) / 32);
  hipLaunchKernelGGL(bnlin_dimg_kernel, dim3(grid), dim3(256), 0, st, gamma, params, wk, wkt_a, K, C, Cp);
  return 0;
}

// fp32 column sums of an NHWC bf16 activation [M][C] (C % 8 == 0, C <= 2048) into out [C],
// which must be zeroed: per-thread 8-channel partials over a grid-stride row walk, combined
// per block in LDS, one atomic per channel per block
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                    long long M, int C) {
  __shared__ float part[2048];
  const int C8 = C >> 3;
  const int tid = threadIdx.x;
  for (int c = tid; c < C; c += 256) part[c] = 0.f;
  __syncthreads();
  // thread -> chunk column (tid % C8) when C8 divides 256, rows strided by 256 / C8 per block
  const int cols = C8 < 256 ? C8 : 256;
  const int rpb = 256 / cols;
  const int cc = tid % cols, rr = tid / cols;
  if (rr < rpb) {
    for (int c8 = cc; c8 < C8; c8 += cols) {
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (long long m = (long long)blockIdx.x * rpb + rr; m < M; m += (long long)gridDim.x * rpb) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + m * C + c8 * 8), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += f[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) atomicAdd(&part[c8 * 8 + e], s[e]);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) atomicAdd(out + c, part[c]);
}

int colsum_launch(const bf16_t* x, float* out, long long M, int C, hipStream_t st) {
  if (C % 8 || C > 2048 || M < 1) return 1;
  long long blocks = (M + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(colsum_kernel, dim3((int)blocks), dim3(256), 0, st, x, out, M, C);
  return 0;
}

// out[k][c] += A_k T[k][c] + B_k sum_c' W[k][c'] Gz[c'][c] + Cc_k colsum[c]
// (out = the fp32 [K][1][1][C] arena view of dW3): block = 8 rows k x all c; W rows staged in LDS
__global__ __launch_bounds__(256) void bnlin_wgrad_kernel(float* __restrict__ out, const float* __restrict__ abc,
                                                         const float* __restrict__ T, const bf16_t* __restrict__ wk,
                                                         const float* __restrict__ gz, const float* __restrict__ cs,
                                                         int K, int C, int Cp) {
  extern __shared__ float wrow[];   // [8][C]
  const int k0 = blockIdx.x * 8;
  const int tid = threadIdx.x;
  for (int i = tid; i < 8 * C; i += 256) {
    const int r = i / C, c = i % C;
    wrow[i] = k0 + r < K ? bf2f(wk[(size_t)(k0 + r) * Cp + c]) : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < 8 * C; i += 256) {
    const int r = i / C, c = i % C, k = k0 + r;
    if (k >= K) continue;
    float s = 0.f;
    for (int q = 0; q < C; ++q) s += wrow[r * C + q] * gz[(size_t)q * C + c];
    out[(size_t)k * C + c] += abc[k] * T[(size_t)k * C + c] + abc[K + k] * s + abc[2 * K + k] * cs[c];
  }
}

int bnlin_wgrad_launch(float* out, const float* abc, const float* T, const bf16_t* wk, const float* gz,
                       const float* cs, int K, int C, int Cp, hipStream_t st) {
  if (K < 1 || C < 1 || C > 2048 || Cp < C) return 1;
  hipLaunchKernelGGL(bnlin_wgrad_kernel, dim3((K + 7) / 8), dim3(256), sizeof(float) * 8 * C, st, out, abc, T, wk,
                     gz, cs, K, C, Cp);
  return 0;
}

}  // namespace pmd
