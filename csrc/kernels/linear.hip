// Classifier GEMMs on gfx950 MFMA (K13, reference model/resnet.py:86,104 -- the
// nn.Linear(512 * expansion, num_classes) head and its two backward GEMMs).
//
// One strided kernel covers all three products of the fp32 [N,K] x [V,K]
// classifier (x = pooled features, W = weight):
//   forward  out[N][V]  = x . W^T (+ bias)          A = x      , B(r,j) = W[j][r]
//   dgrad    dx[N][K]   = dout . W                  A = dout   , B(r,j) = W[r][j]
//   wgrad    dW[V][K]  += dout^T . x                A(i,r) = dout[r][i], B = x
// C[i][j] = sum_r A(i,r) B(r,j) with A(i,r) = A[i*sai + r*sar], B(r,j) = B[r*sbr + j*sbj].
// Operands are fp32 in memory, rounded to bf16 while being staged through LDS
// (the network's compute dtype) and multiplied on v_mfma_f32_16x16x32_bf16 with
// fp32 accumulation.  Each operand's loader walks its unit-stride dimension with
// consecutive threads, so every layout above reads coalesced.  Tile 64x64x32,
// 256 threads = 2x2 waves of 32x32; the reduction is split over grid.z so these
// small-M products (M = the batch) still put ~1024 blocks on the chip.  The
// splits are combined DETERMINISTICALLY: each writes its fp32 partial tile to a
// workspace slab and one combine pass adds the slabs in split order (plus the
// bias or the accumulation target), so logits, loss and dW are bitwise
// reproducible run to run (fp32 atomics would make them order-dependent).
// With a single split the MFMA kernel writes C itself.
// The bias gradient (column sums of dout) is a separate one-pass kernel.
#include "common.h"

namespace pmd {

struct LinArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;  // [Nc] written by the init pass (forward), nullable
  long long sai, sar, sbr, sbj;
  int M, Nc, R;       // C is M x Nc, reduction length R
  int accumulate;     // C += product (grad-arena target) instead of C = product
};

constexpr int LT = 64, LK = 32, LPAD = 8;  // LDS row: 32 bf16 + 8 pad = 80 B (16-B aligned)
constexpr int LE = (LT * LK) / 256;        // operand elements per thread per K-step

// One K-step of an operand tile T[row][k] = src(row0 + row, k0 + k) (zero outside),
// loaded to registers first (the next step's loads fly while this one computes).
// Unit stride along k: consecutive threads walk k; else they walk rows.
struct LinTile {
  const float* src;
  long long s_row, s_k;
  int row0, nrow;
  __device__ __forceinline__ void load(float (&r)[LE], int k0, int kend, int tid) const {
    const bool kfast = s_k == 1;
#pragma unroll
    for (int e = 0; e < LE; ++e) {
      const int idx = e * 256 + tid;
      const int row = kfast ? idx / LK : idx % LT;
      const int k = kfast ? idx % LK : idx / LT;
      const int gr = row0 + row, gk = k0 + k;
      r[e] = (gr < nrow && gk < kend) ? src[(long long)gr * s_row + (long long)gk * s_k] : 0.f;
    }
  }
  __device__ __forceinline__ void store(bf16_t (*T)[LK + LPAD], const float (&r)[LE], int tid) const {
    const bool kfast = s_k == 1;
#pragma unroll
    for (int e = 0; e < LE; ++e) {
      const int idx = e * 256 + tid;
      T[kfast ? idx / LK : idx % LT][kfast ? idx % LK : idx / LT] = f2bf(r[e]);
    }
  }
};

// grid.z splits the reduction: block z covers [z*rchunk, min(R, (z+1)*rchunk)).
// ws == nullptr (one split): C = [C +] bias? + product.  Else the partial product
// goes to slab z of ws ([splits][M][Nc]) and linear_combine_kernel finishes.
__global__ __launch_bounds__(256) void linear_mfma_kernel(LinArgs a, int rchunk, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) bf16_t As[LT][LK + LPAD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[LT][LK + LPAD];  // Bs[j][k] = B(k, j)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int i0 = blockIdx.y * LT, j0 = blockIdx.x * LT;
  const int rb = blockIdx.z * rchunk;
  const int re = min(a.R, rb + rchunk);
  const LinTile ta{a.A, a.sai, a.sar, i0, a.M};
  const LinTile tb{a.B, a.sbj, a.sbr, j0, a.Nc};
  f32x4 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[p][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ra[LE], rbv[LE];
  ta.load(ra, rb, re, tid);
  tb.load(rbv, rb, re, tid);
  for (int k0 = rb; k0 < re; k0 += LK) {
    ta.store(As, ra, tid);
    tb.store(Bs, rbv, tid);
    __syncthreads();
    if (k0 + LK < re) {
      ta.load(ra, k0 + LK, re, tid);
      tb.load(rbv, k0 + LK, re, tid);
    }
    bf16x8 af[2], bfg[2];
    const int kq = (lane >> 4) * 8;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      af[p] = *reinterpret_cast<const bf16x8*>(&As[wm * 32 + p * 16 + (lane & 15)][kq]);
#pragma unroll
    for (int q = 0; q < 2; ++q)
      bfg[q] = *reinterpret_cast<const bf16x8*>(&Bs[wn * 32 + q * 16 + (lane & 15)][kq]);
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        acc[p][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[p], bfg[q], acc[p][q], 0, 0, 0);
    __syncthreads();
  }
  // C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = i0 + wm * 32 + p * 16 + (lane >> 4) * 4 + e;
        const int j = j0 + wn * 32 + q * 16 + (lane & 15);
        if (i < a.M && j < a.Nc) {
          const long long o = (long long)i * a.Nc + j;
          if (ws) {
            ws[(long long)blockIdx.z * a.M * a.Nc + o] = acc[p][q][e];
          } else {
            const float base = a.accumulate ? a.C[o] : (a.bias ? a.bias[j] : 0.f);
            a.C[o] = base + acc[p][q][e];
          }
        }
      }
}

// C[t] = (accumulate ? C[t] : bias[t % Nc] or 0) + sum_z ws[z][t], z in order
__global__ __launch_bounds__(256) void linear_combine_kernel(float* __restrict__ C, const float* __restrict__ bias,
                                                             const float* __restrict__ ws, long long n, int Nc,
                                                             int splits, int accumulate) {
  for (long long t = blockIdx.x * 256ll + threadIdx.x; t < n; t += (long long)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[(long long)z * n + t];
    const float base = accumulate ? C[t] : (bias ? bias[t % Nc] : 0.f);
    C[t] = base + s;
  }
}

// db[j] (+)= sum_i g[i][j]: 64 columns x 4 row lanes per block, LDS combine
__global__ __launch_bounds__(256) void linear_colsum_kernel(const float* __restrict__ g, float* __restrict__ db,
                                                            int rows, int cols, int accumulate) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + c;
  float s = 0.f;
  if (j < cols)
    for (int i = rl; i < rows; i += 4) s += g[(long long)i * cols + j];
  part[rl][c] = s;
  __syncthreads();
  if (rl == 0 && j < cols) {
    s = ((part[0][c] + part[1][c]) + part[2][c]) + part[3][c];
    db[j] = accumulate ? db[j] + s : s;
  }
}

// split plan: the grid covers the chip (>= ~1024 blocks), 4+ K-steps per split
static void linear_plan(int M, int Nc, int R, int* splits_out, int* rchunk_out) {
  const int tiles = ((Nc + LT - 1) / LT) * ((M + LT - 1) / LT);
  int splits = (1024 + tiles - 1) / tiles;
  const int max_splits = (R + 4 * LK - 1) / (4 * LK);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rchunk = (R + splits - 1) / splits;
  rchunk = (rchunk + LK - 1) / LK * LK;
  *splits_out = (R + rchunk - 1) / rchunk;
  *rchunk_out = rchunk;
}

long long linear_workspace_floats(int M, int Nc, int R) {
  if (M <= 0 || Nc <= 0 || R <= 0) return 0;
  int splits, rchunk;
  linear_plan(M, Nc, R, &splits, &rchunk);
  return splits > 1 ? (long long)splits * M * Nc : 0;
}

int linear_mfma_launch(const float* A, const float* B, float* C, const float* bias, long long sai,
                       long long sar, long long sbr, long long sbj, int M, int Nc, int R, bool accumulate,
                       float* ws, hipStream_t st) {
  if (M <= 0 || Nc <= 0 || R <= 0) return 1;
  if (accumulate && bias) return 2;
  LinArgs a{A, B, C, bias, sai, sar, sbr, sbj, M, Nc, R, accumulate ? 1 : 0};
  int splits, rchunk;
  linear_plan(M, Nc, R, &splits, &rchunk);
  if (splits > 1 && !ws) return 3;
  const dim3 grid((Nc + LT - 1) / LT, (M + LT - 1) / LT, splits);
  hipLaunchKernelGGL(linear_mfma_kernel, grid, dim3(256), 0, st, a, rchunk, splits > 1 ? ws : nullptr);
  if (splits > 1) {
    const long long n = (long long)M * Nc;
    const long long nb = (n + 255) / 256;
    hipLaunchKernelGGL(linear_combine_kernel, dim3((int)(nb < 2048 ? nb : 2048)), dim3(256), 0, st, C, bias, ws,
                       n, Nc, splits, accumulate ? 1 : 0);
  }
  return 0;
}

int linear_colsum_launch(const float* g, float* db, int rows, int cols, bool accumulate, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return 1;
  hipLaunchKernelGGL(linear_colsum_kernel, dim3((cols + 63) / 64), dim3(256), 0, st, g, db, rows, cols,
                     accumulate ? 1 : 0);
  return 0;
}

}  // namespace pmd
