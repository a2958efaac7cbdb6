// Pooling, softmax cross-entropy, accuracy and fused SGD kernels (gfx950).
//
//   maxpool3x3s2 fwd/bwd  ImageNet stem (new capability; torch max_pool2d(3,2,1))
//   global avgpool fwd/bwd  reference F.avg_pool2d(out, 4) on 4x4 maps (resnet.py:102)
//                           and the ImageNet 7x7 global pool
//   xent fwd/bwd          nn.CrossEntropyLoss (mean), reference main.py:48,105
//   correct_count         top-1 argmax==target count kept on device
//                         (main.py:150-151 without the per-step host sync)
//   sgd                   torch.optim.SGD(momentum, nesterov, weight_decay) over
//                         flat fp32 arenas in ONE launch (main.py:51-55,110)
#include "common.h"

namespace pmd {

// ---------------------------------------------------------------- maxpool
// x [N,H,W,C] -> out [N,P,Q,C], arg [N,P,Q,C] (uint8 tap index 0..8).
// grid.y = output row (n, p), x covers Q * C/8 chunks: 32-bit index math only
// (C/8 a power of two -> shift/mask), no 64-bit divisions per element.
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ out,
                                                          uint8_t* __restrict__ arg, int N, int H,
                                                          int W, int C, int P, int Q, int log2C8) {
  const int C8 = C >> 3;
  const int row = blockIdx.y;  // n * P + p
  const int n = row / P, p = row - (row / P) * P;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Q * C8) return;
  const int q = j >> log2C8, cc = j & (C8 - 1);
  float best[8];
  int bi[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    best[k] = -INFINITY;
    bi[k] = 0;
  }
  const bf16_t* xb = x + (size_t)n * H * W * C + cc * 8;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int ih = p * 2 - 1 + t / 3, iw = q * 2 - 1 + t % 3;
    if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) continue;
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xb + ((size_t)ih * W + iw) * C), v);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (v[k] > best[k] || (v[k] != v[k] && best[k] == best[k])) {
        best[k] = v[k];
        bi[k] = t;
      }
  }
  const size_t o = (size_t)row * Q * C8 + j;
  reinterpret_cast<uint4*>(out)[o] = pack8(best);
  uint2 packed;
  packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
  packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
  reinterpret_cast<uint2*>(arg)[o] = packed;
}

// gather form: every input chunk sums the dout of the (<= 4) windows whose argmax is it.
// grid.y = input row (n, h), x covers W * C/8 chunks.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dout,
                                                          const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, int N, int H, int W,
                                                          int C, int P, int Q, int log2C8) {
  const int C8 = C >> 3;
  const int row = blockIdx.y;  // n * H + h
  const int n = row / H, h = row - (row / H) * H;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= W * C8) return;
  const int w = j >> log2C8, cc = j & (C8 - 1);
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const int p_lo = h > 0 ? h >> 1 : 0;             // windows p with 2p-1 <= h <= 2p+1
  const int p_hi = min((h + 1) >> 1, P - 1);
  const int q_lo = w > 0 ? w >> 1 : 0;
  const int q_hi = min((w + 1) >> 1, Q - 1);
  for (int p = p_lo; p <= p_hi; ++p)
    for (int q = q_lo; q <= q_hi; ++q) {
      const int dh = h - (p * 2 - 1), dw = w - (q * 2 - 1);
      if (dh < 0 || dh > 2 || dw < 0 || dw > 2) continue;
      const int tap = dh * 3 + dw;
      const size_t o = (((size_t)n * P + p) * Q + q) * C8 + cc;
      const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
      float g[8];
      unpack8(reinterpret_cast<const uint4*>(dout)[o], g);
      const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if ((int)((aw[k >> 2] >> ((k & 3) * 8)) & 0xff) == tap) acc[k] += g[k];
    }
  reinterpret_cast<uint4*>(dx)[(size_t)row * W * C8 + j] = pack8(acc);
}

// ---------------------------------------------------------------- avgpool
__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, float* __restrict__ out, int N,
                                   int HW, int C) {
  const int C8 = C >> 3;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C8) return;
  const int n = i / C8, cc = i % C8;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const bf16_t* base = x + (size_t)n * HW * C + cc * 8;
  for (int p = 0; p < HW; ++p) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(base + (size_t)p * C), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += v[k];
  }
  const float s = 1.f / HW;
  float4* o = reinterpret_cast<float4*>(out + (size_t)n * C + cc * 8);
  o[0] = make_float4(acc[0] * s, acc[1] * s, acc[2] * s, acc[3] * s);
  o[1] = make_float4(acc[4] * s, acc[5] * s, acc[6] * s, acc[7] * s);
}

__global__ void avgpool_bwd_kernel(const float* __restrict__ dout, bf16_t* __restrict__ dx, int N,
                                   int HW, int C) {
  const int C8 = C >> 3;
  const long long total = (long long)N * HW * C8;
  const float s = 1.f / HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % C8);
    const long long n = i / C8 / HW;
    const float4* g = reinterpret_cast<const float4*>(dout + n * C + cc * 8);
    const float4 a = g[0], b = g[1];
    float v[8] = {a.x * s, a.y * s, a.z * s, a.w * s, b.x * s, b.y * s, b.z * s, b.w * s};
    reinterpret_cast<uint4*>(dx)[i] = pack8(v);
  }
}

// ------------------------------------------------------------------- xent
// one block (256 threads) per row: loss += (lse - x[t]) / N ; lse[row]; correct += argmax==t
__global__ __launch_bounds__(256) void xent_fwd_kernel(const float* __restrict__ logits,
                                                       const long long* __restrict__ target,
                                                       float* __restrict__ loss,
                                                       float* __restrict__ lse_out,
                                                       long long* __restrict__ correct, int N,
                                                       int V, int nslots) {
  __shared__ float smax[4];
  __shared__ int sidx[4];
  __shared__ float ssum[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* x = logits + (size_t)row * V;
  float m = -INFINITY;
  int mi = 0x7fffffff;
  for (int j = tid; j < V; j += 256) {
    const float v = x[j];
    if (v > m) {
      m = v;
      mi = j;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) {
      m = om;
      mi = oi;
    }
  }
  if (lane == 0) {
    smax[wid] = m;
    sidx[wid] = mi;
  }
  __syncthreads();
  m = smax[0];
  mi = sidx[0];
  for (int w = 1; w < 4; ++w)
    if (smax[w] > m || (smax[w] == m && sidx[w] < mi)) {
      m = smax[w];
      mi = sidx[w];
    }
  float s = 0.f;
  for (int j = tid; j < V; j += 256) s += __expf(x[j] - m);
  s = wave_sum(s);
  if (lane == 0) ssum[wid] = s;
  __syncthreads();
  if (tid == 0) {
    const float tot = ssum[0] + ssum[1] + ssum[2] + ssum[3];
    const float lse = m + __logf(tot);
    const long long t = target[row];
    lse_out[row] = lse;
    atomicAdd(loss + row % nslots, (lse - x[t]) / N);  // nslots: 1 (deterministic mode: N)
    if (correct && mi == (int)t) atomicAdd((unsigned long long*)correct, 1ull);
  }
}

__global__ void xent_bwd_kernel(const float* __restrict__ logits, const long long* __restrict__ target,
                                const float* __restrict__ lse, const float* __restrict__ gloss,
                                float* __restrict__ grad, int N, int V) {
  const long long total = (long long)N * V;
  const float g = gloss[0] / N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int row = (int)(i / V), j = (int)(i % V);
    float p = __expf(logits[i] - lse[row]);
    if (j == (int)target[row]) p -= 1.f;
    grad[i] = p * g;
  }
}

// --------------------------------------------------------------------- sgd
// torch.optim.SGD: g += wd*p; buf = first ? g : m*buf + (1-damp)*g; g = nesterov ? g + m*buf : buf;
// p -= lr*g.  One launch over the whole flat arena (vectorised float4 + scalar tail).
// lr_dev (optional): learning rate read from device memory, so a captured HIP
// graph of the training step picks up scheduler changes without re-capture.
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                           long long n, float lr_host, const float* __restrict__ lr_dev,
                           float momentum, float wd, float damp, int nesterov, int first) {
  const float lr = lr_dev ? lr_dev[0] : lr_host;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4 + 4; i += stride) {
    float4 pv, gv, bv;
    const bool vec = i < n4;
    if (!vec) {
      const long long j = n4 * 4 + (i - n4);
      if (j >= n) continue;
      float pp = p[j], gg = g[j] + wd * pp, bb;
      if (momentum != 0.f) {
        bb = first ? gg : momentum * buf[j] + (1.f - damp) * gg;
        buf[j] = bb;
        gg = nesterov ? gg + momentum * bb : bb;
      }
      p[j] = pp - lr * gg;
      continue;
    }
    pv = reinterpret_cast<float4*>(p)[i];
    gv = reinterpret_cast<const float4*>(g)[i];
    float pa[4] = {pv.x, pv.y, pv.z, pv.w}, ga[4] = {gv.x, gv.y, gv.z, gv.w}, ba[4];
    if (momentum != 0.f) {
      bv = first ? make_float4(0, 0, 0, 0) : reinterpret_cast<float4*>(buf)[i];
      ba[0] = bv.x; ba[1] = bv.y; ba[2] = bv.z; ba[3] = bv.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = ga[k] + wd * pa[k];
      if (momentum != 0.f) {
        const float bb = first ? gg : momentum * ba[k] + (1.f - damp) * gg;
        ba[k] = bb;
        gg = nesterov ? gg + momentum * bb : bb;
      }
      pa[k] -= lr * gg;
    }
    reinterpret_cast<float4*>(p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    if (momentum != 0.f) reinterpret_cast<float4*>(buf)[i] = make_float4(ba[0], ba[1], ba[2], ba[3]);
  }
}

static int grid_for(long long work, int cap = 4096) {
  long long b = (work + 255) / 256;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

static int log2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}
int maxpool_fwd_launch(const bf16_t* x, bf16_t* out, uint8_t* arg, int N, int H, int W, int C, int P,
                       int Q, hipStream_t st) {
  const int l = log2_exact(C / 8);
  if (C % 8 || l < 0 || N * P > 65535) return 1;
  const dim3 grid((Q * (C / 8) + 255) / 256, N * P);
  hipLaunchKernelGGL(maxpool_fwd_kernel, grid, dim3(256), 0, st, x, out, arg, N, H, W, C, P, Q, l);
  return 0;
}
int maxpool_bwd_launch(const bf16_t* dout, const uint8_t* arg, bf16_t* dx, int N, int H, int W, int C,
                       int P, int Q, hipStream_t st) {
  const int l = log2_exact(C / 8);
  if (C % 8 || l < 0 || N * H > 65535) return 1;
  const dim3 grid((W * (C / 8) + 255) / 256, N * H);
  hipLaunchKernelGGL(maxpool_bwd_kernel, grid, dim3(256), 0, st, dout, arg, dx, N, H, W, C, P, Q, l);
  return 0;
}
int avgpool_fwd_launch(const bf16_t* x, float* out, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return 1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * (C / 8) + 255) / 256), dim3(256), 0, st, x, out, N,
                     HW, C);
  return 0;
}
int avgpool_bwd_launch(const float* dout, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return 1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long long)N * HW * (C / 8))), dim3(256), 0, st,
                     dout, dx, N, HW, C);
  return 0;
}
int xent_fwd_launch(const float* logits, const long long* target, float* loss, float* lse,
                    long long* correct, int N, int V, hipStream_t st) {
  DetStats det;  // deterministic mode: one slot per row, summed in row order
  int ns = det_begin(det, &loss, nullptr, N, 1, st);
  if (ns < 1) return 1;
  if (!det.n) ns = 1;
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(N), dim3(256), 0, st, logits, target, loss, lse, correct, N,
                     V, ns);
  det_end(det, st);
  return 0;
}
int xent_bwd_launch(const float* logits, const long long* target, const float* lse, const float* gloss,
                    float* grad, int N, int V, hipStream_t st) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(grid_for((long long)N * V)), dim3(256), 0, st, logits,
                     target, lse, gloss, grad, N, V);
  return 0;
}
// memset(0) as a framework kernel (gradient-arena zeroing, fresh accumulators): 16-B
// stores for the aligned bulk, bytes for the head/tail
__global__ __launch_bounds__(256) void zero_kernel(unsigned char* __restrict__ p, long long head,
                                                   long long n16, long long tail_off, long long tail) {
  const long long t0 = blockIdx.x * 256ll + threadIdx.x, stride = (long long)gridDim.x * 256;
  uint4* q = reinterpret_cast<uint4*>(p + head);
  for (long long i = t0; i < n16; i += stride) q[i] = make_uint4(0, 0, 0, 0);
  if (t0 < head) p[t0] = 0;
  if (t0 < tail) p[tail_off + t0] = 0;
}

int zero_launch(void* ptr, long long nbytes, hipStream_t st) {
  if (nbytes <= 0) return 0;
  unsigned char* p = static_cast<unsigned char*>(ptr);
  long long head = (16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15;
  if (head > nbytes) head = nbytes;
  const long long n16 = (nbytes - head) / 16;
  const long long tail_off = head + n16 * 16, tail = nbytes - tail_off;
  long long b = (n16 + 255) / 256;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  hipLaunchKernelGGL(zero_kernel, dim3((int)b), dim3(256), 0, st, p, head, n16, tail_off, tail);
  return 0;
}

int sgd_launch(float* p, const float* g, float* buf, long long n, float lr, const float* lr_dev,
               float momentum, float wd, float damp, bool nesterov, bool first, hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4 + 4, 8192)), dim3(256), 0, st, p, g, buf, n, lr,
                     lr_dev,
                     momentum, wd, damp, nesterov ? 1 : 0, first ? 1 : 0);
  return 0;
}

}  // namespace pmd
