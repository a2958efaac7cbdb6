// On-device input pipeline kernels (gfx950).
//
//   synth_images   ImageNet-shaped synthetic batch, NHWC bf16 [N,H,W,Cp]
//                  (channels >= 3 zero padding for the MFMA stem) plus int64
//                  labels, from a counter-based hash: no host->device copy in
//                  the timed loop (BASELINE north star: synthetic data).
//   cifar_augment  the reference train transform (data.py:11-15):
//                  RandomCrop(32, padding=8) -> RandomHorizontalFlip ->
//                  ToTensor -> Normalize(0.5, 0.5), as a gather from a
//                  device-resident uint8 [Nd,32,32,3] dataset into NHWC
//                  bf16/fp32 [B,32,32,Cp].  Zero padding happens before
//                  normalisation, so padded pixels become -1 exactly as in
//                  torchvision.  Per-sample crop/flip come from
//                  hash(seed, epoch, sample index).
#include "common.h"

namespace pmd {

__device__ __forceinline__ uint32_t mix32(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 16);
}

__global__ void synth_images_kernel(bf16_t* __restrict__ x, long long* __restrict__ labels, int N,
                                    int H, int W, int Cp, int Creal, int classes,
                                    unsigned long long seed) {
  const long long npix = (long long)N * H * W;
  const int C8 = Cp >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix * C8;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = (int)(i % C8);
    const long long pix = i / C8;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cc * 8 + k;
      if (c < Creal) {
        const uint32_t h = mix32(seed * 0x100000001B3ull + (uint64_t)pix * 8 + c);
        // approx N(0,1): sum of two uniforms, rescaled (triangular, var 1)
        const float u1 = (h & 0xffff) * (1.f / 65536.f), u2 = (h >> 16) * (1.f / 65536.f);
        v[k] = (u1 + u2 - 1.f) * 2.449489743f;
      } else {
        v[k] = 0.f;
      }
    }
    reinterpret_cast<uint4*>(x)[i] = pack8(v);
    if (cc == 0 && (pix % ((long long)H * W)) == 0) {
      const long long n = pix / ((long long)H * W);
      labels[n] = (long long)(mix32(seed ^ (0xABCDull + (uint64_t)n * 7919ull)) % (uint32_t)classes);
    }
  }
}

// out element (b, y, x, c); OUT_BF16 selects bf16 vs fp32 output
template <bool OUT_BF16>
__global__ void cifar_augment_kernel(const uint8_t* __restrict__ data, const long long* __restrict__ idx,
                                     void* __restrict__ out, int B, int Cp, int train, int pad,
                                     unsigned long long seed, long long epoch) {
  const long long total = (long long)B * 32 * 32 * Cp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    long long t = i / Cp;
    const int xo = (int)(t % 32);
    t /= 32;
    const int yo = (int)(t % 32);
    const int b = (int)(t / 32);
    float v = 0.f;
    if (c < 3) {
      const long long s = idx[b];
      int sy = yo, sx = xo;
      if (train) {
        const uint32_t h = mix32(seed * 1315423911ull + (uint64_t)epoch * 2654435761ull + (uint64_t)s);
        const int span = 2 * pad + 1;
        const int oy = (int)(h % span), ox = (int)((h / span) % span);
        const int flip = (h >> 24) & 1;
        const int cx = flip ? 31 - xo : xo;
        sy = yo + oy - pad;
        sx = cx + ox - pad;
      }
      float px = 0.f;  // zero padding (black) before normalisation
      if ((unsigned)sy < 32u && (unsigned)sx < 32u) px = data[((s * 32 + sy) * 32 + sx) * 3 + c];
      v = (px * (1.f / 255.f) - 0.5f) / 0.5f;
    }
    if (OUT_BF16)
      reinterpret_cast<bf16_t*>(out)[i] = f2bf(v);
    else
      reinterpret_cast<float*>(out)[i] = v;
  }
}

int synth_images_launch(bf16_t* x, long long* labels, int N, int H, int W, int Cp, int Creal,
                        int classes, unsigned long long seed, hipStream_t st) {
  if (Cp % 8) return 1;
  long long work = (long long)N * H * W * (Cp / 8);
  long long b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(synth_images_kernel, dim3((int)b), dim3(256), 0, st, x, labels, N, H, W, Cp, Creal,
                     classes, seed);
  return 0;
}

int cifar_augment_launch(const uint8_t* data, const long long* idx, void* out, bool out_bf16, int B,
                         int Cp, bool train, int pad, unsigned long long seed, long long epoch,
                         hipStream_t st) {
  long long work = (long long)B * 32 * 32 * Cp;
  long long b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  if (out_bf16)
    hipLaunchKernelGGL((cifar_augment_kernel<true>), dim3((int)b), dim3(256), 0, st, data, idx, out, B,
                       Cp, train ? 1 : 0, pad, seed, epoch);
  else
    hipLaunchKernelGGL((cifar_augment_kernel<false>), dim3((int)b), dim3(256), 0, st, data, idx, out, B,
                       Cp, train ? 1 : 0, pad, seed, epoch);
  return 0;
}

}  // namespace pmd
