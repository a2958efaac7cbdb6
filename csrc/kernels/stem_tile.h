// Pooled-gradient tile of the fused ImageNet stem backward (kernels/stem.hip): shared by the
// stem's BN-backward passes and the fused stem weight gradient (kernels/conv_wgrad.hip), which
// produces the stem conv's dY rows from it instead of reading them back from HBM.
#pragma once
#include "common.h"

namespace pmd {

// Backward of the fused stem tail.  Block = (image n, pooled row p): it owns
// input rows 2p and 2p+1 -- exactly the rows whose windows lie in pooled rows p
// and p+1 -- and stages those two pooled rows of dout and argmax taps in LDS
// once, so every input pixel reads its (1, 2 or 4) candidate windows from LDS
// instead of gathering 4 clamped windows from L2 (8 global loads per 16-B
// output chunk before; profiles/pool_bench).  Candidates are visited in
// ascending (p, q) order, the order of the composite maxpool_bwd sum.
struct StemBwdTile {
  const bf16_t* dl;   // LDS [2][Q][C] pooled gradient of rows p, p+1
  const uint8_t* al;  // LDS [2][Q][C] argmax taps
  int p, P, Q, C8;
  // dz of the 8-channel chunk (h, w, cc): bf16-rounded sum of the dout of the
  // windows whose argmax is this pixel, gated by the ReLU of BN(y)
  __device__ __forceinline__ void dz(int h, int w, int cc, const float (&v)[8], const float (&sc)[8],
                                     const float (&sh)[8], float (&out)[8]) const {
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    const int odd_h = h & 1, odd_w = w & 1;
    const int q0 = w >> 1;
#pragma unroll
    for (int a = 0; a < 2; ++a) {      // pooled row p + a
      if (a == 1 && (!odd_h || p + 1 >= P)) break;
      const int dh = odd_h ? (a == 0 ? 2 : 0) : 1;
#pragma unroll
      for (int b = 0; b < 2; ++b) {    // pooled col q0 + b
        if (b == 1 && (!odd_w || q0 + 1 >= Q)) break;
        const int dw = odd_w ? (b == 0 ? 2 : 0) : 1;
        const int tp = dh * 3 + dw;
        const int o = (a * Q + q0 + b) * C8 + cc;
        const uint4 gv = reinterpret_cast<const uint4*>(dl)[o];
        const uint2 av = reinterpret_cast<const uint2*>(al)[o];
        float g[8];
        unpack8(gv, g);
        const uint32_t aw[2] = {av.x, av.y};
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if ((int)((aw[k >> 2] >> ((k & 3) * 8)) & 0xff) == tp) acc[k] += g[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = (v[k] * sc[k] + sh[k] > 0.f) ? round_bf(acc[k]) : 0.f;
  }
};

// BN(+ReLU) backward of the stem: dy = a dz + b y + c with a = gamma invstd, b = -a invstd E[dz xhat],
// c = a (mean invstd E[dz xhat] - E[dz]) -- one explicit FMA form shared by the two-pass kernel
// (stem.hip) and the fused weight gradient (conv_wgrad.hip), so both round identically
__device__ __forceinline__ void stem_bwd_coeffs(float gamma, float inv, float mean, float mdy, float mdyx,
                                                float& a, float& b, float& c) {
  a = gamma * inv;
  b = -(a * inv) * mdyx;
  c = a * __builtin_fmaf(mean * inv, mdyx, -mdy);
}
__device__ __forceinline__ float stem_bwd_dy(float a, float b, float c, float dz, float y) {
  return __builtin_fmaf(a, dz, __builtin_fmaf(b, y, c));
}

// stage pooled rows p, p+1 (the second only if it exists) of image n into LDS
__device__ __forceinline__ void stem_stage_pooled(const bf16_t* __restrict__ dout, const uint8_t* __restrict__ arg,
                                                  bf16_t* dl, uint8_t* al, int n, int p, int P, int Q, int C8) {
  const int per_row = Q * C8;
  const int rows = p + 1 < P ? 2 : 1;
  const size_t base = ((size_t)n * P + p) * per_row;
  for (int i = threadIdx.x; i < rows * per_row; i += blockDim.x) {
    reinterpret_cast<uint4*>(dl)[i] = reinterpret_cast<const uint4*>(dout)[base + i];
    reinterpret_cast<uint2*>(al)[i] = reinterpret_cast<const uint2*>(arg)[base + i];
  }
}

}  // namespace pmd
