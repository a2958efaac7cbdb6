// Probe of ds_read_b64_tr_b8 (gfx950): which LDS bytes each lane receives when
// the 64 lanes supply consecutive 8-byte addresses (LDS byte i holds i & 255,
// second pass holds i >> 8 so bytes >= 256 are identified).  Prints, per lane,
// the 8 source byte offsets it received.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(unsigned char* out, int hi) {
  __shared__ __attribute__((aligned(16))) unsigned char s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = hi ? (i >> 8) : (i & 255);
  __syncthreads();
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(s + threadIdx.x * 8));
  *reinterpret_cast<v2i*>(out + threadIdx.x * 8) = v;
}
int main() {
  unsigned char *d, lo[512], hi[512];
  if (hipMalloc(&d, 512) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0);
  if (hipMemcpy(lo, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 1);
  if (hipMemcpy(hi, d, 512, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) printf(" %4d", hi[l * 8 + j] * 256 + lo[l * 8 + j]);
    printf("\n");
  }
  return 0;
}
