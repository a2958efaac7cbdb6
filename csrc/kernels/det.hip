// Deterministic statistics mode (test / debug only; ops/functional.py set_deterministic).
//
// In production every BN-statistics producer (the conv forward's statistics epilogue, the
// dgrad's fused BN-backward reduce, bn_bwd_reduce, the stem pool backward, the fp8 and
// Winograd forward epilogues) adds one fp32 partial per channel and block into one of
// kStatSlots slot copies, several blocks per slot.  fp32 addition is not associative, so the
// order those atomics retire in moves the low bits of every sum from run to run, and a
// cross-stream hand-off or a graph replay can only be checked against that noise.
//
// Here a launch's slot pointers are swapped for a per-stream zeroed scratch holding one
// private slot per row block (at most one atomic per address: 0 + v is exact), and after the
// launch det_fold sums the slots in a fixed order into slot 0 of the real buffer (and clears
// them), so the consumers (stats_collapse, stats_finalize_local, the xGMI exchange) are
// unchanged and two identical steps are bit-identical.
#include "common.h"

#include <map>
#include <mutex>

namespace pmd {

namespace {
bool g_det = false;
struct Scratch {
  float* p = nullptr;
  size_t n = 0;  // floats
};
std::mutex g_mu;
std::map<hipStream_t, Scratch> g_scr;

// zeroed scratch of >= n floats owned by stream st (grown outside stream capture only).  A
// outgrown buffer is never freed: in-flight launches and captured HIP graphs may still point
// at it (debug mode: the leak is bounded by the largest launch).
float* scratch(hipStream_t st, size_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  Scratch& s = g_scr[st];
  if (s.n >= n) return s.p;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(st, &cs);
  if (cs != hipStreamCaptureStatusNone) return nullptr;  // warm the mode up before capturing
  size_t want = s.n ? 2 * s.n : ((size_t)8 << 20);
  while (want < n) want *= 2;
  float* p = nullptr;
  if (hipMalloc(&p, want * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, want * sizeof(float), st) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  s.p = p;
  s.n = want;
  return p;
}
}  // namespace

bool det_stats_on() { return g_det; }
void det_stats_set(bool on) { g_det = on; }

// out[i] += sum over slots k (ascending, 4 contiguous quarters combined in order) of scr[k][i];
// the scratch slots are cleared for the next launch on this stream
__global__ __launch_bounds__(256) void det_fold_kernel(float* __restrict__ scr, float* __restrict__ out,
                                                       int nslots, int width) {
  __shared__ float part[4][64];
  const int li = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + li;
  float s = 0.f;
  if (i < width) {
    const int q = (nslots + 3) / 4;
    const int lo = g * q, hi = lo + q < nslots ? lo + q : nslots;
    for (int k = lo; k < hi; ++k) {
      float* p = scr + (size_t)k * width + i;
      s += *p;
      *p = 0.f;
    }
  }
  part[g][li] = s;
  __syncthreads();
  if (g == 0 && i < width) out[i] += ((part[0][li] + part[1][li]) + part[2][li]) + part[3][li];
}

int det_begin(DetStats& d, float** p0, float** p1, int nslots_bound, int width, hipStream_t st) {
  d = DetStats{};
  if (!g_det) return kStatSlots;
  float** ps[2] = {p0, p1};
  int n = 0;
  for (float** pp : ps) n += (pp && *pp) ? 1 : 0;
  if (!n) return kStatSlots;
  if (nslots_bound < 1 || width < 1) return -1;
  const size_t per = (size_t)nslots_bound * width;
  float* s = scratch(st, (size_t)n * per);
  if (!s) return -1;
  int k = 0;
  for (float** pp : ps) {
    if (pp && *pp) {
      d.real[k] = *pp;
      *pp = s + (size_t)k * per;
      ++k;
    }
  }
  d.scr = s;
  d.nslots = nslots_bound;
  d.width = width;
  d.n = n;
  return nslots_bound;
}

int det_end(DetStats& d, hipStream_t st) {
  for (int k = 0; k < d.n; ++k)
    hipLaunchKernelGGL(det_fold_kernel, dim3((d.width + 63) / 64), dim3(256), 0, st,
                       d.scr + (size_t)k * d.nslots * d.width, d.real[k], d.nslots, d.width);
  d = DetStats{};
  return 0;
}

// test utility: one wave that idles its stream for `us` microseconds of wall clock (100 MHz
// constant counter), bounded -- the hand-off tests' way to hold a stream back (negative controls)
__global__ void gpu_sleep_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while ((unsigned long long)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int gpu_sleep_launch(int us, hipStream_t st) {
  if (us < 0 || us > 1000000) return 1;
  hipLaunchKernelGGL(gpu_sleep_kernel, dim3(1), dim3(64), 0, st, (unsigned long long)us * 100ull);
  return 0;
}

}  // namespace pmd
