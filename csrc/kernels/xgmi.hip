// One-shot xGMI all-reduce for small, latency-bound messages (K21).
//
// SyncBN issues one tiny all-reduce per BN site per pass (2C+1 floats fwd,
// 2C bwd; 53+53 per ResNet-50 step, reference main.py:43 ->
// torch:nn/modules/_functions.py:65-83,155-165), all on the critical path.
// A ring collective needs 2(W-1) dependent hops; this needs ONE: every rank
// pushes its vector straight into a slot of every peer's receive buffer
// over the point-to-point xGMI links, raises a per-peer flag, waits for all
// W flags of its own buffer, and sums the W slots locally in rank order (so
// every rank produces bit-identical results).
//
// Receive buffers are IPC-mapped, uncached device memory (coherent across
// the fabric without cache maintenance).  Flags carry a per-block epoch that
// only increases; slots are double-buffered by epoch parity, which is
// enough because a rank can run at most one call ahead of any peer (it
// cannot finish call e+1 before every peer has *started* e+1, i.e. finished
// reading call e).  Spins are bounded in WALL time (s_memrealtime, the
// constant 100 MHz clock -- not an iteration count): on timeout the kernel
// sets an error word in device memory AND a host-mapped word, then returns
// instead of hanging the GPU, and POISONS its outputs: every value it would
// have produced (the summed vector; BN params / global backward sums) is
// written as NaN, so whatever consumes it -- activations, loss, gradients,
// weights after the SGD step -- is visibly invalid rather than silently
// wrong (running statistics and the shift are left untouched).  Detection:
// the training loop reads the host-mapped word after every step without a
// device sync (XgmiAllReduce.raise_if_failed), so a failure is raised within
// the host's run-ahead window (the steps already queued when the word is set;
// bounded by the next synchronising print), and the epoch-end synchronise +
// check runs before any checkpoint is written: a poisoned state is never saved.
#include "common.h"

// Memory ordering of the exchange: a RUNTIME choice (XgmiCtl::order), picked at startup by
// the stress self-test (parallel/xgmi.py: light first, strict if light fails, RCCL SyncBN if
// both fail).  Receive buffers and flags live in uncached device memory (runtime/xgmi.cpp),
// and EVERY payload and flag store is a system-scope store (sc0 sc1: write-through to
// memory on the writer's side, whatever MTYPE the importing GPU's IPC mapping carries), every
// payload / flag load a system-scope load (bypasses L1 and L2).
//   kXgmiLight  (0): completion-only publish -- each storing wave waits for its payload stores
//                    (s_waitcnt vmcnt(0)), a workgroup barrier, then ONE relaxed flag store per
//                    peer; the reader polls relaxed and reads the payload after the match.
//   kXgmiStrict (1): the same plus a system-scope RELEASE fence (L2 write-back) between the
//                    barrier and the flag store (followed by an explicit vmcnt(0): the compiler
//                    may drop the wait after the write-back, MI355X_MICROARCH "Compiler hazard"),
//                    and ONE system-scope ACQUIRE fence (L1/L2 invalidate) after the poll
//                    matched, before the workgroup barrier that releases the readers.
// The old C++ release-store / acquire-load forms cost 24 us per call (an L2 write-back per
// block and an invalidate per SPIN ITERATION; profiles/rehearsal_r04.txt); the strict form
// pays one write-back per block and one invalidate per matched flag.
constexpr int kXgmiLight = 0;
constexpr int kXgmiStrict = 1;

namespace pmd {

template <int ORDER>
__device__ __forceinline__ void xgmi_publish_fence() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's payload stores completed
}
template <int ORDER>
__device__ __forceinline__ void xgmi_flag_store(uint32_t* f, uint32_t e) {
  if constexpr (ORDER == kXgmiStrict) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __hip_atomic_store(f, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t xgmi_flag_load(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int ORDER>
__device__ __forceinline__ void xgmi_after_match() {
  if constexpr (ORDER == kXgmiStrict) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// payload store / load: system scope (write-through store, L1+L2-bypassing load)
__device__ __forceinline__ void xgmi_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float xgmi_ld(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Test-only skew injection (XgmiCtl::delay_*): the calling rank idles `ticks` of the wall
// clock at one point of the protocol -- 1: before publishing (a late rank), 2: after its
// flags matched, before reading the payload (a slow reader: what a peer running ahead could
// overwrite).  0 = off (the production value).
__device__ __forceinline__ void xgmi_delay(unsigned long long ticks) {
  const unsigned long long t0 = (unsigned long long)wall_clock64();
  while ((unsigned long long)wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

struct XgmiPeers {
  float* data[kXgmiMaxRanks];
  uint32_t* flags[kXgmiMaxRanks];
};

// Wait until the flag reaches epoch e; false (and both error words set) once
// `ticks` of the constant wall clock have passed.
__device__ __forceinline__ bool xgmi_wait_flag(const uint32_t* f, uint32_t e, const XgmiCtl& c) {
  const unsigned long long t0 = (unsigned long long)wall_clock64();
  while ((int)(xgmi_flag_load(f) - e) < 0) {
    if ((unsigned long long)wall_clock64() - t0 > c.timeout_ticks) {
      atomicOr(c.err, 1u);
      if (c.err_host) __hip_atomic_store(c.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// The exchange shared by both kernels, for block b of a call at epoch e: region
// [b * kXgmiChunk, (b + 1) * kXgmiChunk) of parity slot (e & 1).  ONE block -> region map and
// ONE per-block epoch counter for every kernel, so the "at most one call ahead" argument holds
// for every region whichever kernels are interleaved: a rank that reached epoch e + 1 on block
// b finished epoch e there, which needed every peer's epoch-e flag of block b, which each peer
// raised only after its epoch e - 1 read of that region (stream order) -- so the parity slot it
// now overwrites is no longer read by anyone.  (Round 4 gave the plain all-reduce 2048-float
// regions, so its block 0 overlapped the fused kernel's blocks 1-3 under a different epoch.)
//   push `len` floats from `src` (LDS or global) to slot [par][rank] of every peer, raise my
//   flag, wait for every peer's flag; returns false on timeout.
template <int ORDER>
__device__ __forceinline__ bool xgmi_exchange(const XgmiPeers& peers, const float* src, int len, int extra_idx,
                                              const float* extra, int rank, int world, int b, int region,
                                              uint32_t e, const XgmiCtl& c, int* bad_sh) {
  const int tid = threadIdx.x;
  if (c.delay_where == 1 && c.delay_ticks) xgmi_delay(c.delay_ticks);
  const size_t my_slot = ((size_t)(e & 1) * world + rank) * kXgmiCap + (size_t)region;
  for (int r = 0; r < world; ++r) {
    float* dst = peers.data[r] + my_slot;
    for (int i = tid; i < len; i += 256) xgmi_st(dst + i, src[i]);
    if (extra && tid == 0) xgmi_st(dst + extra_idx, *extra);
  }
  xgmi_publish_fence<ORDER>();
  __syncthreads();
  if (tid < world) xgmi_flag_store<ORDER>(peers.flags[tid] + rank * kXgmiMaxBlocks + b, e);
  if (tid < world) {
    const uint32_t* f = peers.flags[rank] + tid * kXgmiMaxBlocks + b;
    if (!xgmi_wait_flag(f, e, c)) *bad_sh = 1;
    xgmi_after_match<ORDER>();
  }
  if (c.delay_where == 2 && c.delay_ticks) xgmi_delay(c.delay_ticks);
  __syncthreads();   // (the flag loads returned before any thread reads the payload)
  return *bad_sh == 0;
}

template <int ORDER>
__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(XgmiPeers peers, float* __restrict__ x, int n,
                                                            int rank, int world, XgmiCtl c) {
  __shared__ uint32_t e_sh;
  __shared__ int bad_sh;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    e_sh = c.epochs[b] + 1;
    c.epochs[b] = e_sh;
    bad_sh = 0;
  }
  __syncthreads();
  const uint32_t e = e_sh;
  // c.ar_region: floats per block; kXgmiChunk in production.  The round-4 split map (2048) is
  // kept ONLY as the negative control of the interleaving stress test (tests/test_xgmi_gpu.py)
  const int chunk = c.ar_region > 0 ? c.ar_region : kXgmiChunk;
  const int lo = b * chunk;
  const int len = min(chunk, n - lo);
  // 1-3) push my region to every rank, flag, wait for all W flags of my buffer
  const bool ok = xgmi_exchange<ORDER>(peers, x + lo, len, 0, nullptr, rank, world, b, lo, e, c, &bad_sh);
  // 4) sum the W slots in rank order (identical on every rank); NaN on timeout
  const float* mine = peers.data[rank] + (size_t)(e & 1) * world * kXgmiCap + lo;
  for (int i = tid; i < len; i += 256) {
    float s = 0.f;
    for (int r = 0; r < world; ++r) s += xgmi_ld(mine + (size_t)r * kXgmiCap + i);
    x[lo + i] = ok ? s : __builtin_nanf("");
  }
}

int xgmi_allreduce_launch(float* const* data, uint32_t* const* flags, float* x, int n, int rank,
                          int world, const XgmiCtl& c, hipStream_t st) {
  if (world < 1 || world > kXgmiMaxRanks || n < 0 || n > kXgmiCap) return 1;
  if (n == 0) return 0;
  XgmiPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.flags[r] = flags[r];
  }
  const int chunk = c.ar_region > 0 ? c.ar_region : kXgmiChunk;
  if (chunk > kXgmiCap) return 1;
  const int nb = (n + chunk - 1) / chunk;
  if (c.order == kXgmiStrict)
    hipLaunchKernelGGL(xgmi_allreduce_kernel<kXgmiStrict>, dim3(nb), dim3(256), 0, st, p, x, n, rank, world, c);
  else
    hipLaunchKernelGGL(xgmi_allreduce_kernel<kXgmiLight>, dim3(nb), dim3(256), 0, st, p, x, n, rank, world, c);
  return 0;
}

}  // namespace pmd

namespace pmd {

// ---------------------------------------------------------------------------
// SyncBN in ONE kernel per BN site and pass (instead of collapse -> all-reduce
// -> finalize): each block owns up to kBnPairs channels (of BN A, then BN B),
//   0) collapses their kStatSlots statistic slots (read-and-clear) into
//      (s0, s1) pairs -- backward also adds the LOCAL sums into the gamma/beta
//      gradient arena (DDP averages those later, like every other gradient);
//   1-3) exchanges the pairs (+ the local element count) one-shot over xGMI
//      through the same xgmi_exchange (same block -> region map, same epochs)
//      as xgmi_allreduce_kernel;
//   4) forward: BatchNorm finalize from the global sums (params [4][C],
//      running stats, num_batches_tracked, global count); backward: writes the
//      global (sum dz, sum dz*xhat) as [2][C] for bn_bwd_elemt.
constexpr int kBnPairs = (kXgmiChunk - 2) / 2;  // 255 channels per block; [2*kBnPairs] = count
static int g_bn_pairs = 64;  // one 64-channel collapse pass per block (see the kernel)
void xgmi_set_bn_pairs(int pairs) { g_bn_pairs = pairs < 1 ? 1 : (pairs > kBnPairs ? kBnPairs : pairs); }

template <int ORDER>
__global__ __launch_bounds__(256) void xgmi_bn_kernel(XgmiPeers peers, XgmiBnArgs a, int rank, int world,
                                                     XgmiCtl ctl) {
  __shared__ float loc[kXgmiChunk];
  __shared__ float part[4][64][2];
  __shared__ uint32_t e_sh;
  __shared__ int bad_sh;
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    e_sh = ctl.epochs[b] + 1;
    ctl.epochs[b] = e_sh;
    bad_sh = 0;
  }
  const int P = a.CA + a.CB;
  const int p0 = b * a.pairs;
  const int np = min(a.pairs, P - p0);
  // 0) collapse my channels' slots, laid out like the local stats_collapse kernel: 64
  //    channels per pass, the 4 waves each summing 16 of the kStatSlots slots (all loads
  //    issued before the first add -- the slots were filled by memory-side atomics, so each
  //    read is a full memory round trip), then a fixed-order combine of the 4 partials
  //    through LDS.  (One thread per channel summing all 64 slots was 2.5x slower per
  //    call: 4x less memory-level parallelism per channel.)
  static_assert(kStatSlots == 64, "4 groups of 16 slots");
  {
    const int li = tid & 63, g = tid >> 6;
    for (int j0 = 0; j0 < np; j0 += 64) {
      const int j = j0 + li;
      const int pi = p0 + j;
      const bool isA = pi < a.CA;
      float* slots = isA ? a.slotsA : a.slotsB;
      const int C = isA ? a.CA : a.CB;
      const int c = isA ? pi : pi - a.CA;
      float s0 = 0.f, s1 = 0.f;
      if (j < np) {
        float v0[16], v1[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          v0[k] = slots[(size_t)(16 * g + k) * 2 * C + c];
          v1[k] = slots[(size_t)(16 * g + k) * 2 * C + C + c];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          s0 += v0[k];
          s1 += v1[k];
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          slots[(size_t)(16 * g + k) * 2 * C + c] = 0.f;
          slots[(size_t)(16 * g + k) * 2 * C + C + c] = 0.f;
        }
      }
      part[g][li][0] = s0;
      part[g][li][1] = s1;
      __syncthreads();
      if (g == 0 && j < np) {
        s0 = ((part[0][li][0] + part[1][li][0]) + part[2][li][0]) + part[3][li][0];
        s1 = ((part[0][li][1] + part[1][li][1]) + part[2][li][1]) + part[3][li][1];
        loc[2 * j] = s0;
        loc[2 * j + 1] = s1;
        if (a.mode == 1) {
          float* acc0 = isA ? a.accA0 : a.accB0;
          float* acc1 = isA ? a.accA1 : a.accB1;
          if (acc0) acc0[c] += s0;
          if (acc1) acc1[c] += s1;
        }
      }
      __syncthreads();   // part[] is reused by the next pass
    }
  }
  if (tid == 0) loc[2 * kBnPairs] = a.count;
  __syncthreads();
  const uint32_t e = e_sh;
  const int par = e & 1;
  // 1-3) push pairs + count into slot [par][rank] of every rank's receive buffer, flag, wait
  const bool ok = xgmi_exchange<ORDER>(peers, loc, 2 * np, 2 * kBnPairs, &loc[2 * kBnPairs], rank, world, b,
                                       b * kXgmiChunk, e, ctl, &bad_sh);
  const bool bad = !ok;
  // 4) global sums in rank order, then finalize / publish (NaN outputs on timeout)
  const float* mine = peers.data[rank] + (size_t)par * world * kXgmiCap + (size_t)b * kXgmiChunk;
  float cnt = 0.f;
  for (int r = 0; r < world; ++r) cnt += xgmi_ld(mine + (size_t)r * kXgmiCap + 2 * kBnPairs);
  for (int j = tid; j < np; j += 256) {
    float g0 = 0.f, g1 = 0.f;
    for (int r = 0; r < world; ++r) {
      g0 += xgmi_ld(mine + (size_t)r * kXgmiCap + 2 * j);
      g1 += xgmi_ld(mine + (size_t)r * kXgmiCap + 2 * j + 1);
    }
    const int pi = p0 + j;
    const bool isA = pi < a.CA;
    const int C = isA ? a.CA : a.CB;
    const int c = isA ? pi : pi - a.CA;
    if (bad) {
      const float qn = __builtin_nanf("");
      if (a.mode == 0) {
        const BnFinalizeOut& o = isA ? a.fA : a.fB;
        o.params[c] = qn;
        o.params[C + c] = qn;
        o.params[2 * C + c] = qn;
        o.params[3 * C + c] = qn;
      } else {
        float* out = isA ? a.outA : a.outB;
        out[c] = qn;
        out[C + c] = qn;
      }
    } else if (a.mode == 0) {
      const BnFinalizeOut& o = isA ? a.fA : a.fB;
      // every rank shifted its sums by the same K (the previous step's global mean)
      float mean, var;
      bn_moments(g0, g1, cnt, o.shift ? o.shift[c] : 0.f, mean, var);
      if (o.shift) o.shift[c] = mean;
      const float inv = rsqrtf(var + o.eps);
      const float sc = o.gamma[c] * inv;
      o.params[c] = mean;
      o.params[C + c] = inv;
      o.params[2 * C + c] = sc;
      o.params[3 * C + c] = o.beta[c] - mean * sc;
      if (o.rm) {
        const float unb = var * (cnt / fmaxf(cnt - 1.f, 1.f));
        o.rm[c] = (1.f - o.momentum) * o.rm[c] + o.momentum * mean;
        o.rv[c] = (1.f - o.momentum) * o.rv[c] + o.momentum * unb;
      }
      if (c == 0 && o.nbt) o.nbt[0] += 1;
    } else {
      float* out = isA ? a.outA : a.outB;
      out[c] = g0;
      out[C + c] = g1;
    }
  }
  if (a.mode == 0 && b == 0 && tid == 0 && a.count_out) a.count_out[0] = bad ? __builtin_nanf("") : cnt;
}

int xgmi_bn_launch(float* const* data, uint32_t* const* flags, const XgmiBnArgs& args, int rank, int world,
                   const XgmiCtl& c, hipStream_t st) {
  if (world < 1 || world > kXgmiMaxRanks) return 1;
  const int P = args.CA + args.CB;
  XgmiBnArgs a = args;
  a.pairs = g_bn_pairs;
  int nb = (P + a.pairs - 1) / a.pairs;
  if (nb > kXgmiMaxBlocks) {  // too many blocks for the flag table: use fuller ones
    a.pairs = kBnPairs;
    nb = (P + a.pairs - 1) / a.pairs;
  }
  if (P <= 0 || nb > kXgmiMaxBlocks) return 2;
  XgmiPeers p{};
  for (int r = 0; r < world; ++r) {
    p.data[r] = data[r];
    p.flags[r] = flags[r];
  }
  if (c.order == kXgmiStrict)
    hipLaunchKernelGGL(xgmi_bn_kernel<kXgmiStrict>, dim3(nb), dim3(256), 0, st, p, a, rank, world, c);
  else
    hipLaunchKernelGGL(xgmi_bn_kernel<kXgmiLight>, dim3(nb), dim3(256), 0, st, p, a, rank, world, c);
  return 0;
}

}  // namespace pmd
