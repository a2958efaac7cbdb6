// Host-side launch entry points of the gfx950 kernels (implemented in the .hip TUs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace pmd {
typedef unsigned short bf16_t;

// Fused BatchNorm-backward reduce in the dgrad epilogue (see ConvArgs in conv_igemm.hip):
// mask = ReLU bitmask of the BN output (nullptr: no ReLU); one or two (y, params, red) sets.
struct BnReduceArgs {
  const uint8_t* mask;
  const bf16_t* y[2];
  const float* p[2];
  float* red[2];
};
// Deterministic statistics mode (test / debug, kernels/det.hip): det_begin swaps up to two
// slot-buffer pointers of one launch (*p0, *p1) for private per-row-block scratch slots and
// returns the slot count the kernel must index modulo (kStatSlots when the mode is off or
// there is nothing to swap; -1 on failure); det_end folds them, in a fixed order, into slot 0
// of the real buffers after the launch.
struct DetStats {
  float* real[2] = {nullptr, nullptr};
  float* scr = nullptr;
  int nslots = 0, width = 0, n = 0;
};
bool det_stats_on();
void det_stats_set(bool on);
int det_begin(DetStats& d, float** p0, float** p1, int nslots_bound, int width, hipStream_t st);
int det_end(DetStats& d, hipStream_t st);
int gpu_sleep_launch(int us, hipStream_t st);  // test utility: idle the stream for us microseconds
// data-gradient section probe (PMD_DGRAD_PROBE variant builds; 0 otherwise): records of 16 words
int conv_probe_set(void* buf, int cap);
int conv_probe_count();
// stats (optional): BN statistic slots [kStatSlots][2][Nout] of (sum (y-K), sum (y-K)^2) with
// K = shift[n] (nullable: 0) -- see bn_moments in common.h
int conv_igemm_launch(const bf16_t* src, const bf16_t* wt, bf16_t* out, float* stats, int N, int H,
                      int W, int Cs, int OH, int OW, int Nout, int R, int S, int stride, int pad,
                      bool dgrad, const bf16_t* addend, const uint8_t* addend_mask,
                      const BnReduceArgs* bnr, hipStream_t st, const float* shift = nullptr);
// `batch` same-shape forward convolutions in one launch (grid.z), no epilogue fusions
int conv_igemm_batched_launch(const bf16_t* src, const bf16_t* wt, bf16_t* out, int batch, long long bs_src,
                              long long bs_wt, long long bs_out, int N, int H, int W, int Cs, int OH, int OW,
                              int Nout, int R, int S, int stride, int pad, hipStream_t st);
// Winograd F(2x2,3x3) transforms (stride-1 pad-1 3x3; the 16 GEMMs run on conv_igemm as 1x1 convs)
int winograd_filter_launch(const bf16_t* wk, bf16_t* U, int K, int Cp, bool flip, hipStream_t st);
int winograd_input_launch(const bf16_t* x, bf16_t* V, int N, int H, int W, int C, hipStream_t st);
int winograd_output_launch(const bf16_t* M, bf16_t* y, float* stats, int N, int H, int W, int K,
                           hipStream_t st, const float* shift = nullptr);
// the fused forward (input transform, 16 MFMA GEMMs, output transform + BN statistics in one kernel)
// from the transformed filter U [16][K][C]; C % 64 == 0, K % 64 == 0
int winograd_fused_fwd_launch(const bf16_t* x, const bf16_t* U, bf16_t* y, float* stats, const float* shift,
                              int N, int H, int W, int C, int K, hipStream_t st);
int winograd_fused_fwd_run(const bf16_t* x, const bf16_t* U, bf16_t* y, float* stats, const float* shift, int N,
                           int H, int W, int C, int K, int nslots, hipStream_t st);
// filter transform of the weight image wk [K][3][3][C] into a per-stream scratch + the fused kernel
int winograd_conv_fwd_run(const bf16_t* x, const bf16_t* wk, bf16_t* y, float* stats, const float* shift, int N,
                          int H, int W, int C, int K, int nslots, hipStream_t st);
// linear-BN backward helpers (kernels/bnlin.hip)
int bnlin_coeff_launch(const float* red, const float* count, float count_h, const float* gamma, const float* params,
                       const bf16_t* wk, bf16_t* g, float* bias, float* abc, int K, int C, int Cp, hipStream_t st);
int bnlin_dimg_launch(const float* gamma, const float* params, const bf16_t* wk, bf16_t* wkt_a, int K, int C, int Cp,
                      hipStream_t st);
int colsum_launch(const bf16_t* x, float* out, long long M, int C, hipStream_t st);
int bnlin_wgrad_launch(float* out, const float* abc, const float* T, const bf16_t* wk, const float* gz,
                       const float* cs, int K, int C, int Cp, hipStream_t st);
void conv_set_addend_bias(const float* b);  // fp32 [Nout] bias of the next dgrad's addend (this thread)
void conv_set_impl(int impl);
void conv_wgrad_set_impl(int impl);
void conv_set_tile(int t);
void conv_set_big_pipe(int p);
void conv_set_autotune(int on);
int conv_autotune_entries();
void conv_autotune_clear();
// per-shape tuning tables (conv fwd/dgrad: 13 key ints + choice; wgrad: 11 + variant)
std::vector<int> conv_autotune_export();
int conv_autotune_import(const std::vector<int>& flat);
std::vector<int> wgrad_autotune_export();
int wgrad_autotune_import(const std::vector<int>& flat);
void wgrad_autotune_clear();
// grouped weight-image prep (one launch for every conv of a model)
struct WeightPrepDesc {
  const float* w;  // fp32 [K][R][S][C] (channels_last parameter storage)
  bf16_t* wk;      // [K][R][S][Cp]
  bf16_t* wkt;     // [Cp][R][S][K] or nullptr
  int K, RS, C, Cp;
};
// mode bit 0: forward images (wk), bit 1: dgrad images (wkt)
void conv_weight_prep_grouped_launch(const WeightPrepDesc* d_descs, const int* d_block_start, int n,
                                     int total_blocks, hipStream_t st, int mode = 3);  // 0 register staging, 1 LDS-DMA
void conv_weight_prep_launch(const float* w, bf16_t* wk, bf16_t* wkt, int K, int RS, int C, int Cp,
                             hipStream_t st);
// split-K plan: number of partial slices the workspace must hold ([splits][K][R*S*C] fp32)
int conv_wgrad_splits(int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride,
                      int pad);
// dw += dW (dw must be initialised: zeros or an accumulation target)
int conv_wgrad_launch(const bf16_t* dy, const bf16_t* x, float* dw, float* ws, int N, int H, int W,
                      int C, int P, int Q, int K, int R, int S, int stride, int pad, hipStream_t st);
// deferred split-K reductions: queue them (per thread) while on, launch them grouped with
// wgrad_flush on the stream that computed the partial slices (returns nonzero on a mismatch)
void wgrad_set_defer(bool on);
bool wgrad_defer();
int wgrad_pending();
int wgrad_flush(hipStream_t st);
// FP8 weight gradient: e5m2 dY x e4m3 X on the scaled 16x16x128 MFMA (kernels/conv_wgrad.hip)
// FP8 data gradient: e5m2 dY [N,P,Q,K] x e4m3 wkt image [Cp][R][S][K] -> bf16 dX [N,H,W,Cp] with the
// bf16 dgrad's epilogue (addend (+mask), fused BN-backward reduce) (kernels/conv_igemm.hip)
int conv_dgrad_fp8_launch(const uint8_t* dyq, const uint8_t* wtq, const float* sdy, const float* sw, bf16_t* out,
                          int N, int H, int W, int Cs, int OH, int OW, int Nout, int R, int S, int stride, int pad,
                          const bf16_t* addend, const uint8_t* addend_mask, const BnReduceArgs* bnr,
                          hipStream_t st);
int conv_wgrad_fp8_splits(int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride, int pad);
int conv_wgrad_fp8_launch(const uint8_t* dyq, const uint8_t* xq, const float* sdy, const float* sx, float* dw,
                          float* ws, int N, int H, int W, int C, int P, int Q, int K, int R, int S, int stride,
                          int pad, hipStream_t st);

// shift (nullable): the statistics shift K the sums were taken about; overwritten with
// the batch mean (the next step's shift)
int bn_finalize_launch(const float* sums, const float* count, const float* gamma, const float* beta,
                       float* params, float* rm, float* rv, long long* nbt, float* shift, int C,
                       float eps, float momentum, bool eval_mode, hipStream_t st);
int stats_collapse_launch(float* a, int Ca, float* b, int Cb, float count, float* out,
                          bool with_count, bool clear, float* acc_a0, float* acc_a1, float* acc_b0,
                          float* acc_b1, hipStream_t st);
int stats_finalize_local_launch(float* slots, float count, const float* gamma, const float* beta,
                                float* params, float* rm, float* rv, long long* nbt, float* shift, int C,
                                float eps, float momentum, hipStream_t st);
// mask: ReLU bitmask, one byte per 8-channel chunk (bit k = element k of the chunk > 0)
// q8 (optional): e4m3 copy of the output scaled by *qscale, amax(|out|) -> *qamax
int bn_apply_launch(const bf16_t* y1, const float* p1, const bf16_t* r, const float* p2, bf16_t* out,
                    uint8_t* mask, long long M, int C, int mode, bool relu, uint8_t* q8,
                    const float* qscale, float* qamax, hipStream_t st);
int bn_bwd_reduce_launch(const bf16_t* dout, const uint8_t* mask, const bf16_t* y,
                         const float* params, float* red, int M, int C, bool relu, hipStream_t st);
int bn_bwd_elemt_launch(const bf16_t* dout, const uint8_t* mask, const bf16_t* y, const float* params,
                        const float* gamma, const float* red, const float* count, float count_h,
                        bf16_t* dy, bf16_t* dzm, long long M, int C, bool relu, bool eval_mode,
                        hipStream_t st, uint8_t* q8 = nullptr, const float* qscale = nullptr,
                        float* qamax = nullptr);

// fused stem tail (kernels/stem.hip): BN + ReLU + 3x3/s2 max-pool, and its backward
// space-to-depth stem (7x7/s2 over 3 channels as 4x4/s1 over 16)
int stem_s2d_input_launch(const bf16_t* x, bf16_t* xs, int N, int H, int W, hipStream_t st);
int stem_s2d_weight_launch(const float* w, bf16_t* ws, int K, int C, hipStream_t st);
int stem_s2d_wgrad_fold_launch(const float* dws, float* dw, int K, int C, bool accumulate, hipStream_t st);
int stem_pool_fwd_launch(const bf16_t* y, const float* params, bf16_t* out, uint8_t* arg, int N, int H,
                         int W, int C, int P, int Q, hipStream_t st);
int stem_pool_bwd_reduce_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y,
                                const float* params, float* red, int N, int H, int W, int C, int P, int Q,
                                hipStream_t st);
int stem_pool_bwd_elemt_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y, const float* params,
                               const float* gamma, const float* red, const float* count, float count_h,
                               bf16_t* dy, int N, int H, int W, int C, int P, int Q, bool eval_mode,
                               hipStream_t st);
// the fused stem backward: stem conv weight gradient with its dY (max-pool + BN backward) produced
// in-kernel (kernels/conv_wgrad.hip); dw == nullptr: only report the workspace split count
int stem_wgrad_fused_launch(const bf16_t* dout, const uint8_t* arg, const bf16_t* y, const float* params,
                            const float* gamma, const float* red, const float* count, float count_h,
                            const bf16_t* x, float* dw, float* ws, int N, int H, int W, int C, int P, int Q,
                            int K, int R, int S, int pad, int P2, int Q2, int* splits, hipStream_t st);
int maxpool_fwd_launch(const bf16_t* x, bf16_t* out, uint8_t* arg, int N, int H, int W, int C, int P,
                       int Q, hipStream_t st);
int maxpool_bwd_launch(const bf16_t* dout, const uint8_t* arg, bf16_t* dx, int N, int H, int W, int C,
                       int P, int Q, hipStream_t st);
int avgpool_fwd_launch(const bf16_t* x, float* out, int N, int HW, int C, hipStream_t st);
int avgpool_bwd_launch(const float* dout, bf16_t* dx, int N, int HW, int C, hipStream_t st);
int xent_fwd_launch(const float* logits, const long long* target, float* loss, float* lse,
                    long long* correct, int N, int V, hipStream_t st);
int xent_bwd_launch(const float* logits, const long long* target, const float* lse, const float* gloss,
                    float* grad, int N, int V, hipStream_t st);
int zero_launch(void* ptr, long long nbytes, hipStream_t st);  // memset 0 (framework kernel)
int sgd_launch(float* p, const float* g, float* buf, long long n, float lr, const float* lr_dev,
               float momentum, float wd, float damp, bool nesterov, bool first, hipStream_t st);

// classifier GEMMs (kernels/linear.hip): C[i][j] (+)= sum_r A(i,r) B(r,j) on bf16 MFMA, fp32 I/O
int linear_mfma_launch(const float* A, const float* B, float* C, const float* bias, long long sai,
                       long long sar, long long sbr, long long sbj, int M, int Nc, int R, bool accumulate,
                       float* ws, hipStream_t st);
// fp32 workspace the split-K combine needs for this product (0: single split)
long long linear_workspace_floats(int M, int Nc, int R);
int linear_colsum_launch(const float* g, float* db, int rows, int cols, bool accumulate, hipStream_t st);

int synth_images_launch(bf16_t* x, long long* labels, int N, int H, int W, int Cp, int Creal,
                        int classes, unsigned long long seed, hipStream_t st);
int cifar_augment_launch(const uint8_t* data, const long long* idx, void* out, bool out_bf16, int B,
                         int Cp, bool train, int pad, unsigned long long seed, long long epoch,
                         hipStream_t st);

// FP8 e4m3 (kernels/fp8.hip)
int quant_bf16_fp8_launch(const bf16_t* x, uint8_t* q, const float* scale, float* amax, long long n,
                          hipStream_t st, bool bf8 = false);
// all fp8 weight images of a model in one launch (per-conv scale / amax sites)
struct Fp8WeightDesc {
  const float* w;      // fp32 [K][R][S][C]
  uint8_t* q;          // e4m3 [K][R][S][Cp]
  uint8_t* qt;         // optional e4m3 [Cp][R][S][K]: the fp8 dgrad's B^T image (nullptr: none)
  const float* scale;  // [1]
  float* amax;         // [kAmaxSlots]
  int K, RS, C, Cp;
};
void quant_weight_fp8_grouped_launch(const Fp8WeightDesc* d_descs, const int* d_block_start, int n,
                                     int total_blocks, hipStream_t st);
int quant_weight_fp8_launch(const float* w, uint8_t* q, const float* scale, float* amax, int K, int RS,
                            int C, int Cp, hipStream_t st, uint8_t* qt = nullptr);
int fp8_update_scales_launch(float* amax, float* scale, int n, float fmax, hipStream_t st);
int dequant_fp8_launch(const uint8_t* q, float* out, const float* inv_scale, long long n, hipStream_t st,
                       bool bf8 = false);
int fp8_mfma_probe_launch(const uint8_t* A, const uint8_t* Bt, float* C, hipStream_t st);
// y(bf16) = conv(xq, wq) / (sx * sw) with e4m3 NHWC input / KRSC weight; optional BN stats slots
int conv_fwd_fp8_igemm_launch(const uint8_t* xq, const uint8_t* wq, bf16_t* out, float* stats, const float* sx,
                              const float* sw, int N, int H, int W, int Cs, int OH, int OW, int Nout, int R, int S,
                              int stride, int pad, hipStream_t st, const float* shift);
int conv_fp8_fwd_launch(const uint8_t* x, const uint8_t* w, bf16_t* out, float* stats, const float* sx,
                        const float* sw, int N, int H, int W, int C, int OH, int OW, int K, int R,
                        int S, int stride, int pad, hipStream_t st, const float* shift = nullptr);

// One-shot xGMI all-reduce (kernels/xgmi.hip).  Receive-buffer layout per rank:
// flags [kXgmiMaxRanks][kXgmiMaxBlocks] uint32 (kXgmiFlagBytes), then data
// [2 parities][world][kXgmiCap] fp32.
constexpr int kXgmiMaxRanks = 16;
constexpr int kXgmiChunk = 512;        // floats per block of the fused SyncBN kernel (small:
constexpr int kXgmiMaxBlocks = 64;     // its slot collapse is latency-bound, so spread it out)
constexpr int kXgmiCap = kXgmiChunk * kXgmiMaxBlocks;  // max floats per call
constexpr int kXgmiFlagBytes = 4096;
// Per-communicator control block passed to every exchange kernel.  Block b of EVERY kernel
// owns region [b * kXgmiChunk, (b + 1) * kXgmiChunk) of each parity slot and epochs[b].
struct XgmiCtl {
  uint32_t* epochs;                 // [kXgmiMaxBlocks] per-block call counters (device)
  uint32_t* err;                    // device error word
  uint32_t* err_host;               // host-mapped error word (device view; nullable)
  unsigned long long timeout_ticks; // spin deadline, wall-clock ticks
  int order;                        // 0 light (completion-only), 1 strict (release/acquire fences)
  int delay_where;                  // test-only skew: 0 off, 1 before publish, 2 before reading
  unsigned long long delay_ticks;
  int ar_region;                    // plain all-reduce floats per block: 0 = kXgmiChunk (test-only override)
};
int xgmi_allreduce_launch(float* const* data, uint32_t* const* flags, float* x, int n, int rank,
                          int world, const XgmiCtl& c, hipStream_t st);

// SyncBN collapse + one-shot exchange + finalize (fwd) / global sums (bwd) in one kernel
struct BnFinalizeOut {
  const float* gamma;
  const float* beta;
  float* params;  // [4][C]
  float* rm;      // running stats (nullable)
  float* rv;
  long long* nbt;
  float* shift;   // statistics shift K (nullable), overwritten with the batch mean
  float eps, momentum;
};
struct XgmiBnArgs {
  int mode;                 // 0 forward statistics, 1 backward reduce
  float* slotsA;            // [kStatSlots][2][CA], read-and-clear
  float* slotsB;            // optional second BN (projection shortcut)
  int CA, CB;               // CB = 0 without B
  float count;              // local element count per channel (forward)
  BnFinalizeOut fA, fB;     // forward outputs
  float* count_out;         // forward: global count [1]
  float* accA0;             // backward: += local sums (d_beta, d_gamma arena views; nullable)
  float* accA1;
  float* accB0;
  float* accB1;
  float* outA;              // backward: global [2][CA]
  float* outB;
  int pairs;  // channel pairs per block (set by the launcher)
};
// fused SyncBN kernel: channel pairs per block (1..kBnPairs); default kBnPairs
void xgmi_set_bn_pairs(int pairs);
int xgmi_bn_launch(float* const* data, uint32_t* const* flags, const XgmiBnArgs& args, int rank, int world,
                   const XgmiCtl& c, hipStream_t st);
}  // namespace pmd
