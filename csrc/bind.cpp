// Torch <-> gfx950 kernel bindings for pytorch_multiprocessing_distributed_amd._C
//
// Every op validates device / dtype / layout and throws on anything the
// kernels do not support (no silent fallback), allocates its outputs through
// the PyTorch-ROCm caching allocator and launches on the current HIP stream.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include "kernels/launchers.h"

namespace {

using torch::Tensor;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

constexpr int64_t pmd_slots() { return 64; }  // == pmd::kStatSlots (kernels/common.h)

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONT(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == torch::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == torch::kFloat32, #t " must be fp32")
#define CHECK_RC(rc, what) TORCH_CHECK((rc) == 0, what " rejected the shape (code ", rc, ")")

const pmd::bf16_t* bfp(const Tensor& t) { return reinterpret_cast<const pmd::bf16_t*>(t.data_ptr()); }
pmd::bf16_t* bfp_mut(Tensor& t) { return reinterpret_cast<pmd::bf16_t*>(t.data_ptr()); }

// ------------------------------------------------------------------ conv
std::vector<Tensor> conv_weight_prep(Tensor w, int64_t cp, bool want_t) {
  CHECK_DEV(w);
  CHECK_F32(w);
  TORCH_CHECK(w.dim() == 4, "weight must be [K,C,R,S]");
  const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(cp >= C && cp % 8 == 0, "padded channels must be >= C and a multiple of 8");
  c10::DeviceGuard g(w.device());
  Tensor wphys = w.permute({0, 2, 3, 1}).contiguous();  // no-op for channels_last params
  auto opt = w.options().dtype(torch::kBFloat16);
  Tensor wk = torch::empty({K, R, S, cp}, opt);
  Tensor wkt;
  if (want_t) wkt = torch::empty({cp, R, S, K}, opt);
  pmd::conv_weight_prep_launch(wphys.data_ptr<float>(), bfp_mut(wk),
                               want_t ? bfp_mut(wkt) : nullptr, K, R * S, C, (int)cp, cur_stream());
  if (want_t) return {wk, wkt};
  return {wk};
}

// zero-filled tensor on the current stream through the framework's own fill kernel
// (keeps ATen's FillFunctor off the training step)
Tensor pmd_zeros(at::IntArrayRef sizes, const at::TensorOptions& opt) {
  Tensor t = torch::empty(sizes, opt);
  pmd::zero_launch(t.data_ptr(), (long long)t.numel() * t.element_size(), cur_stream());
  return t;
}

// in-place zero of a contiguous GPU tensor (the gradient arena's zero_grad)
Tensor zero_(Tensor t) {
  CHECK_DEV(t);
  CHECK_CONT(t);
  c10::DeviceGuard g(t.device());
  pmd::zero_launch(t.data_ptr(), (long long)t.numel() * t.element_size(), cur_stream());
  return t;
}

float* opt_f32(const c10::optional<Tensor>& t, const char* what) {
  if (!t || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kFloat32 && t->is_contiguous(), what,
              " must be a contiguous fp32 GPU tensor");
  return t->data_ptr<float>();
}

// BatchNorm statistics shift [C] (nullable)
float* shift_ptr(const c10::optional<Tensor>& t, int64_t C) {
  float* p = opt_f32(t, "BN statistics shift");
  if (p) TORCH_CHECK(t->numel() == C, "BN statistics shift must have one value per channel");
  return p;
}

// stats_buf: optional pre-zeroed [S,2,K] slot buffer (pool); allocated zeroed otherwise
// out_h/out_w < 0: the usual (H + 2 pad - R) / stride + 1; otherwise an explicit
// (cropped) output extent -- the space-to-depth stem's 4x4 conv pads 2 rows on
// the top but only 1 at the bottom, i.e. the last full-pad output row is dropped
// shift: optional fp32 [K] BatchNorm statistics shift (the stats are taken about it, bn_moments)
static std::vector<Tensor> conv_fwd_impl(Tensor x, Tensor wk, int64_t stride, int64_t pad, bool want_stats,
                                         c10::optional<Tensor> stats_buf, int64_t out_h, int64_t out_w,
                                         const c10::optional<Tensor>& shift, bool store = true) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  CHECK_DEV(wk); CHECK_BF16(wk); CHECK_CONT(wk);
  TORCH_CHECK(x.dim() == 4 && wk.dim() == 4, "x [N,H,W,C], wk [K,R,S,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = wk.size(0), R = wk.size(1), S = wk.size(2);
  TORCH_CHECK(wk.size(3) == C, "channel mismatch: x has ", C, ", weight has ", wk.size(3));
  const int Pf = (H + 2 * pad - R) / stride + 1, Qf = (W + 2 * pad - S) / stride + 1;
  const int P = out_h < 0 ? Pf : (int)out_h, Q = out_w < 0 ? Qf : (int)out_w;
  TORCH_CHECK(P >= 1 && Q >= 1 && P <= Pf && Q <= Qf, "conv_fwd: output extent beyond the padded input");
  c10::DeviceGuard g(x.device());
  TORCH_CHECK(store || want_stats, "a forward without its output must take statistics");
  Tensor y = store ? torch::empty({N, P, Q, K}, x.options()) : Tensor();
  Tensor stats;
  if (want_stats) {
    if (stats_buf && stats_buf->defined()) {
      TORCH_CHECK(stats_buf->numel() == pmd_slots() * 2 * K, "stats buffer must be [S,2,K]");
      opt_f32(stats_buf, "stats_buf");
      stats = *stats_buf;
    } else {
      stats = pmd_zeros({pmd_slots(), 2, K}, x.options().dtype(torch::kFloat32));
    }
  }
  const float* shp = shift_ptr(shift, K);
  const int rc = pmd::conv_igemm_launch(bfp(x), bfp(wk), store ? bfp_mut(y) : nullptr,
                                        want_stats ? stats.data_ptr<float>() : nullptr, N, H, W, C, P,
                                        Q, K, R, S, (int)stride, (int)pad, false, nullptr, nullptr, nullptr,
                                        cur_stream(), shp);
  CHECK_RC(rc, "conv_fwd");
  if (!store) return {stats};
  if (want_stats) return {y, stats};
  return {y};
}

std::vector<Tensor> conv_fwd(Tensor x, Tensor wk, int64_t stride, int64_t pad, bool want_stats,
                             c10::optional<Tensor> stats_buf, c10::optional<Tensor> shift) {
  return conv_fwd_impl(x, wk, stride, pad, want_stats, stats_buf, -1, -1, shift);
}

std::vector<Tensor> conv_fwd_hw(Tensor x, Tensor wk, int64_t stride, int64_t pad, int64_t out_h,
                                int64_t out_w, bool want_stats, c10::optional<Tensor> stats_buf,
                                c10::optional<Tensor> shift) {
  return conv_fwd_impl(x, wk, stride, pad, want_stats, stats_buf, out_h, out_w, shift);
}

// ----------------------------------------------------------- s2d stem
Tensor stem_s2d_input(Tensor x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 8, "stem input must be [N,H,W,8] (3 channels zero-padded)");
  TORCH_CHECK(x.size(1) % 2 == 0 && x.size(2) % 2 == 0, "space-to-depth needs even H, W");
  c10::DeviceGuard g(x.device());
  Tensor xs = torch::empty({x.size(0), x.size(1) / 2, x.size(2) / 2, 16}, x.options());
  CHECK_RC(pmd::stem_s2d_input_launch(bfp(x), bfp_mut(xs), x.size(0), x.size(1), x.size(2), cur_stream()),
           "stem_s2d_input");
  return xs;
}

Tensor stem_s2d_weight(Tensor w) {
  CHECK_DEV(w); CHECK_F32(w);
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 7 && w.size(3) == 7 && w.size(1) <= 4, "w must be [K,C<=4,7,7]");
  const int K = w.size(0), C = w.size(1);
  c10::DeviceGuard g(w.device());
  Tensor wphys = w.permute({0, 2, 3, 1}).contiguous();  // no-op for channels_last params
  Tensor ws = torch::empty({K, 4, 4, 16}, w.options().dtype(torch::kBFloat16));
  CHECK_RC(pmd::stem_s2d_weight_launch(wphys.data_ptr<float>(), bfp_mut(ws), K, C, cur_stream()),
           "stem_s2d_weight");
  return ws;
}

// dws [K,4,4,16] -> dw [K,7,7,C]; with `out` (a contiguous [K,7,7,C] fp32 view,
// e.g. the gradient arena) the folded gradient is accumulated into it
Tensor stem_s2d_wgrad_fold(Tensor dws, int64_t C, c10::optional<Tensor> out) {
  CHECK_DEV(dws); CHECK_F32(dws); CHECK_CONT(dws);
  TORCH_CHECK(dws.dim() == 4 && dws.size(1) == 4 && dws.size(2) == 4 && dws.size(3) == 16, "dws [K,4,4,16]");
  TORCH_CHECK(C >= 1 && C <= 4, "C <= 4");
  const int K = dws.size(0);
  c10::DeviceGuard g(dws.device());
  Tensor dw;
  const bool acc = out && out->defined();
  if (acc) {
    TORCH_CHECK(out->sizes() == torch::IntArrayRef({K, 7, 7, C}) && out->is_contiguous(), "fold out [K,7,7,C]");
    opt_f32(out, "fold out");
    dw = *out;
  } else {
    dw = torch::empty({K, 7, 7, C}, dws.options());
  }
  CHECK_RC(pmd::stem_s2d_wgrad_fold_launch(dws.data_ptr<float>(), dw.data_ptr<float>(), K, (int)C, acc,
                                           cur_stream()),
           "stem_s2d_wgrad_fold");
  return dw;
}

// ------------------------------------------------------------- winograd
// F(2x2,3x3) for stride-1 pad-1 3x3 convs: U = filter transform of the forward
// weight image wk [K,3,3,Cp] (flip: the dgrad filter, [16,Cp,K]); the 16 GEMMs
// between the input and output transforms are winograd_gemm below.
Tensor winograd_filter(Tensor wk, bool flip) {
  CHECK_DEV(wk); CHECK_BF16(wk); CHECK_CONT(wk);
  TORCH_CHECK(wk.dim() == 4 && wk.size(1) == 3 && wk.size(2) == 3, "wk must be [K,3,3,Cp]");
  const int K = wk.size(0), Cp = wk.size(3);
  c10::DeviceGuard g(wk.device());
  Tensor U = flip ? torch::empty({16, Cp, K}, wk.options()) : torch::empty({16, K, Cp}, wk.options());
  CHECK_RC(pmd::winograd_filter_launch(bfp(wk), bfp_mut(U), K, Cp, flip, cur_stream()), "winograd_filter");
  return U;
}

Tensor winograd_input(Tensor x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  TORCH_CHECK(x.dim() == 4, "x must be [N,H,W,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t T = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2);
  c10::DeviceGuard g(x.device());
  Tensor V = torch::empty({16, T, C}, x.options());
  CHECK_RC(pmd::winograd_input_launch(bfp(x), bfp_mut(V), N, H, W, C, cur_stream()), "winograd_input");
  return V;
}

// The 16 transformed-domain products M[b] = V[b] . U[b]^T ([T,C] x [K,C] -> [T,K]):
// each is a 1x1 stride-1 "convolution" of T pixels with C channels by the K x C
// filter slice U[b], so all 16 run as ONE batched launch (grid.z) of the implicit-GEMM
// MFMA kernel (LDS-DMA ring, per-shape autotuned tile) -- no library GEMM.
Tensor winograd_gemm(Tensor V, Tensor U) {
  CHECK_DEV(V); CHECK_BF16(V); CHECK_CONT(V);
  CHECK_DEV(U); CHECK_BF16(U); CHECK_CONT(U);
  TORCH_CHECK(V.dim() == 3 && U.dim() == 3 && V.size(0) == 16 && U.size(0) == 16 && V.size(2) == U.size(2),
              "winograd_gemm: V [16,T,C], U [16,K,C]");
  TORCH_CHECK(V.size(1) < (int64_t)1 << 31, "winograd_gemm: too many tiles");
  const int T = V.size(1), C = V.size(2), K = U.size(1);
  c10::DeviceGuard g(V.device());
  Tensor M = torch::empty({16, T, K}, V.options());
  const pmd::bf16_t* v = bfp(V);
  const pmd::bf16_t* u = bfp(U);
  pmd::bf16_t* m = bfp_mut(M);
  CHECK_RC(pmd::conv_igemm_batched_launch(v, u, m, 16, (long long)T * C, (long long)K * C, (long long)T * K, 1, T, 1,
                                          C, T, 1, K, 1, 1, 1, 0, cur_stream()),
           "winograd_gemm");
  return M;
}

std::vector<Tensor> winograd_output(Tensor M, int64_t N, int64_t H, int64_t W, bool want_stats,
                                    c10::optional<Tensor> stats_buf, c10::optional<Tensor> shift) {
  CHECK_DEV(M); CHECK_BF16(M); CHECK_CONT(M);
  const int64_t T = N * ((H + 1) / 2) * ((W + 1) / 2);
  TORCH_CHECK(M.dim() == 3 && M.size(0) == 16 && M.size(1) == T, "M must be [16, tiles, K]");
  const int K = M.size(2);
  c10::DeviceGuard g(M.device());
  Tensor y = torch::empty({N, H, W, K}, M.options());
  Tensor stats;
  if (want_stats) {
    if (stats_buf && stats_buf->defined()) {
      TORCH_CHECK(stats_buf->numel() == pmd_slots() * 2 * K, "stats buffer must be [S,2,K]");
      opt_f32(stats_buf, "stats_buf");
      stats = *stats_buf;
    } else {
      stats = pmd_zeros({pmd_slots(), 2, K}, M.options().dtype(torch::kFloat32));
    }
  }
  CHECK_RC(pmd::winograd_output_launch(bfp(M), bfp_mut(y), want_stats ? stats.data_ptr<float>() : nullptr,
                                       (int)N, (int)H, (int)W, K, cur_stream(), shift_ptr(shift, K)),
           "winograd_output");
  if (want_stats) return {y, stats};
  return {y};
}

// fused Winograd forward: y [N,H,W,K] (+ [S,2,K] BN statistics about `shift`) from x [N,H,W,C] and the
// transformed filter U [16,K,C] (winograd_filter) in ONE kernel (kernels/winograd.hip)
std::vector<Tensor> winograd_fused_fwd(Tensor x, Tensor U, bool want_stats, c10::optional<Tensor> stats_buf,
                                       c10::optional<Tensor> shift) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  CHECK_DEV(U); CHECK_BF16(U); CHECK_CONT(U);
  TORCH_CHECK(x.dim() == 4 && U.dim() == 3 && U.size(0) == 16 && U.size(2) == x.size(3),
              "winograd_fused_fwd: x [N,H,W,C], U [16,K,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), K = U.size(1);
  c10::DeviceGuard g(x.device());
  Tensor y = torch::empty({N, H, W, K}, x.options());
  Tensor stats;
  if (want_stats) {
    if (stats_buf && stats_buf->defined()) {
      TORCH_CHECK(stats_buf->numel() == pmd_slots() * 2 * K, "stats buffer must be [S,2,K]");
      opt_f32(stats_buf, "stats_buf");
      stats = *stats_buf;
    } else {
      stats = pmd_zeros({pmd_slots(), 2, K}, x.options().dtype(torch::kFloat32));
    }
  }
  CHECK_RC(pmd::winograd_fused_fwd_launch(bfp(x), bfp(U), bfp_mut(y), want_stats ? stats.data_ptr<float>() : nullptr,
                                          want_stats ? shift_ptr(shift, K) : nullptr, N, H, W, C, K, cur_stream()),
           "winograd_fused_fwd");
  if (want_stats) return {y, stats};
  return {y};
}

// dx[N,H,W,Cp] from dy[N,P,Q,K] and wkt[Cp,R,S,K]
// addend: optional [N,H,W,Cp] bf16 added in the epilogue (dx = dgrad + addend)
// bn_*: optional fused BN-backward reduce of the output (see pmd::BnReduceArgs);
// bn_red* are [kStatSlots, 2, C] fp32 slot buffers that receive += the sums.
Tensor conv_dgrad(Tensor dy, Tensor wkt, int64_t H, int64_t W, int64_t stride, int64_t pad,
                  c10::optional<Tensor> addend, c10::optional<Tensor> bn_mask,
                  c10::optional<Tensor> bn_y0, c10::optional<Tensor> bn_p0,
                  c10::optional<Tensor> bn_red0, c10::optional<Tensor> bn_y1,
                  c10::optional<Tensor> bn_p1, c10::optional<Tensor> bn_red1,
                  c10::optional<Tensor> addend_mask, c10::optional<Tensor> addend_bias) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONT(dy);
  CHECK_DEV(wkt); CHECK_BF16(wkt); CHECK_CONT(wkt);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  const int Cp = wkt.size(0), R = wkt.size(1), S = wkt.size(2);
  TORCH_CHECK(wkt.size(3) == K, "dgrad weight/K mismatch");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == P && (W + 2 * pad - S) / stride + 1 == Q,
              "dgrad spatial mismatch");
  c10::DeviceGuard g(dy.device());
  Tensor dx = torch::empty({N, H, W, Cp}, dy.options());
  const pmd::bf16_t* add = nullptr;
  if (addend && addend->defined()) {
    CHECK_BF16(*addend); CHECK_CONT(*addend);
    TORCH_CHECK(addend->sizes() == dx.sizes(), "addend shape");
    add = bfp(*addend);
  }
  const uint8_t* amask = nullptr;
  if (addend_mask && addend_mask->defined()) {
    TORCH_CHECK(add, "addend_mask needs an addend");
    TORCH_CHECK(addend_mask->scalar_type() == torch::kUInt8 && addend_mask->is_contiguous() &&
                addend_mask->numel() == dx.numel() / 8, "addend_mask must be uint8 [M, C/8]");
    amask = addend_mask->data_ptr<uint8_t>();
  }
  pmd::BnReduceArgs bnr{};
  const bool fused = bn_red0 && bn_red0->defined();
  if (fused) {
    auto chk_set = [&](const c10::optional<Tensor>& y, const c10::optional<Tensor>& p,
                       const c10::optional<Tensor>& r, int t) {
      // y may be None: a sum-only reduce (row 1 = -mean * invstd * sum dz), see conv_igemm.hip
      TORCH_CHECK(p && p->defined() && r && r->defined(), "bn reduce set incomplete");
      CHECK_F32(*p); CHECK_F32(*r); CHECK_CONT(*r); CHECK_CONT(*p);
      if (y && y->defined()) {
        CHECK_BF16(*y); CHECK_CONT(*y);
        TORCH_CHECK(y->sizes() == dx.sizes(), "bn reduce: y must match dx");
      }
      TORCH_CHECK(p->numel() == 4 * Cp, "bn reduce: params must be [4, C]");
      TORCH_CHECK(r->numel() == pmd_slots() * 2 * Cp, "bn reduce: red must be [slots, 2, C]");
      bnr.y[t] = (y && y->defined()) ? bfp(*y) : nullptr;
      bnr.p[t] = p->data_ptr<float>();
      bnr.red[t] = r->data_ptr<float>();
    };
    chk_set(bn_y0, bn_p0, bn_red0, 0);
    if (bn_red1 && bn_red1->defined()) chk_set(bn_y1, bn_p1, bn_red1, 1);
    if (bn_mask && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == torch::kUInt8 && bn_mask->is_contiguous() &&
                  bn_mask->numel() == dx.numel() / 8, "bn reduce: mask must be uint8 [M, C/8]");
      bnr.mask = bn_mask->data_ptr<uint8_t>();
    }
  }
  const float* abias = nullptr;
  if (addend_bias && addend_bias->defined()) {
    TORCH_CHECK(add, "addend_bias needs an addend");
    CHECK_DEV(*addend_bias); CHECK_F32(*addend_bias); CHECK_CONT(*addend_bias);
    TORCH_CHECK(addend_bias->numel() == Cp, "addend_bias must be fp32 [C]");
    abias = addend_bias->data_ptr<float>();
  }
  // the gathered operand is dy (spatial P x Q, K channels); output spatial is H x W
  pmd::conv_set_addend_bias(abias);
  const int rc = pmd::conv_igemm_launch(bfp(dy), bfp(wkt), bfp_mut(dx), nullptr, N, P, Q, K, (int)H,
                                        (int)W, Cp, R, S, (int)stride, (int)pad, true, add, amask,
                                        fused ? &bnr : nullptr, cur_stream(), nullptr);
  pmd::conv_set_addend_bias(nullptr);
  CHECK_RC(rc, "conv_dgrad");
  return dx;
}

// FP8 dgrad: dx[N,H,W,Cp] (bf16) from e5m2 dyq[N,P,Q,K] (scale sdy) and the e4m3 transposed
// weight image wtq[Cp,R,S,K] (scale sw); addend / fused BN reduce as conv_dgrad
Tensor conv_dgrad_fp8(Tensor dyq, Tensor wtq, Tensor sdy, Tensor sw, int64_t H, int64_t W, int64_t stride,
                      int64_t pad, c10::optional<Tensor> addend, c10::optional<Tensor> bn_mask,
                      c10::optional<Tensor> bn_y0, c10::optional<Tensor> bn_p0, c10::optional<Tensor> bn_red0,
                      c10::optional<Tensor> bn_y1, c10::optional<Tensor> bn_p1, c10::optional<Tensor> bn_red1,
                      c10::optional<Tensor> addend_mask) {
  CHECK_DEV(dyq); CHECK_CONT(dyq); CHECK_DEV(wtq); CHECK_CONT(wtq);
  TORCH_CHECK(dyq.scalar_type() == torch::kUInt8 && wtq.scalar_type() == torch::kUInt8,
              "conv_dgrad_fp8: e5m2 dY / e4m3 weight image as uint8");
  CHECK_F32(sdy); CHECK_F32(sw);
  const int N = dyq.size(0), P = dyq.size(1), Q = dyq.size(2), K = dyq.size(3);
  const int Cp = wtq.size(0), R = wtq.size(1), S = wtq.size(2);
  TORCH_CHECK(wtq.size(3) == K, "dgrad weight/K mismatch");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == P && (W + 2 * pad - S) / stride + 1 == Q,
              "dgrad spatial mismatch");
  c10::DeviceGuard g(dyq.device());
  Tensor dx = torch::empty({N, H, W, Cp}, dyq.options().dtype(torch::kBFloat16));
  const pmd::bf16_t* add = nullptr;
  if (addend && addend->defined()) {
    CHECK_BF16(*addend); CHECK_CONT(*addend);
    TORCH_CHECK(addend->sizes() == dx.sizes(), "addend shape");
    add = bfp(*addend);
  }
  const uint8_t* amask = nullptr;
  if (addend_mask && addend_mask->defined()) {
    TORCH_CHECK(add, "addend_mask needs an addend");
    TORCH_CHECK(addend_mask->scalar_type() == torch::kUInt8 && addend_mask->is_contiguous() &&
                addend_mask->numel() == dx.numel() / 8, "addend_mask must be uint8 [M, C/8]");
    amask = addend_mask->data_ptr<uint8_t>();
  }
  pmd::BnReduceArgs bnr{};
  const bool fused = bn_red0 && bn_red0->defined();
  if (fused) {
    auto chk_set = [&](const c10::optional<Tensor>& y, const c10::optional<Tensor>& p,
                       const c10::optional<Tensor>& r, int t) {
      // y may be None: a sum-only reduce (row 1 = -mean * invstd * sum dz), see conv_igemm.hip
      TORCH_CHECK(p && p->defined() && r && r->defined(), "bn reduce set incomplete");
      CHECK_F32(*p); CHECK_F32(*r); CHECK_CONT(*r); CHECK_CONT(*p);
      if (y && y->defined()) {
        CHECK_BF16(*y); CHECK_CONT(*y);
        TORCH_CHECK(y->sizes() == dx.sizes(), "bn reduce: y must match dx");
      }
      TORCH_CHECK(p->numel() == 4 * Cp, "bn reduce: params must be [4, C]");
      TORCH_CHECK(r->numel() == pmd_slots() * 2 * Cp, "bn reduce: red must be [slots, 2, C]");
      bnr.y[t] = (y && y->defined()) ? bfp(*y) : nullptr;
      bnr.p[t] = p->data_ptr<float>();
      bnr.red[t] = r->data_ptr<float>();
    };
    chk_set(bn_y0, bn_p0, bn_red0, 0);
    if (bn_red1 && bn_red1->defined()) chk_set(bn_y1, bn_p1, bn_red1, 1);
    if (bn_mask && bn_mask->defined()) {
      TORCH_CHECK(bn_mask->scalar_type() == torch::kUInt8 && bn_mask->is_contiguous() &&
                  bn_mask->numel() == dx.numel() / 8, "bn reduce: mask must be uint8 [M, C/8]");
      bnr.mask = bn_mask->data_ptr<uint8_t>();
    }
  }
  const int rc = pmd::conv_dgrad_fp8_launch(dyq.data_ptr<uint8_t>(), wtq.data_ptr<uint8_t>(), sdy.data_ptr<float>(),
                                            sw.data_ptr<float>(), bfp_mut(dx), N, P, Q, K, (int)H, (int)W, Cp, R, S,
                                            (int)stride, (int)pad, add, amask, fused ? &bnr : nullptr,
                                            cur_stream());
  CHECK_RC(rc, "conv_dgrad_fp8");
  return dx;
}

// split-K workspaces of the reductions queued in deferred mode (pmd::wgrad_set_defer): kept
// alive until wgrad_flush has launched the grouped reduction that reads them (stream-ordered
// on the same stream, so the caching allocator may recycle them right after)
static thread_local std::vector<Tensor> t_ws_keep;
static void keep_ws(const Tensor& ws) {
  if (pmd::wgrad_defer() && ws.defined()) t_ws_keep.push_back(ws);
}
void wgrad_flush() {
  const int rc = pmd::wgrad_flush(cur_stream());
  TORCH_CHECK(rc == 0, "wgrad_flush: the queued split reductions belong to another stream");
  t_ws_keep.clear();
}

// out: optional [K,R,S,C] fp32 accumulation target (e.g. a grad-arena view); dW is ADDED to it
Tensor conv_wgrad(Tensor dy, Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                  c10::optional<Tensor> out) {
  CHECK_DEV(dy); CHECK_BF16(dy); CHECK_CONT(dy);
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  TORCH_CHECK(dy.size(0) == N, "batch mismatch");
  // P, Q may crop the last rows/cols of the padded extent (s2d stem, see conv_fwd_hw)
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 >= P && (W + 2 * pad - S) / stride + 1 >= Q && P >= 1 && Q >= 1,
              "wgrad spatial mismatch");
  c10::DeviceGuard g(x.device());
  Tensor dw;
  if (out && out->defined()) {
    TORCH_CHECK(out->sizes() == torch::IntArrayRef({K, R, S, C}), "wgrad out shape");
    opt_f32(out, "wgrad out");
    dw = *out;
  } else {
    dw = pmd_zeros({K, R, S, C}, x.options().dtype(torch::kFloat32));
  }
  const int splits = pmd::conv_wgrad_splits(N, H, W, C, P, Q, K, (int)R, (int)S, (int)stride,
                                            (int)pad);
  Tensor ws;
  if (splits > 1) ws = torch::empty({splits, K, R * S * C}, x.options().dtype(torch::kFloat32));
  const int rc = pmd::conv_wgrad_launch(bfp(dy), bfp(x), dw.data_ptr<float>(),
                                        splits > 1 ? ws.data_ptr<float>() : nullptr, N, H, W, C, P, Q,
                                        K, (int)R, (int)S, (int)stride, (int)pad, cur_stream());
  CHECK_RC(rc, "conv_wgrad");
  keep_ws(ws);
  return dw;
}

// ---- linear-BN backward (kernels/bnlin.hip, ops/functional.py _bnlin_final)
static void chk_wk(const Tensor& wk) {
  CHECK_DEV(wk); CHECK_BF16(wk); CHECK_CONT(wk);
  TORCH_CHECK(wk.dim() == 4 && wk.size(1) == 1 && wk.size(2) == 1, "bnlin: 1x1 weight image [K,1,1,Cp]");
}
static void chk_kc(const Tensor& t, int64_t K, int64_t C, const char* what) {
  CHECK_DEV(t); CHECK_F32(t);
  TORCH_CHECK(t.numel() == K * C && t.stride(-1) == 1 && (t.dim() < 2 || t.stride(0) == C), what,
              ": fp32 [K][C] rows expected");
}

std::vector<Tensor> bnlin_coeff(Tensor red, c10::optional<Tensor> count, double count_h, Tensor gamma, Tensor params,
                                Tensor wk, int64_t C) {
  chk_wk(wk);
  const int K = wk.size(0), Cp = wk.size(3);
  CHECK_DEV(red); CHECK_F32(red); CHECK_CONT(red); CHECK_F32(gamma); CHECK_CONT(gamma);
  CHECK_F32(params); CHECK_CONT(params);
  TORCH_CHECK(red.numel() == 2 * K && gamma.numel() == K && params.numel() == 4 * K && C <= Cp,
              "bnlin_coeff: shapes");
  const float* cnt = nullptr;
  if (count && count->defined()) { CHECK_F32(*count); cnt = count->data_ptr<float>(); }
  c10::DeviceGuard g(wk.device());
  Tensor gm = torch::empty({C, 1, 1, C}, wk.options());
  Tensor bias = torch::empty({C}, wk.options().dtype(torch::kFloat32));
  Tensor abc = torch::empty({3, K}, wk.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::bnlin_coeff_launch(red.data_ptr<float>(), cnt, (float)count_h, gamma.data_ptr<float>(),
                                   params.data_ptr<float>(), bfp(wk), bfp_mut(gm), bias.data_ptr<float>(),
                                   abc.data_ptr<float>(), K, (int)C, Cp, cur_stream()),
           "bnlin_coeff");
  return {gm, bias, abc};
}

Tensor bnlin_dimg(Tensor gamma, Tensor params, Tensor wk, int64_t C) {
  chk_wk(wk);
  const int K = wk.size(0), Cp = wk.size(3);
  CHECK_F32(gamma); CHECK_CONT(gamma); CHECK_F32(params); CHECK_CONT(params);
  TORCH_CHECK(gamma.numel() == K && params.numel() == 4 * K && C <= Cp, "bnlin_dimg: shapes");
  c10::DeviceGuard g(wk.device());
  Tensor wkt_a = torch::empty({C, 1, 1, K}, wk.options());
  CHECK_RC(pmd::bnlin_dimg_launch(gamma.data_ptr<float>(), params.data_ptr<float>(), bfp(wk), bfp_mut(wkt_a), K,
                                  (int)C, Cp, cur_stream()),
           "bnlin_dimg");
  return wkt_a;
}

Tensor colsum(Tensor x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  const int C = x.size(-1);
  c10::DeviceGuard g(x.device());
  Tensor out = pmd_zeros({C}, x.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::colsum_launch(bfp(x), out.data_ptr<float>(), x.numel() / C, C, cur_stream()), "colsum");
  return out;
}

void bnlin_wgrad(Tensor out, Tensor abc, Tensor T, Tensor wk, Tensor gz, Tensor cs) {
  chk_wk(wk);
  const int K = wk.size(0), Cp = wk.size(3);
  const int C = T.numel() / K;
  chk_kc(T, K, C, "bnlin_wgrad T");
  chk_kc(out, K, C, "bnlin_wgrad out");
  chk_kc(gz, C, C, "bnlin_wgrad gz");
  CHECK_F32(abc); CHECK_CONT(abc); CHECK_F32(cs); CHECK_CONT(cs);
  TORCH_CHECK(abc.numel() == 3 * K && cs.numel() == C, "bnlin_wgrad: abc / colsum");
  c10::DeviceGuard g(wk.device());
  CHECK_RC(pmd::bnlin_wgrad_launch(out.data_ptr<float>(), abc.data_ptr<float>(), T.data_ptr<float>(), bfp(wk),
                                   gz.data_ptr<float>(), cs.data_ptr<float>(), K, C, Cp, cur_stream()),
           "bnlin_wgrad");
}

// FP8 weight gradient: dyq e5m2 [N,P,Q,K] (scale sdy) x xq e4m3 [N,H,W,C] (scale sx);
// dW / (sdy * sx) is ADDED to out ([K,R,S,C] fp32) when given
Tensor conv_wgrad_fp8(Tensor dyq, Tensor xq, Tensor sdy, Tensor sx, int64_t R, int64_t S, int64_t stride,
                      int64_t pad, c10::optional<Tensor> out) {
  CHECK_DEV(dyq); CHECK_CONT(dyq); CHECK_DEV(xq); CHECK_CONT(xq);
  TORCH_CHECK(dyq.scalar_type() == torch::kUInt8 && xq.scalar_type() == torch::kUInt8,
              "conv_wgrad_fp8: e5m2 / e4m3 operands as uint8");
  CHECK_F32(sdy); CHECK_F32(sx);
  const int N = xq.size(0), H = xq.size(1), W = xq.size(2), C = xq.size(3);
  const int P = dyq.size(1), Q = dyq.size(2), K = dyq.size(3);
  TORCH_CHECK(dyq.size(0) == N, "batch mismatch");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 >= P && (W + 2 * pad - S) / stride + 1 >= Q && P >= 1 && Q >= 1,
              "wgrad spatial mismatch");
  c10::DeviceGuard g(xq.device());
  Tensor dw;
  if (out && out->defined()) {
    TORCH_CHECK(out->sizes() == torch::IntArrayRef({K, R, S, C}), "wgrad out shape");
    opt_f32(out, "wgrad out");
    dw = *out;
  } else {
    dw = pmd_zeros({K, R, S, C}, xq.options().dtype(torch::kFloat32));
  }
  const int splits = pmd::conv_wgrad_fp8_splits(N, H, W, C, P, Q, K, (int)R, (int)S, (int)stride, (int)pad);
  Tensor ws;
  if (splits > 1) ws = torch::empty({splits, K, R * S * C}, xq.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::conv_wgrad_fp8_launch(dyq.data_ptr<uint8_t>(), xq.data_ptr<uint8_t>(), sdy.data_ptr<float>(),
                                      sx.data_ptr<float>(), dw.data_ptr<float>(),
                                      splits > 1 ? ws.data_ptr<float>() : nullptr, N, H, W, C, P, Q, K, (int)R,
                                      (int)S, (int)stride, (int)pad, cur_stream()),
           "conv_wgrad_fp8");
  keep_ws(ws);
  return dw;
}

// -------------------------------------------------------------------- BN
Tensor bn_finalize(c10::optional<Tensor> sums, c10::optional<Tensor> count, Tensor gamma, Tensor beta, double eps,
                   c10::optional<Tensor> rm, c10::optional<Tensor> rv, double momentum,
                   c10::optional<Tensor> nbt, bool eval_mode, c10::optional<Tensor> shift) {
  CHECK_DEV(gamma); CHECK_F32(gamma);
  const int C = gamma.numel();
  c10::DeviceGuard g(gamma.device());
  Tensor params = torch::empty({4, C}, gamma.options());
  float* rmp = nullptr;
  float* rvp = nullptr;
  long long* nb = nullptr;
  if (rm && rm->defined()) { CHECK_F32(*rm); CHECK_CONT(*rm); rmp = rm->data_ptr<float>(); }
  if (rv && rv->defined()) { CHECK_F32(*rv); CHECK_CONT(*rv); rvp = rv->data_ptr<float>(); }
  if (nbt && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == torch::kInt64 && nbt->is_cuda(), "nbt int64 GPU");
    nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  }
  if (eval_mode) TORCH_CHECK(rmp && rvp, "eval BN needs running stats");
  if (!eval_mode) TORCH_CHECK(sums && sums->defined() && count && count->defined(), "train BN needs sums");
  Tensor s = eval_mode ? gamma : sums->contiguous();
  Tensor cnt = eval_mode ? gamma : count->contiguous();
  Tensor gm = gamma.contiguous(), bt = beta.contiguous();
  pmd::bn_finalize_launch(eval_mode ? nullptr : s.data_ptr<float>(),
                          eval_mode ? nullptr : cnt.data_ptr<float>(), gm.data_ptr<float>(),
                          bt.data_ptr<float>(), params.data_ptr<float>(), rmp, rvp, nb,
                          eval_mode ? nullptr : shift_ptr(shift, C), C, (float)eps, (float)momentum,
                          eval_mode, cur_stream());
  return params;
}

// slot-stats [S,2,Ca] (+ [S,2,Cb]) -> flat [2Ca (+2Cb) (+1 count)]; clear: zero the
// slot buffers after reading; acc_*: optional d_beta/d_gamma targets that get += the sums
Tensor stats_collapse(Tensor a, c10::optional<Tensor> b, c10::optional<double> count, bool clear,
                      c10::optional<Tensor> acc_a0, c10::optional<Tensor> acc_a1,
                      c10::optional<Tensor> acc_b0, c10::optional<Tensor> acc_b1) {
  CHECK_DEV(a); CHECK_F32(a); CHECK_CONT(a);
  TORCH_CHECK(a.dim() == 3 && a.size(0) == pmd_slots() && a.size(1) == 2, "slot stats [S,2,C]");
  const int Ca = a.size(2);
  int Cb = 0;
  float* bp = nullptr;
  if (b && b->defined()) {
    CHECK_F32(*b); CHECK_CONT(*b);
    TORCH_CHECK(b->dim() == 3 && b->size(0) == pmd_slots(), "slot stats [S,2,C]");
    Cb = b->size(2);
    bp = b->data_ptr<float>();
  }
  auto chk = [&](const c10::optional<Tensor>& t, int C) {
    float* p = opt_f32(t, "grad target");
    if (p) TORCH_CHECK(t->numel() == C, "grad target size");
    return p;
  };
  const bool wc = count.has_value();
  c10::DeviceGuard g(a.device());
  Tensor out = torch::empty({2 * Ca + 2 * Cb + (wc ? 1 : 0)}, a.options());
  pmd::stats_collapse_launch(a.data_ptr<float>(), Ca, bp, Cb, wc ? (float)*count : 0.f,
                             out.data_ptr<float>(), wc, clear, chk(acc_a0, Ca), chk(acc_a1, Ca),
                             chk(acc_b0, Cb), chk(acc_b1, Cb), cur_stream());
  return out;
}

// collapse(+clear) slot stats and finalize BN params in one launch (no all-reduce case)
Tensor stats_finalize_local(Tensor slots, double count, Tensor gamma, Tensor beta, double eps,
                            c10::optional<Tensor> rm, c10::optional<Tensor> rv, double momentum,
                            c10::optional<Tensor> nbt, c10::optional<Tensor> shift) {
  CHECK_DEV(slots); CHECK_F32(slots); CHECK_CONT(slots);
  const int C = gamma.numel();
  TORCH_CHECK(slots.numel() == pmd_slots() * 2 * C, "slot stats [S,2,C]");
  c10::DeviceGuard g(slots.device());
  Tensor params = torch::empty({4, C}, gamma.options());
  long long* nb = nullptr;
  if (nbt && nbt->defined()) nb = reinterpret_cast<long long*>(nbt->data_ptr<int64_t>());
  Tensor gm = gamma.contiguous(), bt = beta.contiguous();
  pmd::stats_finalize_local_launch(slots.data_ptr<float>(), (float)count, gm.data_ptr<float>(),
                                   bt.data_ptr<float>(), params.data_ptr<float>(), opt_f32(rm, "rm"),
                                   opt_f32(rv, "rv"), nb, shift_ptr(shift, C), C, (float)eps,
                                   (float)momentum, cur_stream());
  return params;
}

// returns {out} or {out, relu_bitmask} (one uint8 per 8-channel chunk) when relu && want_mask
// q8_scale/q8_amax (optional): also return an e4m3 copy of the output (fp8 conv input)
std::vector<Tensor> bn_apply(Tensor y1, Tensor p1, c10::optional<Tensor> res, c10::optional<Tensor> y2,
                             c10::optional<Tensor> p2, bool relu, bool want_mask,
                             c10::optional<Tensor> q8_scale, c10::optional<Tensor> q8_amax, bool q8_only) {
  CHECK_DEV(y1); CHECK_BF16(y1); CHECK_CONT(y1);
  const int C = y1.size(-1);
  const long long M = y1.numel() / C;
  TORCH_CHECK(p1.numel() == 4 * C, "params size");
  int mode = 0;
  const pmd::bf16_t* r = nullptr;
  const float* pp2 = nullptr;
  if (y2 && y2->defined()) {
    CHECK_BF16(*y2); CHECK_CONT(*y2);
    TORCH_CHECK(y2->sizes() == y1.sizes(), "second branch shape");
    TORCH_CHECK(p2 && p2->defined() && p2->numel() == 4 * C, "second branch params");
    mode = 2;
    r = bfp(*y2);
    pp2 = p2->data_ptr<float>();
  } else if (res && res->defined()) {
    CHECK_BF16(*res); CHECK_CONT(*res);
    TORCH_CHECK(res->sizes() == y1.sizes(), "residual shape");
    mode = 1;
    r = bfp(*res);
  }
  c10::DeviceGuard g(y1.device());
  const bool q8 = q8_scale && q8_scale->defined();
  TORCH_CHECK(!q8_only || q8, "q8_only needs the fp8 output");
  // q8_only: the e4m3 copy is the only activation written (returned out is None)
  Tensor out = q8_only ? Tensor() : torch::empty_like(y1);
  Tensor mask;
  const bool wm = relu && want_mask;
  if (wm) mask = torch::empty({M * (C / 8)}, y1.options().dtype(torch::kUInt8));
  Tensor q;
  if (q8) {
    TORCH_CHECK(q8_amax && q8_amax->defined(), "fp8 output needs an amax accumulator");
    CHECK_F32(*q8_scale); CHECK_F32(*q8_amax);
    TORCH_CHECK(q8_amax->numel() >= 64 && q8_amax->is_contiguous(), "amax must be [64] slots");
    q = torch::empty(y1.sizes(), y1.options().dtype(torch::kUInt8));
  }
  const int rc = pmd::bn_apply_launch(bfp(y1), p1.data_ptr<float>(), r, pp2, q8_only ? nullptr : bfp_mut(out),
                                      wm ? mask.data_ptr<uint8_t>() : nullptr, M, C, mode, relu,
                                      q8 ? q.data_ptr<uint8_t>() : nullptr,
                                      q8 ? q8_scale->data_ptr<float>() : nullptr,
                                      q8 ? q8_amax->data_ptr<float>() : nullptr, cur_stream());
  CHECK_RC(rc, "bn_apply");
  std::vector<Tensor> ret{out};
  if (wm) ret.push_back(mask);
  if (q8) ret.push_back(q);
  return ret;
}

const uint8_t* mask_ptr(const c10::optional<Tensor>& mask, long long chunks, bool relu) {
  if (!relu) return nullptr;
  TORCH_CHECK(mask && mask->defined() && mask->scalar_type() == torch::kUInt8 && mask->is_cuda() &&
              mask->is_contiguous() && mask->numel() == chunks, "relu backward needs the uint8 bitmask");
  return mask->data_ptr<uint8_t>();
}

Tensor bn_bwd_reduce(Tensor dout, c10::optional<Tensor> mask, Tensor y, Tensor params, bool relu,
                     c10::optional<Tensor> red_buf) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout);
  CHECK_BF16(y); CHECK_CONT(y);
  const int C = y.size(-1);
  const long long M = y.numel() / C;
  TORCH_CHECK(M < (1ll << 31), "too many rows");
  c10::DeviceGuard g(y.device());
  Tensor red;
  if (red_buf && red_buf->defined()) {
    TORCH_CHECK(red_buf->numel() == pmd_slots() * 2 * C, "reduce buffer must be [S,2,C]");
    opt_f32(red_buf, "red_buf");
    red = *red_buf;
  } else {
    red = pmd_zeros({pmd_slots(), 2, C}, y.options().dtype(torch::kFloat32));
  }
  const int rc = pmd::bn_bwd_reduce_launch(bfp(dout), mask_ptr(mask, M * (C / 8), relu), bfp(y),
                                           params.data_ptr<float>(), red.data_ptr<float>(), (int)M, C,
                                           relu, cur_stream());
  CHECK_RC(rc, "bn_bwd_reduce");
  return red;
}

// count: device scalar (SyncBN global count) or, if absent, count_h from the host
std::vector<Tensor> bn_bwd_elemt(Tensor dout, c10::optional<Tensor> mask, Tensor y, Tensor params,
                                 Tensor gamma, c10::optional<Tensor> red,
                                 c10::optional<Tensor> count, double count_h, bool relu,
                                 bool want_dzm, bool eval_mode, c10::optional<Tensor> q8_scale,
                                 c10::optional<Tensor> q8_amax, bool q8_only) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout);
  const int C = dout.size(-1);
  const long long M = dout.numel() / C;
  c10::DeviceGuard g(dout.device());
  TORCH_CHECK(!q8_only || (q8_scale && q8_scale->defined()), "q8_only needs the e5m2 output");
  // q8_only: only the e5m2 copy is written (returned dy is None)
  Tensor dy = q8_only ? Tensor() : torch::empty_like(dout);
  Tensor dzm;
  if (want_dzm) dzm = torch::empty_like(dout);
  Tensor rr, cc, gm = gamma.contiguous();
  if (!eval_mode) {
    TORCH_CHECK(red && red->defined(), "train backward needs sums");
    CHECK_BF16(y); CHECK_CONT(y);
    rr = red->contiguous();
    if (count && count->defined()) cc = count->contiguous();
  }
  // q8: also the e5m2 copy of dy (scaled by q8_scale, amax into q8_amax) for the fp8 wgrad
  const bool q8 = q8_scale && q8_scale->defined();
  Tensor q;
  if (q8) {
    TORCH_CHECK(!want_dzm && !eval_mode, "e5m2 dY copy: training mode, no dzm");
    TORCH_CHECK(q8_amax && q8_amax->defined() && q8_amax->numel() >= 64 && q8_amax->is_contiguous(),
                "amax must be [64] slots");
    CHECK_F32(*q8_scale); CHECK_F32(*q8_amax);
    q = torch::empty(dout.sizes(), dout.options().dtype(torch::kUInt8));
  }
  const int rc = pmd::bn_bwd_elemt_launch(
      bfp(dout), mask_ptr(mask, M * (C / 8), relu), eval_mode ? nullptr : bfp(y), params.data_ptr<float>(), gm.data_ptr<float>(),
      eval_mode ? nullptr : rr.data_ptr<float>(),
      (eval_mode || !cc.defined()) ? nullptr : cc.data_ptr<float>(), (float)count_h, q8_only ? nullptr : bfp_mut(dy), want_dzm ? bfp_mut(dzm) : nullptr, M, C, relu, eval_mode, cur_stream(),
      q8 ? q.data_ptr<uint8_t>() : nullptr, q8 ? q8_scale->data_ptr<float>() : nullptr,
      q8 ? q8_amax->data_ptr<float>() : nullptr);
  CHECK_RC(rc, "bn_bwd_elemt");
  if (want_dzm) return {dy, dzm};
  if (q8) return {dy, q};
  return {dy};
}

// ----------------------------------------------------------------- pools
std::vector<Tensor> maxpool_fwd(Tensor x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  c10::DeviceGuard g(x.device());
  Tensor out = torch::empty({N, P, Q, C}, x.options());
  Tensor arg = torch::empty({N, P, Q, C}, x.options().dtype(torch::kUInt8));
  CHECK_RC(pmd::maxpool_fwd_launch(bfp(x), bfp_mut(out), arg.data_ptr<uint8_t>(), N, H, W, C, P, Q,
                                   cur_stream()), "maxpool_fwd");
  return {out, arg};
}

Tensor maxpool_bwd(Tensor dout, Tensor arg, int64_t H, int64_t W) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout); CHECK_CONT(arg);
  const int N = dout.size(0), P = dout.size(1), Q = dout.size(2), C = dout.size(3);
  c10::DeviceGuard g(dout.device());
  Tensor dx = torch::empty({N, H, W, C}, dout.options());
  CHECK_RC(pmd::maxpool_bwd_launch(bfp(dout), arg.data_ptr<uint8_t>(), bfp_mut(dx), N, (int)H, (int)W,
                                   C, P, Q, cur_stream()), "maxpool_bwd");
  return dx;
}

// fused stem tail: y (conv1 output) + BN params -> pooled activation + argmax taps
std::vector<Tensor> stem_pool_fwd(Tensor y, Tensor params) {
  CHECK_DEV(y); CHECK_BF16(y); CHECK_CONT(y); CHECK_CONT(params);
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  TORCH_CHECK(params.numel() == 4 * C, "stem_pool_fwd: params [4][C]");
  const int P = (H + 2 - 3) / 2 + 1, Q = (W + 2 - 3) / 2 + 1;
  c10::DeviceGuard g(y.device());
  Tensor out = torch::empty({N, P, Q, C}, y.options());
  Tensor arg = torch::empty({N, P, Q, C}, y.options().dtype(torch::kUInt8));
  CHECK_RC(pmd::stem_pool_fwd_launch(bfp(y), params.data_ptr<float>(), bfp_mut(out), arg.data_ptr<uint8_t>(),
                                     N, H, W, C, P, Q, cur_stream()), "stem_pool_fwd");
  return {out, arg};
}

// pass 1 of the fused stem backward: sum(dz), sum(dz*xhat) into `red` slots [S][2][C]
Tensor stem_pool_bwd_reduce(Tensor dout, Tensor arg, Tensor y, Tensor params, Tensor red) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout); CHECK_CONT(arg);
  CHECK_BF16(y); CHECK_CONT(y); CHECK_CONT(params); CHECK_CONT(red);
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  const int P = dout.size(1), Q = dout.size(2);
  TORCH_CHECK(dout.size(0) == N && dout.size(3) == C && arg.sizes() == dout.sizes(), "stem_pool_bwd: shapes");
  TORCH_CHECK(red.numel() == 64 * 2 * C && red.scalar_type() == torch::kFloat32, "stem_pool_bwd: slots");
  c10::DeviceGuard g(y.device());
  CHECK_RC(pmd::stem_pool_bwd_reduce_launch(bfp(dout), arg.data_ptr<uint8_t>(), bfp(y), params.data_ptr<float>(),
                                            red.data_ptr<float>(), N, H, W, C, P, Q, cur_stream()),
           "stem_pool_bwd_reduce");
  return red;
}

// pass 2: dy (gradient of the conv1 output)
Tensor stem_pool_bwd_elemt(Tensor dout, Tensor arg, Tensor y, Tensor params, Tensor gamma,
                           c10::optional<Tensor> red, c10::optional<Tensor> count, double count_h,
                           bool eval_mode) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout); CHECK_CONT(arg);
  CHECK_BF16(y); CHECK_CONT(y); CHECK_CONT(params);
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  const int P = dout.size(1), Q = dout.size(2);
  TORCH_CHECK(dout.size(0) == N && dout.size(3) == C && arg.sizes() == dout.sizes(), "stem_pool_bwd: shapes");
  Tensor gm = gamma.contiguous(), rr, cc;
  if (!eval_mode) {
    TORCH_CHECK(red && red->defined() && red->numel() == 2 * C, "stem_pool_bwd: train backward needs [2][C] sums");
    rr = red->contiguous();
    if (count && count->defined()) cc = count->contiguous();
  }
  c10::DeviceGuard g(y.device());
  Tensor dy = torch::empty_like(y);
  CHECK_RC(pmd::stem_pool_bwd_elemt_launch(bfp(dout), arg.data_ptr<uint8_t>(), bfp(y), params.data_ptr<float>(),
                                           gm.data_ptr<float>(), eval_mode ? nullptr : rr.data_ptr<float>(),
                                           cc.defined() ? cc.data_ptr<float>() : nullptr, (float)count_h,
                                           bfp_mut(dy), N, H, W, C, P, Q, eval_mode, cur_stream()),
           "stem_pool_bwd_elemt");
  return dy;
}

// Fused stem backward: the stem conv's weight gradient dws [64,4,4,16] (the space-to-depth
// image's 4x4 conv, fp32) straight from the pooled gradient -- the max-pool + BN(+ReLU)
// backward elementwise pass runs inside the weight-gradient kernel, so dy [N,112,112,64] is never
// materialised (kernels/conv_wgrad.hip stem_wgrad_fused_kernel).  Undefined tensor when the
// geometry is outside the kernel's plan (the caller runs stem_pool_bwd_elemt + conv_wgrad).
Tensor stem_wgrad_fused(Tensor dout, Tensor arg, Tensor y, Tensor params, Tensor gamma, Tensor red,
                        c10::optional<Tensor> count, double count_h, Tensor xs, int64_t pad) {
  CHECK_DEV(dout); CHECK_BF16(dout); CHECK_CONT(dout); CHECK_CONT(arg);
  CHECK_DEV(y); CHECK_BF16(y); CHECK_CONT(y); CHECK_F32(params); CHECK_CONT(params);
  CHECK_DEV(xs); CHECK_BF16(xs); CHECK_CONT(xs);
  const int N = xs.size(0), H = xs.size(1), W = xs.size(2), C = xs.size(3);
  const int P = y.size(1), Q = y.size(2), K = y.size(3), P2 = dout.size(1), Q2 = dout.size(2);
  TORCH_CHECK(y.size(0) == N && dout.size(0) == N && dout.size(3) == K && arg.sizes() == dout.sizes(),
              "stem_wgrad_fused: shapes");
  TORCH_CHECK(params.numel() == 4 * K && red.numel() == 2 * K && gamma.numel() == K, "stem_wgrad_fused: BN sizes");
  Tensor gm = gamma.contiguous().to(torch::kFloat32), rr = red.contiguous(), cc;
  if (count && count->defined()) cc = count->contiguous();
  c10::DeviceGuard g(y.device());
  int splits = 0;
  const int q = pmd::stem_wgrad_fused_launch(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f,
                                             nullptr, nullptr, nullptr, N, H, W, C, P, Q, K, 4, 4, (int)pad, P2, Q2,
                                             &splits, cur_stream());
  if (q != 0) return Tensor();
  Tensor dw = pmd_zeros({K, 4, 4, C}, y.options().dtype(torch::kFloat32));
  Tensor ws;
  if (splits > 1) ws = torch::empty({splits, K, 16 * C}, y.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::stem_wgrad_fused_launch(bfp(dout), arg.data_ptr<uint8_t>(), bfp(y), params.data_ptr<float>(),
                                        gm.data_ptr<float>(), rr.data_ptr<float>(),
                                        cc.defined() ? cc.data_ptr<float>() : nullptr, (float)count_h, bfp(xs),
                                        dw.data_ptr<float>(), splits > 1 ? ws.data_ptr<float>() : nullptr, N, H, W, C,
                                        P, Q, K, 4, 4, (int)pad, P2, Q2, nullptr, cur_stream()),
           "stem_wgrad_fused");
  keep_ws(ws);
  return dw;
}

Tensor avgpool_fwd(Tensor x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x);
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  c10::DeviceGuard g(x.device());
  Tensor out = torch::empty({N, C}, x.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::avgpool_fwd_launch(bfp(x), out.data_ptr<float>(), N, HW, C, cur_stream()), "avgpool");
  return out;
}

Tensor avgpool_bwd(Tensor dout, int64_t H, int64_t W) {
  CHECK_DEV(dout); CHECK_F32(dout); CHECK_CONT(dout);
  const int N = dout.size(0), C = dout.size(1);
  c10::DeviceGuard g(dout.device());
  Tensor dx = torch::empty({N, H, W, C}, dout.options().dtype(torch::kBFloat16));
  CHECK_RC(pmd::avgpool_bwd_launch(dout.data_ptr<float>(), bfp_mut(dx), N, (int)(H * W), C,
                                   cur_stream()), "avgpool_bwd");
  return dx;
}

// ------------------------------------------------------------------ loss
std::vector<Tensor> xent_fwd(Tensor logits, Tensor target) {
  CHECK_DEV(logits); CHECK_F32(logits); CHECK_CONT(logits);
  TORCH_CHECK(target.scalar_type() == torch::kInt64 && target.is_cuda(), "target int64 GPU");
  const int N = logits.size(0), V = logits.size(1);
  c10::DeviceGuard g(logits.device());
  Tensor loss = pmd_zeros({1}, logits.options());
  Tensor lse = torch::empty({N}, logits.options());
  Tensor correct = pmd_zeros({1}, logits.options().dtype(torch::kInt64));
  Tensor tg = target.contiguous();
  CHECK_RC(pmd::xent_fwd_launch(logits.data_ptr<float>(), reinterpret_cast<const long long*>(tg.data_ptr<int64_t>()),
                                loss.data_ptr<float>(), lse.data_ptr<float>(),
                                reinterpret_cast<long long*>(correct.data_ptr<int64_t>()), N, V, cur_stream()),
           "xent_fwd");
  return {loss, lse, correct};
}

Tensor xent_bwd(Tensor logits, Tensor target, Tensor lse, Tensor gloss) {
  CHECK_DEV(logits); CHECK_F32(logits); CHECK_CONT(logits);
  const int N = logits.size(0), V = logits.size(1);
  c10::DeviceGuard g(logits.device());
  Tensor grad = torch::empty_like(logits);
  Tensor tg = target.contiguous(), gl = gloss.to(torch::kFloat32).contiguous();
  pmd::xent_bwd_launch(logits.data_ptr<float>(), reinterpret_cast<const long long*>(tg.data_ptr<int64_t>()),
                       lse.data_ptr<float>(), gl.data_ptr<float>(), grad.data_ptr<float>(), N, V,
                       cur_stream());
  return grad;
}

// ------------------------------------------------------------------ optim
void sgd_(Tensor p, Tensor g, Tensor buf, double lr, double momentum, double wd, double damp,
          bool nesterov, bool first, c10::optional<Tensor> lr_dev) {
  CHECK_DEV(p); CHECK_F32(p); CHECK_CONT(p);
  CHECK_F32(g); CHECK_CONT(g); CHECK_F32(buf); CHECK_CONT(buf);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == buf.numel(), "arena sizes differ");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(p.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(buf.data_ptr()) % 16 == 0, "arenas must be 16-B aligned");
  c10::DeviceGuard gd(p.device());
  pmd::sgd_launch(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(), p.numel(), (float)lr,
                  opt_f32(lr_dev, "lr_dev"), (float)momentum, (float)wd, (float)damp, nesterov, first,
                  cur_stream());
}

// ------------------------------------------------------------------- data
std::vector<Tensor> synth_images(int64_t N, int64_t H, int64_t W, int64_t Cp, int64_t Creal,
                                 int64_t classes, int64_t seed, int64_t device) {
  auto dev = torch::Device(torch::kCUDA, (c10::DeviceIndex)device);
  c10::DeviceGuard g(dev);
  Tensor x = torch::empty({N, H, W, Cp}, torch::TensorOptions().device(dev).dtype(torch::kBFloat16));
  Tensor y = torch::empty({N}, torch::TensorOptions().device(dev).dtype(torch::kInt64));
  CHECK_RC(pmd::synth_images_launch(bfp_mut(x), reinterpret_cast<long long*>(y.data_ptr<int64_t>()), N,
                                    H, W, Cp, Creal, classes, (unsigned long long)seed, cur_stream()),
           "synth_images");
  return {x, y};
}

Tensor cifar_augment(Tensor data, Tensor idx, int64_t Cp, bool train, int64_t pad, int64_t seed,
                     int64_t epoch, bool out_bf16) {
  CHECK_DEV(data); CHECK_CONT(data);
  TORCH_CHECK(data.scalar_type() == torch::kUInt8 && data.dim() == 4 && data.size(1) == 32 &&
              data.size(2) == 32 && data.size(3) == 3, "data must be uint8 [Nd,32,32,3]");
  TORCH_CHECK(idx.scalar_type() == torch::kInt64 && idx.is_cuda(), "idx int64 GPU");
  const int B = idx.numel();
  c10::DeviceGuard g(data.device());
  Tensor out = torch::empty({B, 32, 32, Cp}, data.options().dtype(out_bf16 ? torch::kBFloat16 : torch::kFloat32));
  Tensor ix = idx.contiguous();
  pmd::cifar_augment_launch(data.data_ptr<uint8_t>(), reinterpret_cast<const long long*>(ix.data_ptr<int64_t>()),
                            out.data_ptr(), out_bf16, B, Cp, train, pad, (unsigned long long)seed, epoch,
                            cur_stream());
  return out;
}

// ------------------------------------------------------------------ fp8 (e4m3)
#define CHECK_U8(t) TORCH_CHECK((t).scalar_type() == torch::kUInt8, #t " must be uint8 (e4m3 bytes)")

Tensor quant_bf16_fp8(Tensor x, Tensor scale, c10::optional<Tensor> amax, bool bf8) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONT(x); CHECK_F32(scale);
  TORCH_CHECK(x.numel() % 16 == 0, "quant: numel must be a multiple of 16");
  c10::DeviceGuard g(x.device());
  Tensor q = torch::empty(x.sizes(), x.options().dtype(torch::kUInt8));
  float* am = (amax && amax->defined()) ? amax->data_ptr<float>() : nullptr;
  TORCH_CHECK(!am || (amax->numel() >= 64 && amax->is_contiguous()), "amax must be [64] slots");
  CHECK_RC(pmd::quant_bf16_fp8_launch(bfp(x), q.data_ptr<uint8_t>(), scale.data_ptr<float>(), am,
                                      x.numel(), cur_stream(), bf8), "quant_bf16_fp8");
  return q;
}

std::vector<Tensor> quant_weight_fp8_t(Tensor w, int64_t cp, Tensor scale, c10::optional<Tensor> amax);
Tensor quant_weight_fp8(Tensor w, int64_t cp, Tensor scale, c10::optional<Tensor> amax) {
  return quant_weight_fp8_t(w, cp, scale, amax)[0];
}

// -> [q [K,R,S,cp], qt [cp,R,S,K]]: the forward image and the fp8 dgrad's transposed image
std::vector<Tensor> quant_weight_fp8_t(Tensor w, int64_t cp, Tensor scale, c10::optional<Tensor> amax) {
  CHECK_DEV(w); CHECK_F32(w); CHECK_F32(scale);
  TORCH_CHECK(w.dim() == 4, "weight must be [K,C,R,S]");
  const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(cp >= C && cp % 16 == 0, "fp8 weight: padded channels must be >= C and a multiple of 16");
  c10::DeviceGuard g(w.device());
  Tensor wphys = w.permute({0, 2, 3, 1}).contiguous();
  Tensor q = torch::empty({K, R, S, cp}, w.options().dtype(torch::kUInt8));
  Tensor qt = torch::empty({cp, R, S, K}, w.options().dtype(torch::kUInt8));
  float* am = (amax && amax->defined()) ? amax->data_ptr<float>() : nullptr;
  TORCH_CHECK(!am || (amax->numel() >= 64 && amax->is_contiguous()), "amax must be [64] slots");
  CHECK_RC(pmd::quant_weight_fp8_launch(wphys.data_ptr<float>(), q.data_ptr<uint8_t>(),
                                        scale.data_ptr<float>(), am, K, R * S, C, (int)cp, cur_stream(),
                                        qt.data_ptr<uint8_t>()),
           "quant_weight_fp8");
  return {q, qt};
}

// Fp8Scaling.update(): amax [capacity, kAmaxSlots] fp32, scale [capacity] fp32, first n sites
void fp8_update_scales(Tensor amax, Tensor scale, int64_t n, double fmax) {
  CHECK_DEV(amax); CHECK_F32(amax); CHECK_CONT(amax);
  CHECK_DEV(scale); CHECK_F32(scale); CHECK_CONT(scale);
  TORCH_CHECK(amax.dim() == 2 && amax.size(1) == 64 && scale.dim() == 1 && n >= 0 && n <= amax.size(0) &&
                  n <= scale.size(0),
              "fp8_update_scales: amax [cap, 64], scale [cap], n <= cap");
  c10::DeviceGuard g(amax.device());
  CHECK_RC(pmd::fp8_update_scales_launch(amax.data_ptr<float>(), scale.data_ptr<float>(), (int)n, (float)fmax,
                                         cur_stream()),
           "fp8_update_scales");
}

Tensor dequant_fp8(Tensor q, c10::optional<Tensor> inv_scale, bool bf8) {
  CHECK_DEV(q); CHECK_U8(q); CHECK_CONT(q);
  c10::DeviceGuard g(q.device());
  Tensor out = torch::empty(q.sizes(), q.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::dequant_fp8_launch(q.data_ptr<uint8_t>(), out.data_ptr<float>(),
                                   (inv_scale && inv_scale->defined()) ? inv_scale->data_ptr<float>() : nullptr,
                                   q.numel(), cur_stream(), bf8), "dequant_fp8");
  return out;
}

Tensor fp8_mfma_probe(Tensor A, Tensor Bt) {
  CHECK_DEV(A); CHECK_U8(A); CHECK_CONT(A); CHECK_U8(Bt); CHECK_CONT(Bt);
  TORCH_CHECK(A.numel() == 16 * 128 && Bt.numel() == 16 * 128, "probe: A, Bt must be [16,128]");
  c10::DeviceGuard g(A.device());
  Tensor C = torch::empty({16, 16}, A.options().dtype(torch::kFloat32));
  CHECK_RC(pmd::fp8_mfma_probe_launch(A.data_ptr<uint8_t>(), Bt.data_ptr<uint8_t>(), C.data_ptr<float>(),
                                      cur_stream()), "fp8_mfma_probe");
  return C;
}

// sx, sw: device scalars the operands were quantised with (y = conv(xq, wq) / (sx * sw))
static int g_fp8_fwd_impl = -1;  // -1: PMD_FP8_FWD_IMPL (default 1)

std::vector<Tensor> conv_fp8_fwd(Tensor xq, Tensor wq, Tensor sx, Tensor sw, int64_t stride, int64_t pad,
                                 bool want_stats, c10::optional<Tensor> stats_buf,
                                 c10::optional<Tensor> shift) {
  CHECK_DEV(xq); CHECK_U8(xq); CHECK_CONT(xq); CHECK_U8(wq); CHECK_CONT(wq); CHECK_F32(sx); CHECK_F32(sw);
  TORCH_CHECK(xq.dim() == 4 && wq.dim() == 4, "fp8 conv: NHWC input and KRSC weight");
  const int N = xq.size(0), H = xq.size(1), W = xq.size(2), C = xq.size(3);
  const int K = wq.size(0), R = wq.size(1), S = wq.size(2);
  TORCH_CHECK(wq.size(3) == C, "fp8 conv: weight channels must match the (padded) input");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  c10::DeviceGuard g(xq.device());
  Tensor y = torch::empty({N, P, Q, K}, xq.options().dtype(torch::kBFloat16));
  Tensor stats;
  if (want_stats) {
    if (stats_buf && stats_buf->defined()) {
      stats = *stats_buf;
      TORCH_CHECK(stats.numel() == pmd_slots() * 2 * K, "stats buffer must be [slots, 2, K]");
    } else {
      stats = pmd_zeros({pmd_slots(), 2, K}, xq.options().dtype(torch::kFloat32));
    }
  }
  // implementation: 1 (default) = the implicit-GEMM kernel's fp8 path, 0 = conv_fp8_fwd_kernel
  // (fp8.hip); the igemm path measured +2.5% on the fp8 step (16.87-16.96 vs 17.31-17.40 ms)
  static int impl = -1;
  if (impl < 0) {
    const char* e = getenv("PMD_FP8_FWD_IMPL");
    impl = (e && e[0] == '0') ? 0 : 1;
  }
  if (g_fp8_fwd_impl >= 0) impl = g_fp8_fwd_impl;
  if (impl == 1) {
    CHECK_RC(pmd::conv_fwd_fp8_igemm_launch(xq.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), bfp_mut(y),
                                            want_stats ? stats.data_ptr<float>() : nullptr,
                                            sx.data_ptr<float>(), sw.data_ptr<float>(), N, H, W, C, P, Q, K, R,
                                            S, (int)stride, (int)pad, cur_stream(), shift_ptr(shift, K)),
             "conv_fp8_fwd (igemm)");
  } else {
    CHECK_RC(pmd::conv_fp8_fwd_launch(xq.data_ptr<uint8_t>(), wq.data_ptr<uint8_t>(), bfp_mut(y),
                                      want_stats ? stats.data_ptr<float>() : nullptr,
                                      sx.data_ptr<float>(), sw.data_ptr<float>(), N, H, W, C, P, Q, K, R, S,
                                      (int)stride, (int)pad, cur_stream(), shift_ptr(shift, K)),
             "conv_fp8_fwd");
  }
  if (want_stats) return {y, stats};
  return {y};
}

// ------------------------------------------------------------- classifier
static void chk_lin(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() && t.dim() == 2, what,
              " must be a contiguous 2-D fp32 GPU tensor");
}

// out[N][V] = x[N][K] . w[V][K]^T (+ b)
// split-K workspace of one classifier product (stream-ordered via the caching allocator)
float* linear_ws(Tensor& holder, const Tensor& like, int M, int Nc, int R) {
  const long long n = pmd::linear_workspace_floats(M, Nc, R);
  if (n == 0) return nullptr;
  holder = torch::empty({n}, like.options().dtype(torch::kFloat32));
  return holder.data_ptr<float>();
}

Tensor linear_fwd(Tensor x, Tensor w, c10::optional<Tensor> b) {
  chk_lin(x, "x");
  chk_lin(w, "w");
  TORCH_CHECK(x.size(1) == w.size(1), "linear: feature mismatch");
  const int N = x.size(0), K = x.size(1), V = w.size(0);
  const float* bp = opt_f32(b, "bias");
  if (bp) TORCH_CHECK(b->numel() == V, "linear: bias size");
  c10::DeviceGuard g(x.device());
  Tensor out = torch::empty({N, V}, x.options());
  Tensor ws;
  float* wsp = linear_ws(ws, x, N, V, K);
  CHECK_RC(pmd::linear_mfma_launch(x.data_ptr<float>(), w.data_ptr<float>(), out.data_ptr<float>(), bp,
                                   K, 1, 1, K, N, V, K, false, wsp, cur_stream()), "linear_fwd");
  return out;
}

// dx[N][K] = dout[N][V] . w[V][K]
Tensor linear_dgrad(Tensor dout, Tensor w) {
  chk_lin(dout, "dout");
  chk_lin(w, "w");
  TORCH_CHECK(dout.size(1) == w.size(0), "linear dgrad: class mismatch");
  const int N = dout.size(0), V = w.size(0), K = w.size(1);
  c10::DeviceGuard g(dout.device());
  Tensor dx = torch::empty({N, K}, dout.options());
  Tensor ws;
  float* wsp = linear_ws(ws, dout, N, K, V);
  CHECK_RC(pmd::linear_mfma_launch(dout.data_ptr<float>(), w.data_ptr<float>(), dx.data_ptr<float>(), nullptr,
                                   V, 1, K, 1, N, K, V, false, wsp, cur_stream()), "linear_dgrad");
  return dx;
}

// dw[V][K] (+)= dout^T . x ; db[V] (+)= column sums of dout (both optional targets,
// e.g. grad-arena views; accumulate=false overwrites)
void linear_wgrad(Tensor dout, Tensor x, Tensor dw, c10::optional<Tensor> db, bool accumulate) {
  chk_lin(dout, "dout");
  chk_lin(x, "x");
  chk_lin(dw, "dw");
  const int N = dout.size(0), V = dout.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == N && dw.size(0) == V && dw.size(1) == K, "linear wgrad: shapes");
  c10::DeviceGuard g(dout.device());
  Tensor ws;
  float* wsp = linear_ws(ws, dout, V, K, N);
  CHECK_RC(pmd::linear_mfma_launch(dout.data_ptr<float>(), x.data_ptr<float>(), dw.data_ptr<float>(), nullptr,
                                   1, V, K, 1, V, K, N, accumulate, wsp, cur_stream()), "linear_wgrad");
  float* dbp = opt_f32(db, "db");
  if (dbp) {
    TORCH_CHECK(db->numel() == V, "linear wgrad: bias grad size");
    CHECK_RC(pmd::linear_colsum_launch(dout.data_ptr<float>(), dbp, N, V, accumulate, cur_stream()),
             "linear_colsum");
  }
}

}  // namespace

namespace pmd { void register_runtime(pybind11::module& m); }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) kernels for pytorch_multiprocessing_distributed_amd";
  pmd::register_runtime(m);
  m.def("conv_weight_prep", &conv_weight_prep);
  m.def("wgrad_set_defer", &pmd::wgrad_set_defer,
        "queue the split-K reductions of the following weight gradients (this thread)");
  m.def("wgrad_pending", &pmd::wgrad_pending);
  m.def("wgrad_flush", &wgrad_flush, "launch the queued split-K reductions as one grouped kernel");
  m.def("conv_fp8_fwd_set_impl", [](int64_t i) { g_fp8_fwd_impl = (int)i; },
        "fp8 forward conv kernel: 0 conv_fp8_fwd_kernel, 1 the implicit-GEMM kernel's fp8 path (default), -1 env");
  m.def("conv_set_impl", &pmd::conv_set_impl, "conv staging/pipeline variant 0-4, 5 = per-shape default");
  m.def("det_stats_set", &pmd::det_stats_set,
        "deterministic BN-statistics mode (test/debug): private per-block slots folded in a fixed order");
  m.def("det_stats_on", &pmd::det_stats_on);
  m.def("gpu_sleep", [](int64_t us) { CHECK_RC(pmd::gpu_sleep_launch((int)us, cur_stream()), "gpu_sleep"); },
        "test utility: idle the current stream for `us` microseconds (<= 1 s)");
  m.def("conv_probe_set", [](torch::Tensor buf) {
          TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == torch::kInt64 && buf.dim() == 2 && buf.size(1) == 16,
                      "probe buffer: int64 [records, 16] on the GPU");
          return (int64_t)pmd::conv_probe_set(buf.data_ptr(), (int)buf.size(0));
        },
        "data-gradient section probe buffer (PMD_DGRAD_PROBE builds: returns 1; production builds: 0, no-op)");
  m.def("conv_probe_count", []() { return (int64_t)pmd::conv_probe_count(); });
  m.def("conv_set_tile", &pmd::conv_set_tile,
        "conv fwd/dgrad tile policy: 0 auto, 1 128-row only, 2 256x128, 3 256x256 where legal");
  m.def("conv_set_big_pipe", &pmd::conv_set_big_pipe,
        "256-row conv tiles: 0 BK=64 x2 stages, 1 BK=64 x3 (256x128 only), 2 BK=32 x4");
  m.def("conv_set_autotune", &pmd::conv_set_autotune, "per-shape conv kernel autotuning on/off");
  m.def("conv_autotune_entries", &pmd::conv_autotune_entries);
  m.def("conv_autotune_clear", &pmd::conv_autotune_clear);
  m.def("conv_autotune_export", &pmd::conv_autotune_export);
  m.def("conv_autotune_import", &pmd::conv_autotune_import);
  m.def("wgrad_autotune_export", &pmd::wgrad_autotune_export);
  m.def("wgrad_autotune_import", &pmd::wgrad_autotune_import);
  m.def("wgrad_autotune_clear", &pmd::wgrad_autotune_clear);
  m.def("conv_wgrad_set_impl", &pmd::conv_wgrad_set_impl,
        "wgrad staging variant: 0 registers, 1 LDS-DMA 64x2 (default), 2 LDS-DMA 32x4, 3 LDS-DMA 64x3");
  namespace py = pybind11;
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("wk"), py::arg("stride"), py::arg("pad"),
        py::arg("want_stats"), py::arg("stats_buf"), py::arg("shift") = py::none());
  m.def("conv_fwd_hw", &conv_fwd_hw, py::arg("x"), py::arg("wk"), py::arg("stride"), py::arg("pad"),
        py::arg("out_h"), py::arg("out_w"), py::arg("want_stats"), py::arg("stats_buf"),
        py::arg("shift") = py::none());
  m.def("stem_s2d_input", &stem_s2d_input);
  m.def("stem_s2d_weight", &stem_s2d_weight);
  m.def("stem_s2d_wgrad_fold", &stem_s2d_wgrad_fold);
  m.def("stem_wgrad_fused", &stem_wgrad_fused, py::arg("dout"), py::arg("arg"), py::arg("y"), py::arg("params"),
        py::arg("gamma"), py::arg("red"), py::arg("count"), py::arg("count_h"), py::arg("xs"), py::arg("pad"));
  m.def("winograd_filter", &winograd_filter);
  m.def("winograd_input", &winograd_input);
  m.def("winograd_gemm", &winograd_gemm, py::arg("V"), py::arg("U"));
  m.def("winograd_fused_fwd", &winograd_fused_fwd, py::arg("x"), py::arg("U"), py::arg("want_stats"),
        py::arg("stats_buf") = py::none(), py::arg("shift") = py::none());
  m.def("winograd_output", &winograd_output, py::arg("M"), py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("want_stats"), py::arg("stats_buf"), py::arg("shift") = py::none());
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("wkt"), py::arg("H"), py::arg("W"),
        py::arg("stride"), py::arg("pad"), py::arg("addend"), py::arg("bn_mask"), py::arg("bn_y0"),
        py::arg("bn_p0"), py::arg("bn_red0"), py::arg("bn_y1"), py::arg("bn_p1"), py::arg("bn_red1"),
        py::arg("addend_mask"), py::arg("addend_bias") = py::none());
  m.def("bnlin_coeff", &bnlin_coeff, py::arg("red"), py::arg("count"), py::arg("count_h"), py::arg("gamma"),
        py::arg("params"), py::arg("wk"), py::arg("C"),
        "linear-BN backward coefficients -> [G image, bias, abc]");
  m.def("bnlin_dimg", &bnlin_dimg, py::arg("gamma"), py::arg("params"), py::arg("wk"), py::arg("C"),
        "linear-BN backward: the gamma*invstd-scaled transposed dgrad image [C,1,1,K]");
  m.def("colsum", &colsum, "fp32 column sums of an NHWC bf16 activation");
  m.def("bnlin_wgrad", &bnlin_wgrad, "linear-BN backward weight gradient combine (+= into out)");
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("out") = py::none());
  m.def("bn_finalize", &bn_finalize, py::arg("sums"), py::arg("count"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("rm"), py::arg("rv"), py::arg("momentum"), py::arg("nbt"),
        py::arg("eval_mode"), py::arg("shift") = py::none());
  m.def("bn_apply", &bn_apply, py::arg("y1"), py::arg("p1"), py::arg("res"), py::arg("y2"), py::arg("p2"),
        py::arg("relu"), py::arg("want_mask"), py::arg("q8_scale"), py::arg("q8_amax"), py::arg("q8_only") = false);
  m.def("stats_collapse", &stats_collapse);
  m.def("stats_finalize_local", &stats_finalize_local, py::arg("slots"), py::arg("count"), py::arg("gamma"),
        py::arg("beta"), py::arg("eps"), py::arg("rm"), py::arg("rv"), py::arg("momentum"), py::arg("nbt"),
        py::arg("shift") = py::none());
  m.def("bn_bwd_reduce", &bn_bwd_reduce);
  m.def("bn_bwd_elemt", &bn_bwd_elemt, py::arg("dout"), py::arg("mask"), py::arg("y"), py::arg("params"),
        py::arg("gamma"), py::arg("red"), py::arg("count"), py::arg("count_h"), py::arg("relu"),
        py::arg("want_dzm"), py::arg("eval_mode"), py::arg("q8_scale") = py::none(),
        py::arg("q8_amax") = py::none(), py::arg("q8_only") = false);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("stem_pool_fwd", &stem_pool_fwd);
  m.def("stem_pool_bwd_reduce", &stem_pool_bwd_reduce);
  m.def("stem_pool_bwd_elemt", &stem_pool_bwd_elemt);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_dgrad", &linear_dgrad);
  m.def("linear_wgrad", &linear_wgrad);
  m.def("zero_", &zero_, "in-place zero of a contiguous GPU tensor (framework fill kernel)");
  m.def(
      "create_stream",
      [](int64_t device, int64_t priority, std::vector<int64_t> cu_mask) {
        c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device));
        hipStream_t s = nullptr;
        if (!cu_mask.empty()) {
          // a stream restricted to a subset of the CUs (bit i of word i/32 = CU i); HIP gives
          // it normal priority and a hardware queue of its own
          std::vector<uint32_t> m(cu_mask.begin(), cu_mask.end());
          const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data());
          TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
          return (int64_t) reinterpret_cast<uintptr_t>(s);
        }
        const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, (int)priority);
        TORCH_CHECK(e == hipSuccess, "hipStreamCreateWithPriority: ", hipGetErrorString(e));
        return (int64_t) reinterpret_cast<uintptr_t>(s);
      },
      py::arg("device"), py::arg("priority"), py::arg("cu_mask") = std::vector<int64_t>(),
      "a new non-blocking HIP stream (lives for the process; wrap with torch.cuda.ExternalStream): the "
      "step's streams are created up front so each gets its own hardware queue");
  m.def("sgd_", &sgd_);
  m.def("synth_images", &synth_images);
  m.def("cifar_augment", &cifar_augment);
  m.def("quant_bf16_fp8", &quant_bf16_fp8, py::arg("x"), py::arg("scale"), py::arg("amax") = py::none(),
        py::arg("bf8") = false);
  m.def("quant_weight_fp8_t", &quant_weight_fp8_t);
  m.def("conv_dgrad_fp8", &conv_dgrad_fp8, py::arg("dyq"), py::arg("wtq"), py::arg("sdy"), py::arg("sw"),
        py::arg("H"), py::arg("W"), py::arg("stride"), py::arg("pad"), py::arg("addend") = py::none(),
        py::arg("bn_mask") = py::none(), py::arg("bn_y0") = py::none(), py::arg("bn_p0") = py::none(),
        py::arg("bn_red0") = py::none(), py::arg("bn_y1") = py::none(), py::arg("bn_p1") = py::none(),
        py::arg("bn_red1") = py::none(), py::arg("addend_mask") = py::none());
  m.def("conv_wgrad_fp8", &conv_wgrad_fp8, py::arg("dyq"), py::arg("xq"), py::arg("sdy"), py::arg("sx"),
        py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("out") = py::none());
  m.def("quant_weight_fp8", &quant_weight_fp8);
  m.def("dequant_fp8", &dequant_fp8, py::arg("q"), py::arg("inv_scale") = py::none(), py::arg("bf8") = false);
  m.def("fp8_update_scales", &fp8_update_scales, py::arg("amax"), py::arg("scale"), py::arg("n"), py::arg("fmax"));
  m.def("fp8_mfma_probe", &fp8_mfma_probe);
  m.def("conv_fp8_fwd", &conv_fp8_fwd, py::arg("xq"), py::arg("wq"), py::arg("sx"), py::arg("sw"),
        py::arg("stride"), py::arg("pad"), py::arg("want_stats"), py::arg("stats_buf"),
        py::arg("shift") = py::none());
}
