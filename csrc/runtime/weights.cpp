// Persistent bf16 weight images for every convolution of a model, refreshed
// by ONE grouped kernel per step (kernels/conv_igemm.hip) instead of one
// conv_weight_prep launch per conv (53 for ResNet-50, ~7 us each).
//
// The fp32 master weights live in the flat parameter arena (parallel/flat.py)
// at fixed addresses, so the descriptor table (source pointer, destination
// images, shapes) is built once and kept on the device; refresh() is a single
// launch with no host->device traffic -- also safe inside a captured HIP graph.
// The images are overwritten in place: a backward pass must run before the next
// refresh() -- the training loop's fwd -> bwd -> step order (and gradient
// accumulation, where the weights do not change) guarantees it.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/launchers.h"

namespace pmd {

class WeightImages {
 public:
  // entries: (weight [K,C,R,S] fp32 channels_last, padded channels Cp, want transposed image)
  WeightImages(std::vector<at::Tensor> weights, std::vector<int64_t> cps, std::vector<bool> want_t)
      : weights_(std::move(weights)) {
    TORCH_CHECK(weights_.size() == cps.size() && cps.size() == want_t.size() && !weights_.empty(),
                "weight images: mismatched entry lists");
    const auto dev = weights_[0].device();
    std::vector<WeightPrepDesc> descs;
    std::vector<int> starts{0};
    for (size_t i = 0; i < weights_.size(); ++i) {
      const at::Tensor& w = weights_[i];
      TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.device() == dev,
                  "weight images: fp32 GPU [K,C,R,S] weights on one device");
      TORCH_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast), "weight images: channels_last weights");
      const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
      const int cp = (int)cps[i];
      TORCH_CHECK(cp >= C && cp % 8 == 0, "weight images: padded channels");
      auto opt = w.options().dtype(at::kBFloat16);
      at::Tensor wk = at::empty({K, R, S, cp}, opt);
      at::Tensor wkt = want_t[i] ? at::empty({cp, R, S, K}, opt) : at::Tensor();
      wk_.push_back(wk);
      wkt_.push_back(wkt);
      WeightPrepDesc d;
      d.w = w.data_ptr<float>();
      d.wk = reinterpret_cast<bf16_t*>(wk.data_ptr());
      d.wkt = wkt.defined() ? reinterpret_cast<bf16_t*>(wkt.data_ptr()) : nullptr;
      d.K = K;
      d.RS = R * S;
      d.C = C;
      d.Cp = cp;
      descs.push_back(d);
      const long long total = (long long)K * R * S * cp;
      long long nb = (total + 256 * 8 - 1) / (256 * 8);  // ~8 elements per thread
      if (nb < 1) nb = 1;
      if (nb > 1024) nb = 1024;
      starts.push_back(starts.back() + (int)nb);
      ptrs_.push_back(d.w);
    }
    total_blocks_ = starts.back();
    n_ = (int)descs.size();
    d_descs_ = at::empty({(int64_t)(descs.size() * sizeof(WeightPrepDesc))},
                         weights_[0].options().dtype(at::kByte));
    d_starts_ = at::empty({(int64_t)starts.size()}, weights_[0].options().dtype(at::kInt));
    c10::DeviceGuard g(dev);
    auto st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(hipMemcpyAsync(d_descs_.data_ptr(), descs.data(), descs.size() * sizeof(WeightPrepDesc),
                               hipMemcpyHostToDevice, st) == hipSuccess, "weight images: descriptor copy");
    TORCH_CHECK(hipMemcpyAsync(d_starts_.data_ptr(), starts.data(), starts.size() * sizeof(int),
                               hipMemcpyHostToDevice, st) == hipSuccess, "weight images: table copy");
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess, "weight images: sync");
  }

  // mode 1: forward images only, 2: dgrad images only, 3: both (current stream)
  void refresh(int64_t mode) {
    TORCH_CHECK(mode >= 1 && mode <= 3, "weight images: refresh mode 1..3");
    for (size_t i = 0; i < weights_.size(); ++i)
      TORCH_CHECK(weights_[i].data_ptr<float>() == ptrs_[i],
                  "weight images: a weight was re-allocated; rebuild the image set");
    c10::DeviceGuard g(weights_[0].device());
    conv_weight_prep_grouped_launch(reinterpret_cast<const WeightPrepDesc*>(d_descs_.data_ptr()),
                                    d_starts_.data_ptr<int>(), n_, total_blocks_,
                                    c10::hip::getCurrentHIPStream().stream(), (int)mode);
    if (mode & 1) refreshed_++;
  }

  std::vector<at::Tensor> get(int64_t i) const {
    TORCH_CHECK(i >= 0 && i < n_, "weight images: index");
    if (wkt_[i].defined()) return {wk_[i], wkt_[i]};
    return {wk_[i]};
  }

  int64_t size() const { return n_; }
  int64_t refreshed() const { return refreshed_; }

 private:
  std::vector<at::Tensor> weights_, wk_, wkt_;
  std::vector<const float*> ptrs_;
  at::Tensor d_descs_, d_starts_;
  int n_ = 0, total_blocks_ = 0;
  int64_t refreshed_ = 0;
};

// FP8 (config 5) counterpart: e4m3 images of the block convs' weights with their
// delayed-scaling sites (scale [1], amax [kAmaxSlots] views of Fp8Scaling's
// buffers), quantised by ONE grouped launch per step instead of one
// quant_weight_fp8 launch per conv (52 x ~11 us for ResNet-50).
class Fp8WeightImages {
 public:
  // want_t[i]: also keep the transposed e4m3 image [Cp][R][S][K] (fp8 dgrad B^T)
  Fp8WeightImages(std::vector<at::Tensor> weights, std::vector<int64_t> cps, std::vector<at::Tensor> scales,
                  std::vector<at::Tensor> amaxes, std::vector<bool> want_t)
      : weights_(std::move(weights)), scales_(std::move(scales)), amaxes_(std::move(amaxes)) {
    TORCH_CHECK(want_t.empty() || want_t.size() == weights_.size(), "fp8 weight images: want_t size");
    TORCH_CHECK(!weights_.empty() && weights_.size() == cps.size() && cps.size() == scales_.size() &&
                    scales_.size() == amaxes_.size(),
                "fp8 weight images: mismatched entry lists");
    const auto dev = weights_[0].device();
    std::vector<Fp8WeightDesc> descs;
    std::vector<int> starts{0};
    for (size_t i = 0; i < weights_.size(); ++i) {
      const at::Tensor& w = weights_[i];
      TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.device() == dev &&
                      w.is_contiguous(at::MemoryFormat::ChannelsLast),
                  "fp8 weight images: fp32 channels_last GPU weights on one device");
      TORCH_CHECK(scales_[i].is_cuda() && scales_[i].scalar_type() == at::kFloat && scales_[i].numel() >= 1 &&
                      amaxes_[i].is_cuda() && amaxes_[i].scalar_type() == at::kFloat &&
                      amaxes_[i].is_contiguous() && amaxes_[i].numel() == 64,
                  "fp8 weight images: scale [1] / amax [64] fp32 sites");
      const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
      const int cp = (int)cps[i];
      TORCH_CHECK(cp >= C && cp % 8 == 0, "fp8 weight images: padded channels");
      at::Tensor q = at::empty({K, R, S, cp}, w.options().dtype(at::kByte));
      q_.push_back(q);
      at::Tensor qt;
      if (!want_t.empty() && want_t[i]) qt = at::empty({cp, R, S, K}, w.options().dtype(at::kByte));
      qt_.push_back(qt);
      Fp8WeightDesc d;
      d.w = w.data_ptr<float>();
      d.q = q.data_ptr<uint8_t>();
      d.qt = qt.defined() ? qt.data_ptr<uint8_t>() : nullptr;
      d.scale = scales_[i].data_ptr<float>();
      d.amax = amaxes_[i].data_ptr<float>();
      d.K = K;
      d.RS = R * S;
      d.C = C;
      d.Cp = cp;
      descs.push_back(d);
      const long long total = (long long)K * R * S * cp;
      long long nb = (total + 256 * 16 - 1) / (256 * 16);
      if (nb < 1) nb = 1;
      if (nb > 512) nb = 512;
      starts.push_back(starts.back() + (int)nb);
      ptrs_.push_back(d.w);
    }
    total_blocks_ = starts.back();
    n_ = (int)descs.size();
    d_descs_ = at::empty({(int64_t)(descs.size() * sizeof(Fp8WeightDesc))}, weights_[0].options().dtype(at::kByte));
    d_starts_ = at::empty({(int64_t)starts.size()}, weights_[0].options().dtype(at::kInt));
    c10::DeviceGuard g(dev);
    auto st = c10::hip::getCurrentHIPStream().stream();
    TORCH_CHECK(hipMemcpyAsync(d_descs_.data_ptr(), descs.data(), descs.size() * sizeof(Fp8WeightDesc),
                               hipMemcpyHostToDevice, st) == hipSuccess, "fp8 weight images: descriptor copy");
    TORCH_CHECK(hipMemcpyAsync(d_starts_.data_ptr(), starts.data(), starts.size() * sizeof(int),
                               hipMemcpyHostToDevice, st) == hipSuccess, "fp8 weight images: table copy");
    TORCH_CHECK(hipStreamSynchronize(st) == hipSuccess, "fp8 weight images: sync");
  }

  void refresh() {
    for (size_t i = 0; i < weights_.size(); ++i)
      TORCH_CHECK(weights_[i].data_ptr<float>() == ptrs_[i],
                  "fp8 weight images: a weight was re-allocated; rebuild the image set");
    c10::DeviceGuard g(weights_[0].device());
    quant_weight_fp8_grouped_launch(reinterpret_cast<const Fp8WeightDesc*>(d_descs_.data_ptr()),
                                    d_starts_.data_ptr<int>(), n_, total_blocks_,
                                    c10::hip::getCurrentHIPStream().stream());
  }

  at::Tensor get(int64_t i) const {
    TORCH_CHECK(i >= 0 && i < n_, "fp8 weight images: index");
    return q_[i];
  }

  // transposed image (undefined -> None when not requested)
  at::Tensor get_t(int64_t i) const {
    TORCH_CHECK(i >= 0 && i < n_, "fp8 weight images: index");
    return qt_[i];
  }

 private:
  std::vector<at::Tensor> weights_, scales_, amaxes_, q_, qt_;
  std::vector<const float*> ptrs_;
  at::Tensor d_descs_, d_starts_;
  int n_ = 0, total_blocks_ = 0;
};

void register_weights(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<WeightImages>(m, "WeightImages")
      .def(py::init<std::vector<at::Tensor>, std::vector<int64_t>, std::vector<bool>>())
      .def("refresh", &WeightImages::refresh, pybind11::arg("mode") = 3)
      .def("get", &WeightImages::get)
      .def_property_readonly("size", &WeightImages::size)
      .def_property_readonly("refreshed", &WeightImages::refreshed);
  py::class_<Fp8WeightImages>(m, "Fp8WeightImages")
      .def(py::init<std::vector<at::Tensor>, std::vector<int64_t>, std::vector<at::Tensor>,
                    std::vector<at::Tensor>, std::vector<bool>>(),
           py::arg("weights"), py::arg("cps"), py::arg("scales"), py::arg("amaxes"),
           py::arg("want_t") = std::vector<bool>())
      .def("refresh", &Fp8WeightImages::refresh)
      .def("get", &Fp8WeightImages::get)
      .def("get_t", &Fp8WeightImages::get_t);
}

}  // namespace pmd
