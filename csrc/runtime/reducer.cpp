// Native bucketed gradient reducer.
//
// The reference gets gradient averaging from torch's C++ DDP Reducer
// (reference main.py:44 -> torch:nn/parallel/distributed.py:828-834).  This is
// the framework's own, much smaller reducer built around the flat grad arena
// (parallel/flat.py):
//
//   * buckets are contiguous [start, end) slices of the fp32 grad arena, laid
//     out in reverse registration order at construction and re-laid out in the
//     OBSERVED gradient-ready order after the first iteration (parallel/dp.py
//     calls rebuild(); torch's Reducer does the same with its bucket views), so
//     a bucket all-reduce is in place and zero-copy (optionally through a bf16
//     wire buffer: half the xGMI bytes);
//   * mark(i) is called once gradient i is final in the arena -- from the
//     AccumulateGrad post-hook or from a fused op that wrote it directly.
//     Buckets are launched strictly in INDEX order (a cursor, like DDP's
//     next_bucket): a bucket whose gradients are complete waits for every
//     lower-index bucket, so all ranks issue the identical collective sequence
//     even if marks arrive in a different order on different ranks;
//   * transport: the native RCCL communicator (runtime/rccl_comm.cpp: its own
//     HIP stream, hipEvent fences, no host blocking) or any c10d ProcessGroup
//     (RCCL via ProcessGroupNCCL, gloo on the CPU test path -- the identical
//     bookkeeping runs in the 2-rank CPU tests);
//   * the first mark of an iteration queues a final callback on the autograd
//     engine; finalize() first runs the Python pre-finalize hook (it joins the
//     weight gradients still running on the side stream and marks them, see
//     ops/functional.py::flush_pending_wgrads), then launches buckets whose
//     params got no gradient, joins every bucket (a stream-side wait), copies
//     compressed buckets back and checks every bucket fired exactly once;
//   * optional timeline: host time of every launch relative to the first mark,
//     and (RCCL transport) device start/end of every bucket's all-reduce
//     relative to the end of the backward's compute work.
#include <torch/extension.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <chrono>
#include <limits>
#include <memory>
#include <mutex>
#include <sstream>

#include "runtime/rccl_comm.h"

namespace pmd {

namespace py = pybind11;

class Reducer {
 public:
  Reducer(py::object pg, py::object rccl, at::Tensor grad_arena, std::vector<int64_t> bounds,
          std::vector<int64_t> param_bucket, bool use_avg, bool compress_bf16, py::object pre_finalize,
          bool timeline)
      : arena_(std::move(grad_arena)), use_avg_(use_avg), compress_(compress_bf16), timeline_(timeline) {
    if (!rccl.is_none()) {
      rccl_ = rccl.cast<RcclComm*>();
      rccl_keep_ = rccl;  // keep the Python owner alive as long as the reducer
      world_ = (int)rccl_->world();
    } else {
      TORCH_CHECK(!pg.is_none(), "reducer: needs a process group or an RcclComm");
      pg_ = pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
      world_ = pg_->getSize();
    }
    if (!pre_finalize.is_none()) pre_finalize_ = pre_finalize;
    TORCH_CHECK(arena_.dim() == 1 && arena_.is_contiguous(), "grad arena must be a flat contiguous tensor");
    setup_(std::move(bounds), std::move(param_bucket));
  }

  ~Reducer() {
    for (auto* v : {&done_ev_, &start_ev_})
      for (auto e : *v)
        if (e) (void)hipEventDestroy(e);
    if (fin_ev_) (void)hipEventDestroy(fin_ev_);
  }

  // gradient of parameter i is final in the arena. Returns true if this call
  // launched at least one bucket.
  bool mark(int64_t i) {
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(i >= 0 && i < static_cast<int64_t>(param_bucket_.size()), "param index out of range");
    if (!enabled_ || marked_[i]) return false;
    if (mark_order_.empty()) t0_ = now_us_();
    marked_[i] = 1;
    mark_order_.push_back(i);
    if (!callback_queued_) {
      callback_queued_ = true;
      torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
    }
    const int b = static_cast<int>(param_bucket_[i]);
    --pending_[b];
    bool launched = false;
    while (next_ < nb_ && pending_[next_] == 0) {
      launch_(next_++);
      launched = true;
    }
    return launched;
  }

  void finalize() {
    if (pre_finalize_) {
      // outside mu_: the hook marks the deferred weights, which takes mu_
      py::gil_scoped_acquire gil;
      pre_finalize_();
    }
    std::lock_guard<std::mutex> lk(mu_);
    const double t_fin = now_us_();
    if (rccl_ && timeline_) {
      c10::DeviceGuard g(arena_.device());
      (void)hipEventRecord(fin_ev_, c10::hip::getCurrentHIPStream().stream());
    }
    while (next_ < nb_) launch_(next_++);  // buckets whose params produced no gradient
    if (rccl_) {
      c10::DeviceGuard g(arena_.device());
      for (int b = 0; b < nb_; ++b) rccl_->wait(done_ev_[b]);
    } else {
      for (int b = 0; b < nb_; ++b) works_[b]->wait();
    }
    if (compress_) {
      for (int b = 0; b < nb_; ++b) slice_(b).copy_(wire_[b]);
    }
    std::vector<int> bad;
    for (int b = 0; b < nb_; ++b)
      if (fired_[b] != 1) bad.push_back(b);
    last_order_ = order_;
    last_mark_order_ = mark_order_;
    last_launch_us_ = launch_us_;
    last_fin_us_ = t_fin - t0_;
    have_dev_timeline_ = rccl_ && timeline_;
    reset_();
    iteration_++;
    if (!bad.empty()) {
      std::ostringstream os;
      for (int b : bad) os << b << " ";
      TORCH_CHECK(false, "reducer: buckets [", os.str(), "] did not fire exactly once this iteration");
    }
  }

  // New bucket layout (between iterations only): same arena, new bounds.
  void rebuild(std::vector<int64_t> bounds, std::vector<int64_t> param_bucket) {
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(!callback_queued_, "reducer: rebuild() during a backward pass");
    TORCH_CHECK(param_bucket.size() == param_bucket_.size(), "reducer: rebuild changes the parameter count");
    setup_(std::move(bounds), std::move(param_bucket));
  }

  void set_enabled(bool e) {
    std::lock_guard<std::mutex> lk(mu_);
    enabled_ = e;
  }
  bool enabled() const { return enabled_; }
  int64_t iteration() const { return iteration_; }
  int num_buckets() const { return nb_; }
  std::vector<int64_t> bounds() const { return bounds_; }
  std::vector<int> last_launch_order() const { return last_order_; }
  std::vector<int64_t> last_mark_order() const { return last_mark_order_; }
  bool uses_rccl() const { return rccl_ != nullptr; }

  // Last iteration, one tuple per bucket in launch order:
  //   (bucket, host launch time [us after the first mark], host finalize time [us],
  //    device all-reduce start, device end [ms relative to the end of the backward's
  //    compute stream work; negative = overlapped with backward]  -- NaN without the
  //    RCCL transport or with the timeline off)
  py::list timeline() {
    std::lock_guard<std::mutex> lk(mu_);
    py::list out;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    if (have_dev_timeline_) (void)hipEventSynchronize(done_ev_.empty() ? fin_ev_ : done_ev_.back());
    for (size_t k = 0; k < last_order_.size(); ++k) {
      const int b = last_order_[k];
      double s = nan, e = nan;
      if (have_dev_timeline_) {
        float ms = 0.f;
        (void)hipEventSynchronize(done_ev_[b]);
        if (hipEventElapsedTime(&ms, fin_ev_, start_ev_[b]) == hipSuccess) s = ms;
        if (hipEventElapsedTime(&ms, fin_ev_, done_ev_[b]) == hipSuccess) e = ms;
      }
      out.append(py::make_tuple(b, k < last_launch_us_.size() ? last_launch_us_[k] : nan, last_fin_us_, s, e));
    }
    return out;
  }

 private:
  static double now_us_() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }

  void setup_(std::vector<int64_t> bounds, std::vector<int64_t> param_bucket) {
    bounds_ = std::move(bounds);
    param_bucket_ = std::move(param_bucket);
    TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() == arena_.numel(),
                "bucket bounds must cover the arena");
    for (size_t b = 0; b + 1 < bounds_.size(); ++b)
      TORCH_CHECK(bounds_[b] < bounds_[b + 1], "bucket bounds must be increasing");
    nb_ = static_cast<int>(bounds_.size()) - 1;
    pending0_.assign(nb_, 0);
    for (auto b : param_bucket_) {
      TORCH_CHECK(b >= 0 && b < nb_, "param bucket index out of range");
      pending0_[b]++;
    }
    for (int b = 0; b < nb_; ++b) TORCH_CHECK(pending0_[b] > 0, "bucket ", b, " has no parameters");
    works_.assign(nb_, {});
    wire_.assign(nb_, at::Tensor());
    if (rccl_) {
      c10::DeviceGuard g(arena_.device());
      const unsigned flags = timeline_ ? hipEventDefault : hipEventDisableTiming;
      while ((int)done_ev_.size() < nb_) {
        hipEvent_t d = nullptr, s = nullptr;
        TORCH_CHECK(hipEventCreateWithFlags(&d, flags) == hipSuccess, "reducer: event");
        if (timeline_) TORCH_CHECK(hipEventCreateWithFlags(&s, flags) == hipSuccess, "reducer: event");
        done_ev_.push_back(d);
        start_ev_.push_back(s);
      }
      if (timeline_ && !fin_ev_) TORCH_CHECK(hipEventCreate(&fin_ev_) == hipSuccess, "reducer: event");
    }
    reset_();
  }

  at::Tensor slice_(int b) { return arena_.narrow(0, bounds_[b], bounds_[b + 1] - bounds_[b]); }

  void launch_(int b) {
    TORCH_CHECK(fired_[b] == 0, "reducer: bucket ", b, " launched twice in one iteration");
    fired_[b]++;
    order_.push_back(b);
    launch_us_.push_back(now_us_() - t0_);
    at::Tensor s = slice_(b);
    at::Tensor t = compress_ ? s.to(at::kBFloat16) : s;
    if (compress_) wire_[b] = t;
    if (!use_avg_ && world_ > 1) t.mul_(1.0 / world_);  // pre-scale + SUM (gloo has no AVG)
    if (rccl_) {
      rccl_->all_reduce_record(t, use_avg_ ? 1 : 0, done_ev_[b], timeline_ ? start_ev_[b] : nullptr);
      return;
    }
    c10d::AllreduceOptions opts;
    opts.reduceOp = use_avg_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
    std::vector<at::Tensor> ts{t};
    works_[b] = pg_->allreduce(ts, opts);
  }

  void reset_() {
    pending_ = pending0_;
    marked_.assign(param_bucket_.size(), 0);
    fired_.assign(nb_, 0);
    for (auto& w : works_) w.reset();
    for (auto& w : wire_) w = at::Tensor();
    order_.clear();
    mark_order_.clear();
    launch_us_.clear();
    next_ = 0;
    callback_queued_ = false;
  }

  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  RcclComm* rccl_ = nullptr;
  py::object rccl_keep_;
  py::object pre_finalize_;
  at::Tensor arena_;
  std::vector<int64_t> bounds_, param_bucket_;
  bool use_avg_, compress_, timeline_;
  int nb_ = 0, world_ = 1, next_ = 0;
  std::vector<int> pending0_, pending_, fired_, order_, last_order_;
  std::vector<int64_t> mark_order_, last_mark_order_;
  std::vector<double> launch_us_, last_launch_us_;
  double t0_ = 0.0, last_fin_us_ = 0.0;
  std::vector<char> marked_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_;
  std::vector<hipEvent_t> done_ev_, start_ev_;
  hipEvent_t fin_ev_ = nullptr;
  bool have_dev_timeline_ = false;
  std::vector<at::Tensor> wire_;
  bool enabled_ = true, callback_queued_ = false;
  int64_t iteration_ = 0;
  std::mutex mu_;
};

void register_xgmi(pybind11::module& m);
void register_trace(pybind11::module& m);
void register_weights(pybind11::module& m);
void register_rccl(pybind11::module& m);
void register_events(pybind11::module& m);

void register_runtime(pybind11::module& m) {
  register_xgmi(m);
  register_trace(m);
  register_weights(m);
  register_rccl(m);
  register_events(m);
  py::class_<Reducer>(m, "Reducer")
      .def(py::init<py::object, py::object, at::Tensor, std::vector<int64_t>, std::vector<int64_t>, bool, bool,
                    py::object, bool>(),
           py::arg("process_group"), py::arg("rccl"), py::arg("grad_arena"), py::arg("bounds"),
           py::arg("param_bucket"), py::arg("use_avg"), py::arg("compress_bf16") = false,
           py::arg("pre_finalize") = py::none(), py::arg("timeline") = false)
      .def("mark", &Reducer::mark, py::arg("index"))
      .def("finalize", &Reducer::finalize)
      .def("rebuild", &Reducer::rebuild, py::arg("bounds"), py::arg("param_bucket"))
      .def("set_enabled", &Reducer::set_enabled)
      .def("timeline", &Reducer::timeline)
      .def_property_readonly("enabled", &Reducer::enabled)
      .def_property_readonly("iteration", &Reducer::iteration)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("bounds", &Reducer::bounds)
      .def_property_readonly("uses_rccl", &Reducer::uses_rccl)
      .def("last_launch_order", &Reducer::last_launch_order)
      .def("last_mark_order", &Reducer::last_mark_order);
}

}  // namespace pmd
