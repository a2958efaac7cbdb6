// Native bucketed gradient reducer.
//
// The reference gets gradient averaging from torch's C++ DDP Reducer
// (reference main.py:44 -> torch:nn/parallel/distributed.py:828-834).  This is
// the framework's own, much smaller reducer built around the flat grad arena
// (parallel/flat.py):
//
//   * buckets are contiguous [start, end) slices of the fp32 grad arena laid
//     out in backward-ready order, so a bucket all-reduce is in place and
//     zero-copy (optionally through a bf16 wire buffer: half the xGMI bytes);
//   * mark(i) is called once gradient i is final in the arena -- from the
//     AccumulateGrad post-hook or from a fused op that wrote it directly.
//     When a bucket's last gradient arrives it is launched immediately as an
//     async all-reduce on the process group (RCCL: its own HIP stream, fenced
//     against the producing compute stream with HIP events, so it overlaps
//     the rest of backward; ncclAvg does the 1/W);
//   * the first mark of an iteration queues a final callback on the autograd
//     engine; finalize() launches buckets whose params got no gradient,
//     joins every Work (RCCL: a stream-side wait, no host block), copies
//     compressed buckets back and checks every bucket fired exactly once.
//
// Collectives go through c10d::ProcessGroup, i.e. the same RCCL communicator
// torch.distributed("nccl") owns -- and gloo on the CPU test path, so the
// identical code runs in the 2-rank CPU tests.
#include <torch/extension.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <mutex>
#include <sstream>

namespace pmd {

class Reducer {
 public:
  Reducer(c10::intrusive_ptr<c10d::ProcessGroup> pg, at::Tensor grad_arena,
          std::vector<int64_t> bounds, std::vector<int64_t> param_bucket, bool use_avg,
          bool compress_bf16)
      : pg_(std::move(pg)),
        arena_(std::move(grad_arena)),
        bounds_(std::move(bounds)),
        param_bucket_(std::move(param_bucket)),
        use_avg_(use_avg),
        compress_(compress_bf16) {
    TORCH_CHECK(arena_.dim() == 1 && arena_.is_contiguous(), "grad arena must be a flat contiguous tensor");
    TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() == arena_.numel(),
                "bucket bounds must cover the arena");
    nb_ = static_cast<int>(bounds_.size()) - 1;
    world_ = pg_->getSize();
    pending0_.assign(nb_, 0);
    for (auto b : param_bucket_) {
      TORCH_CHECK(b >= 0 && b < nb_, "param bucket index out of range");
      pending0_[b]++;
    }
    for (int b = 0; b < nb_; ++b) TORCH_CHECK(pending0_[b] > 0, "bucket ", b, " has no parameters");
    works_.resize(nb_);
    wire_.resize(nb_);
    reset_();
  }

  // gradient of parameter i is final in the arena. Returns true if this call
  // launched a bucket.
  bool mark(int64_t i) {
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(i >= 0 && i < static_cast<int64_t>(param_bucket_.size()), "param index out of range");
    if (!enabled_ || marked_[i]) return false;
    marked_[i] = 1;
    if (!callback_queued_) {
      callback_queued_ = true;
      torch::autograd::Engine::get_default_engine().queue_callback([this] { this->finalize(); });
    }
    int b = static_cast<int>(param_bucket_[i]);
    if (--pending_[b] == 0) {
      launch_(b);
      return true;
    }
    return false;
  }

  void finalize() {
    std::lock_guard<std::mutex> lk(mu_);
    for (int b = 0; b < nb_; ++b)
      if (!works_[b]) launch_(b);  // params that produced no gradient this iteration
    for (int b = 0; b < nb_; ++b) works_[b]->wait();
    if (compress_) {
      for (int b = 0; b < nb_; ++b) slice_(b).copy_(wire_[b]);
    }
    std::vector<int> bad;
    for (int b = 0; b < nb_; ++b)
      if (fired_[b] != 1) bad.push_back(b);
    last_order_ = order_;
    reset_();
    iteration_++;
    if (!bad.empty()) {
      std::ostringstream os;
      for (int b : bad) os << b << " ";
      TORCH_CHECK(false, "reducer: buckets [", os.str(), "] did not fire exactly once this iteration");
    }
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

 private:
  at::Tensor slice_(int b) { return arena_.narrow(0, bounds_[b], bounds_[b + 1] - bounds_[b]); }

  void launch_(int b) {
    TORCH_CHECK(!works_[b], "reducer: bucket ", b, " launched twice in one iteration");
    fired_[b]++;
    order_.push_back(b);
    at::Tensor s = slice_(b);
    at::Tensor t = compress_ ? s.to(at::kBFloat16) : s;
    if (!use_avg_ && world_ > 1) t.mul_(1.0 / world_);
    c10d::AllreduceOptions opts;
    opts.reduceOp = use_avg_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
    std::vector<at::Tensor> ts{t};
    works_[b] = pg_->allreduce(ts, opts);
    if (compress_) wire_[b] = t;
  }

  void reset_() {
    pending_ = pending0_;
    marked_.assign(param_bucket_.size(), 0);
    fired_.assign(nb_, 0);
    for (auto& w : works_) w.reset();
    for (auto& w : wire_) w = at::Tensor();
    order_.clear();
    callback_queued_ = false;
  }

  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  at::Tensor arena_;
  std::vector<int64_t> bounds_, param_bucket_;
  bool use_avg_, compress_;
  int nb_ = 0, world_ = 1;
  std::vector<int> pending0_, pending_, fired_, order_, last_order_;
  std::vector<char> marked_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_;
  std::vector<at::Tensor> wire_;
  bool enabled_ = true, callback_queued_ = false;
  int64_t iteration_ = 0;
  std::mutex mu_;
};

void register_xgmi(pybind11::module& m);
void register_trace(pybind11::module& m);
void register_weights(pybind11::module& m);

void register_runtime(pybind11::module& m) {
  namespace py = pybind11;
  register_xgmi(m);
  register_trace(m);
  register_weights(m);
  py::class_<Reducer>(m, "Reducer")
      .def(py::init<c10::intrusive_ptr<c10d::ProcessGroup>, at::Tensor, std::vector<int64_t>,
                    std::vector<int64_t>, bool, bool>(),
           py::arg("process_group"), py::arg("grad_arena"), py::arg("bounds"), py::arg("param_bucket"),
           py::arg("use_avg"), py::arg("compress_bf16") = false)
      .def("mark", &Reducer::mark, py::arg("index"))
      .def("finalize", &Reducer::finalize)
      .def("set_enabled", &Reducer::set_enabled)
      .def_property_readonly("enabled", &Reducer::enabled)
      .def_property_readonly("iteration", &Reducer::iteration)
      .def_property_readonly("num_buckets", &Reducer::num_buckets)
      .def_property_readonly("bounds", &Reducer::bounds)
      .def("last_launch_order", &Reducer::last_launch_order);
}

}  // namespace pmd
