// Cross-stream fork / join points of the training step (main stream <-> the
// weight-gradient side stream, both on ONE device) as a pooled ring of HIP
// events whose fence scope is chosen at construction:
//   mode 0: hipEventDisableTiming only -- torch.cuda.Event's behaviour: the
//           recorded marker carries a SYSTEM-scope release (L2 writeback for the
//           host / peer devices) that the main stream pays between two kernels;
//   mode 1: + hipEventDisableSystemFence;
//   mode 2: + hipEventReleaseToDevice (device-scope release).
// Both streams live on the same device and every kernel already ends with the
// device-scope release the next same-device consumer needs, so the system-scope
// part buys nothing here (host- and peer-visible points -- bucket launches,
// host syncs -- keep torch's own events).  hipStreamWaitEvent snapshots the
// event's current recording when it is enqueued, so a slot can be re-recorded
// once its waits are queued; the ring only has to outlive a deferred join
// (a few blocks of one backward).
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <vector>

namespace pmd {

class StreamEvents {
 public:
  StreamEvents(int64_t n, int64_t mode, int64_t device) : mode_((int)mode) {
    TORCH_CHECK(n >= 2 && n <= 4096, "stream events: ring size 2..4096");
    TORCH_CHECK(mode >= 0 && mode <= 2, "stream events: mode 0..2");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
    unsigned flags = hipEventDisableTiming;
    if (mode == 1) flags |= hipEventDisableSystemFence;
    if (mode == 2) flags |= hipEventReleaseToDevice;
    ev_.resize(n, nullptr);
    for (auto& e : ev_) TORCH_CHECK(hipEventCreateWithFlags(&e, flags) == hipSuccess, "stream events: create");
  }
  ~StreamEvents() {
    for (auto e : ev_)
      if (e) (void)hipEventDestroy(e);
  }
  StreamEvents(const StreamEvents&) = delete;
  StreamEvents& operator=(const StreamEvents&) = delete;

  // record the next ring slot on `stream` (a hipStream_t as an integer); returns the slot
  int64_t record(int64_t stream) {
    const int64_t s = next_;
    next_ = (next_ + 1) % (int64_t)ev_.size();
    TORCH_CHECK(hipEventRecord(ev_[s], reinterpret_cast<hipStream_t>(stream)) == hipSuccess,
                "stream events: record");
    records_++;
    return s;
  }

  // make `stream` wait for slot's current recording
  void wait(int64_t stream, int64_t slot) {
    TORCH_CHECK(slot >= 0 && slot < (int64_t)ev_.size(), "stream events: slot");
    TORCH_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), ev_[slot], 0) == hipSuccess,
                "stream events: wait");
  }

  // `to` waits for everything issued so far on `from`
  void fork(int64_t from, int64_t to) { wait(to, record(from)); }

  bool query(int64_t slot) {
    TORCH_CHECK(slot >= 0 && slot < (int64_t)ev_.size(), "stream events: slot");
    return hipEventQuery(ev_[slot]) == hipSuccess;
  }

  int64_t mode() const { return mode_; }
  int64_t records() const { return records_; }

 private:
  std::vector<hipEvent_t> ev_;
  int64_t next_ = 0, records_ = 0;
  int mode_;
};

void register_events(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<StreamEvents>(m, "StreamEvents")
      .def(py::init<int64_t, int64_t, int64_t>(), py::arg("n"), py::arg("mode"), py::arg("device"))
      .def("record", &StreamEvents::record, py::arg("stream"))
      .def("wait", &StreamEvents::wait, py::arg("stream"), py::arg("slot"))
      .def("fork", &StreamEvents::fork, py::arg("from_stream"), py::arg("to_stream"))
      .def("query", &StreamEvents::query, py::arg("slot"))
      .def_property_readonly("mode", &StreamEvents::mode)
      .def_property_readonly("records", &StreamEvents::records);
}

}  // namespace pmd
