// Native RCCL communicator: see rccl_comm.h.
#include "runtime/rccl_comm.h"

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <chrono>
#include <cstring>
#include <thread>

namespace pmd {

#define RCCL_OK(x)                                                                   \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    TORCH_CHECK(r_ == ncclSuccess, #x " failed: ", ncclGetErrorString(r_));           \
  } while (0)
// A non-blocking communicator (below) may answer ncclInProgress while it finishes work it
// started in the background (the first collective's connection setup): poll its async state
// until it settles, then check it
#define RCCL_CALL(x)                                                                 \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ == ncclInProgress) r_ = settle_();                                        \
    TORCH_CHECK(r_ == ncclSuccess, #x " failed: ", ncclGetErrorString(r_));           \
  } while (0)
#define HIP_OK2(x)                                                                   \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));             \
  } while (0)

static ncclDataType_t nccl_dtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t);
  }
  return ncclFloat32;
}

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  RCCL_OK(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(const std::string& uid, int64_t rank, int64_t world, int64_t device, int64_t priority,
                   int64_t stream, double init_timeout_s)
    : rank_(rank), world_(world), device_(device) {
  TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "rccl: unique id must be ", NCCL_UNIQUE_ID_BYTES,
              " bytes");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl: bad rank/world");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device));
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  // NON-BLOCKING init bounded in wall time: a peer that never arrives (it failed before its
  // own init) must not leave this rank stuck inside ncclCommInitRank -- on the deadline the
  // half-built communicator is aborted and the constructor throws (parallel/rccl.py then
  // agrees the failure with every rank and falls back to c10d)
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&comm_, (int)world, id, (int)rank, &cfg);
  if (r == ncclInProgress || r == ncclSuccess) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      ncclResult_t ae = ncclSuccess;
      r = comm_ ? ncclCommGetAsyncError(comm_, &ae) : ncclInternalError;
      if (r == ncclSuccess) r = ae;
      if (r != ncclInProgress) break;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (init_timeout_s > 0 && el > init_timeout_s) {
        (void)ncclCommAbort(comm_);
        comm_ = nullptr;
        TORCH_CHECK(false, "rccl: ncclCommInitRank did not complete within ", init_timeout_s,
                    " s (a peer rank never joined); communicator aborted");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }
  if (r != ncclSuccess) {
    if (comm_) (void)ncclCommAbort(comm_);
    comm_ = nullptr;
    TORCH_CHECK(false, "rccl: ncclCommInitRankConfig failed: ", ncclGetErrorString(r));
  }
  if (stream) {
    stream_ = reinterpret_cast<hipStream_t>(stream);
    owns_stream_ = false;
  } else {
    HIP_OK2(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, (int)priority));
  }
  HIP_OK2(hipEventCreateWithFlags(&in_ev_, hipEventDisableTiming));
  ring_.resize(64);
  for (auto& e : ring_) HIP_OK2(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

RcclComm::~RcclComm() {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
  if (comm_) {
    if (aborted_) {
      // already torn down by abort()
    } else {
      (void)hipStreamSynchronize(stream_);
      // non-blocking communicator: finalize, let it settle (bounded), then destroy
      if (ncclCommFinalize(comm_) == ncclInProgress) {
        const auto t0 = std::chrono::steady_clock::now();
        ncclResult_t ae = ncclInProgress;
        while (ae == ncclInProgress &&
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 30.0) {
          if (ncclCommGetAsyncError(comm_, &ae) != ncclSuccess) break;
          std::this_thread::yield();
        }
      }
      (void)ncclCommDestroy(comm_);
    }
  }
  for (auto& e : ring_) (void)hipEventDestroy(e);
  if (in_ev_) (void)hipEventDestroy(in_ev_);
  if (stream_ && owns_stream_) (void)hipStreamDestroy(stream_);
}

ncclResult_t RcclComm::settle_() {
  ncclResult_t ae = ncclInProgress;
  const auto t0 = std::chrono::steady_clock::now();
  while (ae == ncclInProgress) {
    ncclResult_t r = ncclCommGetAsyncError(comm_, &ae);
    if (r != ncclSuccess) return r;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 600.0) return ncclInternalError;
    if (ae == ncclInProgress) std::this_thread::yield();
  }
  return ae;
}

hipEvent_t RcclComm::next_event_() {
  hipEvent_t e = ring_[ring_pos_];
  ring_pos_ = (ring_pos_ + 1) % ring_.size();
  return e;
}

void RcclComm::fence_in_() {
  // the collective starts after everything already issued on the caller's stream
  hipStream_t cur = c10::hip::getCurrentHIPStream().stream();
  HIP_OK2(hipEventRecord(in_ev_, cur));
  HIP_OK2(hipStreamWaitEvent(stream_, in_ev_, 0));
}

hipEvent_t RcclComm::all_reduce_async(const at::Tensor& t, int op) {
  hipEvent_t done = next_event_();
  all_reduce_record(t, op, done);
  return done;
}

void RcclComm::all_reduce_record(const at::Tensor& t, int op, hipEvent_t done, hipEvent_t start) {
  TORCH_CHECK(!aborted_, "rccl: communicator was aborted");
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.get_device() == device_,
              "rccl: contiguous tensor on this rank's device expected");
  c10::DeviceGuard g(t.device());
  fence_in_();
  if (start) HIP_OK2(hipEventRecord(start, stream_));
  RCCL_CALL(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t.scalar_type()),
                          op == 1 ? ncclAvg : ncclSum, comm_, stream_));
  HIP_OK2(hipEventRecord(done, stream_));
  calls_++;
}

void RcclComm::wait(hipEvent_t ev) {
  HIP_OK2(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), ev, 0));
}

void RcclComm::all_reduce_(const at::Tensor& t, int64_t op) {
  wait(all_reduce_async(t, (int)op));
}

void RcclComm::broadcast_(const at::Tensor& t, int64_t root) {
  TORCH_CHECK(!aborted_, "rccl: communicator was aborted");
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.get_device() == device_,
              "rccl: contiguous tensor on this rank's device expected");
  c10::DeviceGuard g(t.device());
  fence_in_();
  RCCL_CALL(ncclBroadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), nccl_dtype(t.scalar_type()),
                          (int)root, comm_, stream_));
  hipEvent_t done = next_event_();
  HIP_OK2(hipEventRecord(done, stream_));
  wait(done);
  calls_++;
}

bool RcclComm::check() {
  if (aborted_ || !comm_) return false;
  ncclResult_t ae = ncclSuccess;
  RCCL_OK(ncclCommGetAsyncError(comm_, &ae));
  return ae == ncclSuccess || ae == ncclInProgress;
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    aborted_ = true;
    (void)ncclCommAbort(comm_);
  }
}

void register_rccl(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<RcclComm>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def(py::init<const std::string&, int64_t, int64_t, int64_t, int64_t, int64_t, double>(),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("priority") = 0,
           py::arg("stream") = 0, py::arg("init_timeout_s") = 300.0)
      .def("all_reduce_", &RcclComm::all_reduce_, py::arg("tensor"), py::arg("op") = 0)
      .def("broadcast_", &RcclComm::broadcast_, py::arg("tensor"), py::arg("root") = 0)
      .def("check", &RcclComm::check)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("calls", &RcclComm::calls)
      .def_property_readonly("stream_handle", &RcclComm::stream_handle);
}

}  // namespace pmd
