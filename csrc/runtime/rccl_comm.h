// Native RCCL communicator.
//
// The reference reaches NCCL only through torch's ProcessGroupNCCL
// (reference main.py:190-193 -> dist.init_process_group('nccl')).  Here the
// gradient path owns its communicator directly:
//   * bootstrap: rank 0 calls ncclGetUniqueId; the 128-byte id travels through
//     the c10d TCPStore that init_process_group already created (Python side,
//     parallel/rccl.py); every rank then calls ncclCommInitRank on its own HIP
//     device.  The store is the only thing borrowed from c10d.
//   * one communication stream per communicator, created with an explicit
//     priority, so the number of HIP streams a rank uses -- and therefore how
//     they map onto GPU_MAX_HW_QUEUES hardware queues -- is fixed and known
//     (docs/ARCHITECTURE.md, "Streams").
//   * every collective is fenced with HIP events: it waits for the caller's
//     current stream at the point of issue and returns an event the consumer
//     stream waits on (no host blocking anywhere on the hot path).
//   * abort(): ncclCommAbort, so a failing rank unblocks its peers; check()
//     surfaces asynchronous RCCL errors.
//   * the communicator is NON-BLOCKING (ncclConfig_t.blocking = 0) so that its init is
//     bounded in wall time (a peer that failed before joining cannot hang this rank); calls
//     that answer ncclInProgress are settled by polling ncclCommGetAsyncError.
#pragma once
#include <torch/extension.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

namespace pmd {

class RcclComm {
 public:
  // 128-byte ncclUniqueId (call on ONE rank, share through the store)
  static std::string unique_id();

  // stream: an existing HIP stream handle to run the collectives on (the rank's step
  // streams are created up front, ops/functional.py init_step_streams), 0 = create one
  // init_timeout_s: wall-time bound of the (non-blocking) ncclCommInitRankConfig; <= 0 = unbounded
  RcclComm(const std::string& uid, int64_t rank, int64_t world, int64_t device, int64_t priority,
           int64_t stream = 0, double init_timeout_s = 300.0);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // In-place all-reduce of `t` on the communication stream, ordered after all
  // work already issued on the caller's current stream.  op: 0 sum, 1 avg.
  // Returns an event recorded on the communication stream after the collective.
  hipEvent_t all_reduce_async(const at::Tensor& t, int op);
  // same, recording the caller-owned event `done` (the reducer keeps one per bucket)
  // (optionally also `start`, recorded on the communication stream right before it)
  void all_reduce_record(const at::Tensor& t, int op, hipEvent_t done, hipEvent_t start = nullptr);
  // all_reduce_async + make the caller's current stream wait for it
  void all_reduce_(const at::Tensor& t, int64_t op);
  void broadcast_(const at::Tensor& t, int64_t root);
  // current stream waits for `ev` (recorded by all_reduce_async)
  void wait(hipEvent_t ev);

  // asynchronous RCCL error state (ncclCommGetAsyncError); true when healthy
  bool check();
  void abort();

  int64_t rank() const { return rank_; }
  int64_t world() const { return world_; }
  int64_t device() const { return device_; }
  int64_t calls() const { return calls_; }
  hipStream_t stream() const { return stream_; }
  uintptr_t stream_handle() const { return reinterpret_cast<uintptr_t>(stream_); }

 private:
  hipEvent_t next_event_();
  void fence_in_();
  ncclResult_t settle_();   // wait out ncclInProgress of the non-blocking communicator

  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  bool owns_stream_ = true;
  hipEvent_t in_ev_ = nullptr;
  std::vector<hipEvent_t> ring_;  // done-events, reused round robin
  size_t ring_pos_ = 0;
  int64_t rank_ = 0, world_ = 1, device_ = 0, calls_ = 0;
  bool aborted_ = false;
};

}  // namespace pmd
