// Host side of the one-shot xGMI all-reduce (kernels/xgmi.hip, K21).
//
// Each rank owns one receive buffer in uncached device memory
// (hipExtMallocWithFlags(hipDeviceMallocUncached): peers write it over xGMI
// and the owner polls it, with no cache maintenance).  Buffers are exported
// with hipIpcGetMemHandle; the 64-byte handles are exchanged by the Python
// wrapper through the c10d store (parallel/xgmi.py) and opened here with
// hipIpcOpenMemHandle, giving every rank the pointer table the kernel writes
// through.  Everything runs on the caller's current HIP stream; nothing
// blocks the host except check().
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <cstring>

#include "kernels/launchers.h"

namespace pmd {

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));                 \
  } while (0)

class XgmiComm {
 public:
  XgmiComm(int64_t rank, int64_t world, int64_t device, double timeout_s)
      : rank_(rank), world_(world), device_(device) {
    TORCH_CHECK(world >= 1 && world <= kXgmiMaxRanks, "xgmi: world size must be 1..", kXgmiMaxRanks);
    TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device));
    bytes_ = (size_t)kXgmiFlagBytes + sizeof(float) * 2 * (size_t)world * kXgmiCap;
    HIP_OK(hipExtMallocWithFlags(&buf_, bytes_, hipDeviceMallocUncached));
    HIP_OK(hipMemset(buf_, 0, bytes_));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&epochs_), sizeof(uint32_t) * (kXgmiMaxBlocks + 1)));
    HIP_OK(hipMemset(epochs_, 0, sizeof(uint32_t) * (kXgmiMaxBlocks + 1)));
    err_ = epochs_ + kXgmiMaxBlocks;
    // host-mapped error word: the kernels set it on a timeout, the training loop
    // reads it after every step with no device synchronisation
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&err_host_), sizeof(uint32_t),
                         hipHostMallocMapped | hipHostMallocCoherent));
    *err_host_ = 0;
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_host_dev_), err_host_, 0));
    HIP_OK(hipDeviceSynchronize());
    peers_.assign(world, nullptr);
    peers_[rank] = buf_;
    // the spin deadline is in ticks of the constant wall clock (s_memrealtime)
    int khz = 0;
    HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, (int)device));
    wall_khz_ = khz > 0 ? khz : 100000;
    set_timeout(timeout_s);
  }

  // the control block every launch passes (epochs, error words, ordering, test-only skew)
  XgmiCtl ctl() const {
    XgmiCtl c{};
    c.epochs = epochs_;
    c.err = err_;
    c.err_host = err_host_dev_;
    c.timeout_ticks = timeout_ticks_;
    c.order = order_;
    c.delay_where = delay_where_;
    c.delay_ticks = delay_ticks_;
    c.ar_region = ar_region_;
    return c;
  }

  // memory ordering of the exchange: 0 light (completion-only publish), 1 strict
  // (system release fence before each flag, acquire fence after each match).  Every rank
  // must use the same value; parallel/xgmi.py picks it with the stress self-test.
  void set_order(int64_t order) {
    TORCH_CHECK(order == 0 || order == 1, "xgmi: order must be 0 (light) or 1 (strict)");
    order_ = (int)order;
  }
  int64_t order() const { return order_; }

  // TEST-ONLY skew injection: every following call of THIS rank idles `seconds` at `where`
  // (1 before publishing, 2 after the flags matched, before reading); where 0 = off.
  void set_debug_delay(double seconds, int64_t where) {
    TORCH_CHECK(where >= 0 && where <= 2 && seconds >= 0, "xgmi: bad debug delay");
    delay_where_ = (int)where;
    delay_ticks_ = static_cast<unsigned long long>(seconds * 1000.0 * wall_khz_);
  }
  // TEST-ONLY: floats per block of the plain all-reduce (0 = the shared map's kXgmiChunk);
  // 2048 reproduces round 4's split map (the negative control of the interleaving test)
  void set_ar_region(int64_t floats) {
    TORCH_CHECK(floats == 0 || (floats >= 256 && floats <= kXgmiCap && floats % 256 == 0), "xgmi: bad region");
    ar_region_ = (int)floats;
  }

  // clear both error words (host-synchronising; collective use only, after a failed self-test
  // whose peers have all finished: the epochs stay aligned, every rank ran every call)
  void reset_error() {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemset(err_, 0, sizeof(uint32_t)));
    __atomic_store_n(err_host_, 0u, __ATOMIC_RELEASE);
    HIP_OK(hipDeviceSynchronize());
  }

  void set_timeout(double timeout_s) {
    TORCH_CHECK(timeout_s > 0, "xgmi: timeout must be positive");
    timeout_s_ = timeout_s;
    timeout_ticks_ = static_cast<unsigned long long>(timeout_s * 1000.0 * wall_khz_);
  }
  double timeout() const { return timeout_s_; }
  int64_t wall_clock_khz() const { return wall_khz_; }

  // non-blocking: has any kernel (that finished so far) timed out on a peer?
  bool failed() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) != 0; }

  ~XgmiComm() {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && peers_[r]) (void)hipIpcCloseMemHandle(peers_[r]);
    if (buf_) (void)hipFree(buf_);
    if (epochs_) (void)hipFree(epochs_);
    if (err_host_) (void)hipHostFree(err_host_);
  }

  pybind11::bytes handle() {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    hipIpcMemHandle_t h;
    HIP_OK(hipIpcGetMemHandle(&h, buf_));
    return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK(static_cast<int64_t>(handles.size()) == world_, "xgmi: need one handle per rank");
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "xgmi: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      HIP_OK(hipIpcOpenMemHandle(&peers_[r], h, hipIpcMemLazyEnablePeerAccess));
    }
    opened_ = true;
  }

  // in-place SUM over ranks of a contiguous fp32 GPU tensor (<= capacity())
  at::Tensor all_reduce_(at::Tensor x) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi: open() the peer handles first");
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(),
                "xgmi: expects a contiguous fp32 GPU tensor");
    TORCH_CHECK(x.get_device() == device_, "xgmi: tensor on the wrong device");
    TORCH_CHECK(x.numel() <= kXgmiCap, "xgmi: message of ", x.numel(), " floats exceeds capacity ",
                kXgmiCap);
    float* data[kXgmiMaxRanks];
    uint32_t* flags[kXgmiMaxRanks];
    for (int r = 0; r < world_; ++r) {
      flags[r] = reinterpret_cast<uint32_t*>(peers_[r]);
      data[r] = reinterpret_cast<float*>(static_cast<char*>(peers_[r]) + kXgmiFlagBytes);
    }
    c10::DeviceGuard g(x.device());
    const int rc = xgmi_allreduce_launch(data, flags, x.data_ptr<float>(), static_cast<int>(x.numel()),
                                         rank_, world_, ctl(), c10::hip::getCurrentHIPStream().stream());
    TORCH_CHECK(rc == 0, "xgmi: launch rejected");
    calls_++;
    return x;
  }

  // SyncBN fused statistics exchange (see xgmi_bn_kernel).  Forward (mode 0):
  // slots -> params_a/params_b [4][C], running stats, nbt, count_out [1].
  // Backward (mode 1): slots -> acc_* += local sums, out_a/out_b [2][C] global.
  void bn_(int64_t mode, at::Tensor slots_a, c10::optional<at::Tensor> slots_b, double count,
           c10::optional<at::Tensor> gamma_a, c10::optional<at::Tensor> beta_a,
           c10::optional<at::Tensor> params_a, c10::optional<at::Tensor> rm_a,
           c10::optional<at::Tensor> rv_a, c10::optional<at::Tensor> nbt_a, double eps_a, double mom_a,
           c10::optional<at::Tensor> gamma_b, c10::optional<at::Tensor> beta_b,
           c10::optional<at::Tensor> params_b, c10::optional<at::Tensor> rm_b,
           c10::optional<at::Tensor> rv_b, c10::optional<at::Tensor> nbt_b, double eps_b, double mom_b,
           c10::optional<at::Tensor> count_out, c10::optional<at::Tensor> acc_a0,
           c10::optional<at::Tensor> acc_a1, c10::optional<at::Tensor> acc_b0,
           c10::optional<at::Tensor> acc_b1, c10::optional<at::Tensor> out_a,
           c10::optional<at::Tensor> out_b, c10::optional<at::Tensor> shift_a,
           c10::optional<at::Tensor> shift_b) {
    TORCH_CHECK(opened_ || world_ == 1, "xgmi: open() the peer handles first");
    auto fptr = [](const c10::optional<at::Tensor>& t) -> float* {
      if (!t || !t->defined()) return nullptr;
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->is_cuda(),
                  "xgmi bn: fp32 contiguous GPU tensors expected");
      return t->data_ptr<float>();
    };
    TORCH_CHECK(slots_a.scalar_type() == at::kFloat && slots_a.is_contiguous() && slots_a.dim() == 3 &&
                    slots_a.size(0) == 64 && slots_a.size(1) == 2, "xgmi bn: slots must be [64, 2, C]");
    pmd::XgmiBnArgs a{};
    a.mode = (int)mode;
    a.slotsA = slots_a.data_ptr<float>();
    a.CA = (int)slots_a.size(2);
    const bool hasB = slots_b && slots_b->defined();
    if (hasB) {
      TORCH_CHECK(slots_b->dim() == 3 && slots_b->size(0) == 64 && slots_b->size(1) == 2 &&
                  slots_b->is_contiguous(), "xgmi bn: slots_b must be [64, 2, C]");
      a.slotsB = slots_b->data_ptr<float>();
      a.CB = (int)slots_b->size(2);
    }
    a.count = (float)count;
    auto fin = [&](pmd::BnFinalizeOut& o, const c10::optional<at::Tensor>& g, const c10::optional<at::Tensor>& bt,
                   const c10::optional<at::Tensor>& pr, const c10::optional<at::Tensor>& rm,
                   const c10::optional<at::Tensor>& rv, const c10::optional<at::Tensor>& nbt, double eps,
                   double mom, int C, const c10::optional<at::Tensor>& shift) {
      o.gamma = fptr(g);
      o.beta = fptr(bt);
      o.params = fptr(pr);
      TORCH_CHECK(o.gamma && o.beta && o.params && pr->numel() == 4 * C, "xgmi bn fwd: gamma/beta/params");
      o.rm = fptr(rm);
      o.rv = fptr(rv);
      o.nbt = (nbt && nbt->defined()) ? reinterpret_cast<long long*>(nbt->data_ptr<int64_t>()) : nullptr;
      o.eps = (float)eps;
      o.momentum = (float)mom;
      o.shift = fptr(shift);  // statistics shift K [C]: every rank must pass the same values
      TORCH_CHECK(!o.shift || shift->numel() == C, "xgmi bn fwd: shift must be [C]");
    };
    if (mode == 0) {
      fin(a.fA, gamma_a, beta_a, params_a, rm_a, rv_a, nbt_a, eps_a, mom_a, a.CA, shift_a);
      if (hasB) fin(a.fB, gamma_b, beta_b, params_b, rm_b, rv_b, nbt_b, eps_b, mom_b, a.CB, shift_b);
      a.count_out = fptr(count_out);
    } else {
      a.accA0 = fptr(acc_a0);
      a.accA1 = fptr(acc_a1);
      a.accB0 = fptr(acc_b0);
      a.accB1 = fptr(acc_b1);
      a.outA = fptr(out_a);
      a.outB = fptr(out_b);
      TORCH_CHECK(a.outA && out_a->numel() == 2 * a.CA && (!hasB || (a.outB && out_b->numel() == 2 * a.CB)),
                  "xgmi bn bwd: out tensors [2, C]");
    }
    float* data[kXgmiMaxRanks];
    uint32_t* flags[kXgmiMaxRanks];
    for (int r = 0; r < world_; ++r) {
      flags[r] = reinterpret_cast<uint32_t*>(peers_[r]);
      data[r] = reinterpret_cast<float*>(static_cast<char*>(peers_[r]) + kXgmiFlagBytes);
    }
    c10::DeviceGuard g(slots_a.device());
    const int rc = xgmi_bn_launch(data, flags, a, rank_, world_, ctl(), c10::hip::getCurrentHIPStream().stream());
    TORCH_CHECK(rc == 0, "xgmi bn: launch rejected (", rc, ")");
    calls_++;
  }

  // ---- compact per-step entry points (the host path of 106 (R50) / 310 (R152) SyncBN
  // exchanges per step): a BN module's persistent tensors (gamma, beta, running stats,
  // num_batches_tracked -- the Parameter / buffer objects themselves, so a flat-arena
  // relayout that re-points their storage is followed) are registered ONCE as a site;
  // each exchange then passes only its per-step tensors.
  int64_t add_site(at::Tensor gamma, at::Tensor beta, c10::optional<at::Tensor> rm, c10::optional<at::Tensor> rv,
                   c10::optional<at::Tensor> nbt, double eps, double momentum) {
    Site st;
    st.gamma = gamma;
    st.beta = beta;
    st.rm = rm && rm->defined() ? *rm : at::Tensor();
    st.rv = rv && rv->defined() ? *rv : at::Tensor();
    st.nbt = nbt && nbt->defined() ? *nbt : at::Tensor();
    st.eps = (float)eps;
    st.mom = (float)momentum;
    sites_.push_back(st);
    return (int64_t)sites_.size() - 1;
  }

  void bn_fwd(at::Tensor slots_a, c10::optional<at::Tensor> slots_b, double count, int64_t site_a, int64_t site_b,
              at::Tensor params_a, c10::optional<at::Tensor> params_b, at::Tensor count_out,
              c10::optional<at::Tensor> shift_a, c10::optional<at::Tensor> shift_b) {
    TORCH_CHECK(site_a >= 0 && site_a < (int64_t)sites_.size() && site_b < (int64_t)sites_.size(),
                "xgmi bn: unknown site");
    const Site& A = sites_[site_a];
    auto opt = [](const at::Tensor& t) { return t.defined() ? c10::optional<at::Tensor>(t) : c10::nullopt; };
    if (site_b < 0) {
      bn_(0, slots_a, c10::nullopt, count, A.gamma, A.beta, params_a, opt(A.rm), opt(A.rv), opt(A.nbt), A.eps,
          A.mom, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, 1e-5, 0.1,
          count_out, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, shift_a,
          c10::nullopt);
    } else {
      const Site& B = sites_[site_b];
      bn_(0, slots_a, slots_b, count, A.gamma, A.beta, params_a, opt(A.rm), opt(A.rv), opt(A.nbt), A.eps, A.mom,
          B.gamma, B.beta, params_b, opt(B.rm), opt(B.rv), opt(B.nbt), B.eps, B.mom, count_out, c10::nullopt,
          c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, shift_a, shift_b);
    }
  }

  void bn_bwd(at::Tensor slots_a, c10::optional<at::Tensor> slots_b, c10::optional<at::Tensor> acc_a0,
              c10::optional<at::Tensor> acc_a1, c10::optional<at::Tensor> acc_b0,
              c10::optional<at::Tensor> acc_b1, at::Tensor out_a, c10::optional<at::Tensor> out_b) {
    bn_(1, slots_a, slots_b, 0.0, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt,
        c10::nullopt, 1e-5, 0.1, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt,
        c10::nullopt, 1e-5, 0.1, c10::nullopt, acc_a0, acc_a1, acc_b0, acc_b1, out_a, out_b, c10::nullopt,
        c10::nullopt);
  }

  // host-blocking: did any call time out waiting for a peer?
  bool check() {
    c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, device_));
    uint32_t e = 0;
    HIP_OK(hipMemcpy(&e, err_, sizeof(e), hipMemcpyDeviceToHost));
    return e == 0;
  }

  int64_t capacity() const { return kXgmiCap; }
  int64_t calls() const { return calls_; }

 private:
  int rank_, world_, device_;
  size_t bytes_ = 0;
  void* buf_ = nullptr;
  uint32_t* epochs_ = nullptr;
  uint32_t* err_ = nullptr;
  std::vector<void*> peers_;
  uint32_t* err_host_ = nullptr;      // host view of the mapped error word
  uint32_t* err_host_dev_ = nullptr;  // device view of the same word
  unsigned long long timeout_ticks_ = 0;
  double timeout_s_ = 0.0;
  int64_t wall_khz_ = 100000;
  int order_ = 0;
  int delay_where_ = 0;
  unsigned long long delay_ticks_ = 0;
  int ar_region_ = 0;
  bool opened_ = false;
  int64_t calls_ = 0;
  struct Site {
    at::Tensor gamma, beta, rm, rv, nbt;
    float eps = 1e-5f, mom = 0.1f;
  };
  std::vector<Site> sites_;
};

void register_xgmi(pybind11::module& m) {
  m.def("xgmi_set_bn_pairs", &pmd::xgmi_set_bn_pairs,
        "fused SyncBN kernel: channel pairs per block (1..255)");
  namespace py = pybind11;
  py::class_<XgmiComm>(m, "XgmiComm")
      .def(py::init<int64_t, int64_t, int64_t, double>(), py::arg("rank"), py::arg("world"),
           py::arg("device"), py::arg("timeout_s") = 60.0)
      .def("handle", &XgmiComm::handle)
      .def("open", &XgmiComm::open)
      .def("all_reduce_", &XgmiComm::all_reduce_)
      .def("bn_", &XgmiComm::bn_)
      .def("add_site", &XgmiComm::add_site)
      .def("bn_fwd", &XgmiComm::bn_fwd)
      .def("bn_bwd", &XgmiComm::bn_bwd)
      .def("check", &XgmiComm::check)
      .def("failed", &XgmiComm::failed)
      .def("set_timeout", &XgmiComm::set_timeout, py::arg("timeout_s"))
      .def("set_order", &XgmiComm::set_order, py::arg("order"))
      .def_property_readonly("order", &XgmiComm::order)
      .def("set_debug_delay", &XgmiComm::set_debug_delay, py::arg("seconds"), py::arg("where"))
      .def("set_ar_region", &XgmiComm::set_ar_region, py::arg("floats"))
      .def("reset_error", &XgmiComm::reset_error)
      .def_property_readonly("timeout", &XgmiComm::timeout)
      .def_property_readonly("wall_clock_khz", &XgmiComm::wall_clock_khz)
      .def_property_readonly("capacity", &XgmiComm::capacity)
      .def_property_readonly("calls", &XgmiComm::calls);
}

}  // namespace pmd
