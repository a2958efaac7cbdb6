// roctx ranges / markers: named regions around forward,
// backward, communication and optimizer steps that rocprofv3
// --marker-trace records next to the kernel trace.
#include <torch/extension.h>
#include <rocprofiler-sdk-roctx/roctx.h>

namespace pmd {

void register_trace(pybind11::module& m) {
  m.def("roctx_push", [](const std::string& s) { return static_cast<int64_t>(roctxRangePushA(s.c_str())); });
  m.def("roctx_pop", []() { return static_cast<int64_t>(roctxRangePop()); });
  m.def("roctx_mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
}

}  // namespace pmd
