// Python extension entry point: agent_hypervisor_amd._C
//
// One shared object holds the host runtime (scalar audit path, interner, time
// base) and the gfx950 kernel library with its launchers.  Every source file
// under csrc/ is compiled by hipcc --offload-arch=gfx950 (see
// agent_hypervisor_amd/utils/build.py).
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace ahv {
namespace host {
void register_audit(py::module_& m);
void register_runtime(py::module_& m);
void register_kernels(py::module_& m);
void register_comm(py::module_& m);
void register_store(py::module_& m);
void register_global_liability(py::module_& m);
void register_merkle_tree(py::module_& m);
void register_store_views(py::module_& m);
void register_control(py::module_& m);
}  // namespace host
}  // namespace ahv

PYBIND11_MODULE(_C, m) {
  m.doc() = "agent-hypervisor MI355X native core (host runtime + gfx950 kernels)";
  m.attr("OFFLOAD_ARCH") = "gfx950";
  ahv::host::register_audit(m);
  ahv::host::register_runtime(m);
  ahv::host::register_kernels(m);
  ahv::host::register_comm(m);
  ahv::host::register_store(m);
  ahv::host::register_global_liability(m);
  ahv::host::register_merkle_tree(m);
  ahv::host::register_store_views(m);
  ahv::host::register_control(m);
}
