#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace ahv { namespace host {
void register_kernels(py::module_& m) { (void)m; }
}}
