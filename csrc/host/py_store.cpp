// Python binding of the device state store's host runtime (ahv/store_host.h):
// argument conversion only — the transport, allocators and CPU twin live in
// `StoreCore`, which the host self test drives without Python.
#include "ahv/py_store_class.h"

namespace ahv {
namespace host {

using storebind::Store;
using storebind::I32Array;

void register_store(py::module_& m) {
  py::class_<Store>(m, "Store", "Device-authoritative governance state store (gfx950 worker or CPU twin)")
      .def(py::init<int, const py::dict&, const py::dict&, int64_t, int64_t, int64_t, int64_t, int64_t>(),
           py::arg("device"), py::arg("ptrs"), py::arg("caps"), py::arg("nslots") = 4096,
           py::arg("staging_bytes") = 1 << 22, py::arg("bulk_bytes") = 1 << 24, py::arg("idle_us") = 500,
           py::arg("max_ms") = 2000)
      .def("post", &Store::post, py::arg("op"), py::arg("args"), py::arg("inline") = py::none())
      .def("keep", &Store::keep, py::arg("seq"))
      .def("expect", &Store::expect, py::arg("seq"), py::arg("want"), py::arg("token"))
      .def("post_expect", &Store::post_expect, py::arg("op"), py::arg("args"), py::arg("inline"), py::arg("want"),
           py::arg("token"))
      .def("verify_expects", &Store::verify_expects, py::arg("block") = false)
      .def("n_expects", &Store::n_expects)
      .def("discard", &Store::discard, py::arg("seq"))
      .def("call", &Store::call, py::arg("op"), py::arg("args"), py::arg("nres") = 4, py::arg("inline") = py::none())
      .def("result", &Store::result, py::arg("seq"), py::arg("nres") = 4)
      .def("try_result", &Store::try_result, py::arg("seq"), py::arg("nres") = 4, py::arg("spin_ns") = 0)
      .def("drain", &Store::drain)
      .def("stage", &Store::stage)
      .def("bulk", &Store::bulk)
      .def("payload", &Store::payload)
      .def("write_payload", &Store::write_payload)
      .def("write_records", &Store::write_records)
      .def("payload_gather", &Store::payload_gather, py::arg("offs"), py::arg("lens"))
      .def("capture", &Store::capture, py::arg("slot"), py::arg("turn"), py::arg("ts_us"), py::arg("delta"),
           py::arg("parent") = py::none())
      .def("capture_bytes", &Store::capture_bytes, py::arg("slot"), py::arg("turn"), py::arg("ts_us"),
           py::arg("payload"), py::arg("null_at"), py::arg("parent") = py::none())
      .def_static("merkle_predict", &Store::merkle_predict)
      .def("restore_delta", &Store::restore_delta)
      .def("free_deltas", &Store::free_deltas)
      .def("free_deltas_arr", [](Store& st, I32Array a) { st.free_deltas(std::vector<int32_t>(a.data(), a.data() + a.size())); })
      .def("free_rows_arr", [](Store& st, uint64_t kind, I32Array a) {
        st.free_rows_cmd(kind, std::vector<int32_t>(a.data(), a.data() + a.size()));
      })
      .def("reserve_deltas", &Store::reserve_deltas)
      .def("alloc_row", &Store::alloc_row)
      .def("alloc_rows", &Store::alloc_rows)
      .def("release_row", &Store::release_row)
      .def("release_rows", &Store::release_rows)
      .def("release_list", &Store::release_list)
      .def("return_row", &Store::return_row)
      .def("reclaim_pool", &Store::reclaim_pool)
      .def("check_frees", &Store::check_frees, py::arg("block") = false)
      .def("npend", &Store::npend)
      .def("live_rows", &Store::live_rows)
      .def("set_row_cap", &Store::set_row_cap)
      .def("run_pipeline", &Store::run_pipeline)
      .def("run_template", &Store::run_template)
      .def("free_rows", &Store::free_rows_cmd)
      .def("quiesce", &Store::quiesce)
      .def("rebind", &Store::rebind_py)
      .def("grow_payload", &Store::grow_payload)
      .def("close", &Store::close)
      .def("info", &Store::info)
      .def("trace", &Store::trace)
      .def("set_timeout", &Store::set_timeout)
      .def_property_readonly("delta_live", &Store::delta_live)
      .def_property_readonly("payload_cap", &Store::payload_cap)
      .def_property_readonly("bulk_cap", &Store::bulk_cap)
      .def_property_readonly("payload_ptr", &Store::payload_ptr)
      .def_property_readonly("staging_cap", &Store::staging_cap)
      .def_property_readonly("gpu", &Store::gpu);
  py::dict ops;
#define AHV_OP(n) ops[#n] = static_cast<int>(ahv::store::n);
  AHV_OP(OP_NOP) AHV_OP(OP_STOP) AHV_OP(OP_FLUSH) AHV_OP(OP_ACQUIRE) AHV_OP(OP_FREE_ROWS) AHV_OP(OP_SESS_READ_MANY)
  AHV_OP(OP_V_RETIRE) AHV_OP(OP_SESS_CREATE) AHV_OP(OP_SESS_JOIN)
  AHV_OP(OP_SESS_LEAVE) AHV_OP(OP_SESS_ACTIVATE) AHV_OP(OP_SESS_TERMINATE) AHV_OP(OP_SESS_ARCHIVE)
  AHV_OP(OP_SESS_UPDATE_RING) AHV_OP(OP_SESS_SET_MODE) AHV_OP(OP_SESS_READ) AHV_OP(OP_SESS_SET_SIGMA)
  AHV_OP(OP_SESS_CLOSE) AHV_OP(OP_SESS_HANDSHAKE) AHV_OP(OP_DELTA_CAPTURE) AHV_OP(OP_DELTA_MERKLE)
  AHV_OP(OP_DELTA_VERIFY) AHV_OP(OP_DELTA_READ) AHV_OP(OP_VOUCH) AHV_OP(OP_SIGMA_EFF) AHV_OP(OP_EXPOSURE)
  AHV_OP(OP_RELEASE_BOND) AHV_OP(OP_RELEASE_SESSION) AHV_OP(OP_VOUCH_LIST) AHV_OP(OP_EDGE_READ) AHV_OP(OP_SLASH)
  AHV_OP(OP_SAGA_CREATE) AHV_OP(OP_STEP_READ)
  AHV_OP(OP_STEP_ADD) AHV_OP(OP_STEP_TRANSITION) AHV_OP(OP_STEP_SET) AHV_OP(OP_SAGA_TRANSITION)
  AHV_OP(OP_SAGA_READ) AHV_OP(OP_SAGA_PLAN)
#undef AHV_OP
  m.attr("STORE_OPS") = ops;
  m.attr("STORE_HDR_WORDS") = static_cast<int>(ahv::store::kHdrWords);
  py::list cols;
#define AHV_COL(name, type, ext) cols.append(py::make_tuple(#name, #type, #ext));
  AHV_STORE_COLUMNS(AHV_COL)
#undef AHV_COL
  m.attr("STORE_COLUMNS") = cols;
}

}  // namespace host
}  // namespace ahv
