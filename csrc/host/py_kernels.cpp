// Python bindings of the gfx950 kernel launchers and their host twins.
//
// Tensors are owned by PyTorch (device-resident SoA tables, see
// agent_hypervisor_amd/models/tables.py); Python passes raw data pointers, the
// current HIP stream, and scalar arguments in a dict.  Shape/dtype validation is
// done by the Python wrappers in agent_hypervisor_amd/ops/, which fail loudly.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ahv/launch.h"
#include "ahv/pipeline.h"

namespace py = pybind11;

namespace ahv {
namespace host {

template <class T>
static T* ptr(const py::dict& d, const char* k) {
  if (!d.contains(k)) throw py::key_error(std::string("missing pointer argument: ") + k);
  py::object v = d[k];
  if (v.is_none()) return nullptr;
  return reinterpret_cast<T*>(v.cast<uintptr_t>());
}

template <class T>
static T val(const py::dict& d, const char* k) {
  if (!d.contains(k)) throw py::key_error(std::string("missing scalar argument: ") + k);
  return d[k].cast<T>();
}

static PipelineArgs pipeline_args(const py::dict& d) {
  PipelineArgs a{};
  a.n = val<int64_t>(d, "n");
  a.slot_base = val<int64_t>(d, "slot_base");
  a.capacity = val<int64_t>(d, "capacity");
  a.deltas = val<int32_t>(d, "deltas");
  a.nch = val<int32_t>(d, "nch");
  a.dmax = val<int32_t>(d, "dmax");
  a.max_participants = val<int32_t>(d, "max_participants");
  a.min_sigma_eff = val<double>(d, "min_sigma_eff");
  a.now_us = val<int64_t>(d, "now_us");
  a.seed = val<uint64_t>(d, "seed");
  a.id_base = val<uint64_t>(d, "id_base");
  a.creator_id = val<int32_t>(d, "creator_id");
  a.audit = val<int32_t>(d, "audit");
  if (a.deltas < 0 || a.deltas > kMaxDeltasPipeline) throw py::value_error("deltas out of range");
  if (a.nch < 1 || a.nch > kMaxChanges) throw py::value_error("nch out of range");
  if (a.dmax < a.deltas) throw py::value_error("dmax < deltas");
  if (a.max_participants > kMaxParticipants) throw py::value_error("max_participants > 16");
  if (a.capacity <= 0 || a.n > a.capacity) throw py::value_error("batch larger than table capacity");
  a.session_agent = ptr<const int32_t>(d, "session_agent");
  a.agent_sigma = ptr<const double>(d, "agent_sigma");
  a.agent_did = ptr<const int32_t>(d, "agent_did");
  a.changes = ptr<const ChangeIds>(d, "changes");
  a.vouch_offsets = ptr<const int32_t>(d, "vouch_offsets");
  a.vouch_active = ptr<uint8_t>(d, "vouch_active");
  a.vouch_released_us = ptr<int64_t>(d, "vouch_released_us");
  a.pool.bytes = ptr<const uint8_t>(d, "pool_bytes");
  a.pool.off = ptr<const int64_t>(d, "pool_off");
  a.pool.len = ptr<const int32_t>(d, "pool_len");
  a.stats = ptr<unsigned long long>(d, "stats");
  SessionTables& t = a.t;
  t.sess_uuid = ptr<uint32_t>(d, "sess_uuid");
  t.sess_state = ptr<uint8_t>(d, "sess_state");
  t.sess_mode = ptr<uint8_t>(d, "sess_mode");
  t.sess_creator = ptr<int32_t>(d, "sess_creator");
  t.sess_created_us = ptr<int64_t>(d, "sess_created_us");
  t.sess_terminated_us = ptr<int64_t>(d, "sess_terminated_us");
  t.part_count = ptr<int32_t>(d, "part_count");
  t.part_agent = ptr<int32_t>(d, "part_agent");
  t.part_ring = ptr<uint8_t>(d, "part_ring");
  t.part_sigma_raw = ptr<double>(d, "part_sigma_raw");
  t.part_sigma_eff = ptr<double>(d, "part_sigma_eff");
  t.part_joined_us = ptr<int64_t>(d, "part_joined_us");
  t.delta_hash = ptr<uint32_t>(d, "delta_hash");
  t.delta_count = ptr<int32_t>(d, "delta_count");
  t.merkle_root = ptr<uint32_t>(d, "merkle_root");
  t.saga_uuid = ptr<uint32_t>(d, "saga_uuid");
  t.step_uuid = ptr<uint32_t>(d, "step_uuid");
  t.saga_state = ptr<uint8_t>(d, "saga_state");
  t.step_state = ptr<uint8_t>(d, "step_state");
  t.step_started_us = ptr<int64_t>(d, "step_started_us");
  t.step_completed_us = ptr<int64_t>(d, "step_completed_us");
  t.committed_at_us = ptr<int64_t>(d, "committed_at_us");
  t.gc_retained = ptr<int32_t>(d, "gc_retained");
  t.bonds_released = ptr<int32_t>(d, "bonds_released");
  t.status = ptr<int32_t>(d, "status");
  return a;
}

void register_kernels(py::module_& m) {
  m.def(
      "pipeline",
      [](const py::dict& d, uintptr_t stream) {
        PipelineArgs a = pipeline_args(d);
        py::gil_scoped_release nogil;
        launch_pipeline(a, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("args"), py::arg("stream"),
      "Launch the batched governance pipeline kernel on `stream`.");
  m.def(
      "pipeline_host",
      [](const py::dict& d) {
        PipelineArgs a = pipeline_args(d);
        py::gil_scoped_release nogil;
        pipeline_host(a);
      },
      py::arg("args"), "Run the same per-session pipeline body on the CPU (host twin).");
  m.attr("PIPE_MAX_PARTICIPANTS") = kMaxParticipants;
  m.attr("PIPE_MAX_DELTAS") = kMaxDeltasPipeline;
  m.attr("PIPE_MAX_CHANGES") = kMaxChanges;
}

}  // namespace host
}  // namespace ahv
