// Python bindings of the gfx950 kernel launchers and their host twins.
//
// Tensors are owned by PyTorch (device-resident SoA tables, see
// agent_hypervisor_amd/models/tables.py); Python passes raw data pointers, the
// current HIP stream, and scalar arguments in a dict.  Shape/dtype validation is
// done by the Python wrappers in agent_hypervisor_amd/ops/, which fail loudly.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ahv/kernels.h"
#include "ahv/launch.h"
#include "ahv/pipeline.h"
#include "ahv/saga_batch.h"

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


// ---------------------------------------------------------------------------
// Generic binding: every kernel gets `<name>(args: dict, stream: int)` (device)
// and `<name>_host(args: dict)` (CPU twin).  Field readers below map dict keys
// to struct members by name.

#define P(field, T) a.field = ptr<T>(d, #field)
#define V(field, T) a.field = val<T>(d, #field)

static RingGateArgs to_ring_gate(const py::dict& d) {
  RingGateArgs a{};
  V(n, int64_t); P(sigma, const double); P(consensus, const uint8_t); P(ring, uint8_t);
  return a;
}
static RingCheckArgs to_ring_check(const py::dict& d) {
  RingCheckArgs a{};
  V(n, int64_t); P(agent_ring, const uint8_t); P(action_flags, const uint8_t); P(sigma, const double);
  P(consensus, const uint8_t); P(witness, const uint8_t); P(required, uint8_t); P(reason, uint8_t);
  return a;
}
static FsmArgs to_fsm(const py::dict& d) {
  FsmArgs a{};
  V(n, int64_t); V(kind, int32_t); V(now_us, int64_t); P(state, uint8_t); P(target, const uint8_t);
  P(ok, uint8_t); P(started_us, int64_t); P(completed_us, int64_t);
  return a;
}
static FanoutArgs to_fanout(const py::dict& d) {
  FanoutArgs a{};
  V(groups, int64_t); P(offsets, const int32_t); P(policy, const uint8_t); P(succeeded, const uint8_t);
  P(satisfied, uint8_t); P(success_count, int32_t); P(compensate, uint8_t);
  return a;
}
static BreachArgs to_breach(const py::dict& d) {
  BreachArgs a{};
  V(n, int64_t); V(window_cap, int32_t); V(window_us, int64_t); V(cooldown_us, int64_t);
  P(rows, const int32_t); P(offsets, const int32_t);
  P(now_us, const int64_t); P(agent_ring, const uint8_t); P(new_called, const uint8_t); P(ts, int64_t);
  P(called, uint8_t); P(head, int32_t); P(count, int32_t); P(total, int64_t); P(tripped, uint8_t);
  P(tripped_at_us, int64_t); P(ring_counts, int64_t); P(severity, uint8_t); P(rate, double); P(hits, int32_t);
  P(event, uint8_t); P(window, int32_t);
  return a;
}
static BucketArgs to_bucket(const py::dict& d) {
  BucketArgs a{};
  V(n, int64_t); V(now_us, int64_t); P(rows, const int32_t); P(offsets, const int32_t); P(tokens, double);
  P(last_us, int64_t); P(capacity, const double); P(rate, const double); P(cost, const double);
  P(total, int64_t); P(rejected, int64_t); P(ok, uint8_t);
  return a;
}
static ExpiryArgs to_expiry(const py::dict& d) {
  ExpiryArgs a{};
  V(n, int64_t); V(now_us, int64_t); P(active, uint8_t); P(expires_us, const int64_t);
  P(released_us, int64_t); P(expired, uint8_t);
  return a;
}
static BondFusedArgs to_bond_fused(const py::dict& d) {
  BondFusedArgs a{};
  V(sessions, int64_t); V(now_us, int64_t); P(offsets, const int32_t); P(voucher, const uint8_t);
  P(vouchee, const uint8_t); P(bonded, const double); P(active, const uint8_t); P(expiry_us, const int64_t);
  P(sigma, const double); P(omega, const double); P(sigma_eff, double); P(exposure, double); P(bonded_in, double);
  P(members, const int64_t); P(agent_exposure, double);
  return a;
}
static LedgerArgs to_ledger(const py::dict& d) {
  LedgerArgs a{};
  V(agents, int64_t); P(offsets, const int32_t); P(type, const uint8_t); P(severity, const double);
  P(raw_risk, double); P(risk, double); P(recommendation, uint8_t); P(slash_count, int32_t);
  P(quarantine_count, int32_t); P(clean_count, int32_t); P(fault_avg, double);
  return a;
}
static DriftArgs to_drift(const py::dict& d) {
  DriftArgs a{};
  V(n, int64_t); V(low, double); V(medium, double); V(high, double); V(critical, double);
  P(drift, const double); P(severity, uint8_t);
  return a;
}
static AttributionArgs to_attribution(const py::dict& d) {
  AttributionArgs a{};
  V(cases, int64_t); P(node_offsets, const int32_t); P(agent_offsets, const int32_t);
  P(agent_of_node, const int32_t); P(success, const uint8_t); P(root_cause, const uint8_t);
  P(risk_weight, const double); P(raw, double); P(node_count, int32_t);
  return a;
}
static BondTileArgs to_bond_tiles(const py::dict& d) {
  BondTileArgs a{};
  V(sessions, int64_t); P(tiles, const double); P(sigma, const double); P(omega, const double);
  P(sigma_eff, double); P(exposure, double); P(bonded_in, double);
  if (d.contains("members")) {
    P(members, const int64_t); P(agent_exposure, double);
  }
  return a;
}
static VouchCsrArgs to_vouch_csr(const py::dict& d) {
  VouchCsrArgs a{};
  V(sessions, int64_t); V(now_us, int64_t); P(offsets, const int32_t); P(voucher, const uint8_t);
  P(vouchee, const uint8_t); P(bonded, const double); P(active, uint8_t); P(expiry_us, const int64_t);
  P(released_us, int64_t); P(tiles, double); P(sigma, const double); P(omega, const double);
  P(sigma_eff, double); P(released, int32_t);
  return a;
}
static VouchAdmitArgs to_vouch_admit(const py::dict& d) {
  VouchAdmitArgs a{};
  V(sessions, int64_t); V(now_us, int64_t); V(max_exposure, double); P(e_offsets, const int32_t);
  P(e_voucher, const uint8_t); P(e_vouchee, const uint8_t); P(e_bonded, const double);
  P(e_active, const uint8_t); P(e_expiry, const int64_t); P(r_offsets, const int32_t);
  P(r_voucher, const uint8_t); P(r_vouchee, const uint8_t); P(r_sigma, const double); P(r_pct, const double);
  P(r_bonded, double); P(code, uint8_t);
  return a;
}
static SlashArgs to_slash(const py::dict& d) {
  SlashArgs a{};
  V(sessions, int64_t); V(now_us, int64_t); P(offsets, const int32_t); P(voucher, const uint8_t);
  P(vouchee, const uint8_t); P(active, uint8_t); P(expiry_us, const int64_t); P(released_us, int64_t);
  P(target, const uint8_t); P(omega, const double); P(scores, double); P(clip_offsets, int32_t);
  P(clip_count, int32_t); P(clip_voucher, uint8_t); P(clip_depth, uint8_t); P(clip_before, double);
  P(clip_after, double); V(clip_cap, int32_t); P(clip_walk, uint8_t);
  a.bonded = d.contains("bonded") ? ptr<const double>(d, "bonded") : nullptr;
  a.sigma_eff = d.contains("sigma_eff") ? ptr<double>(d, "sigma_eff") : nullptr;
  a.mode = d.contains("mode") ? val<int32_t>(d, "mode") : -1;
  if (d.contains("touched") && !d["touched"].is_none()) {
    P(touched_tmp, int32_t); P(touched_blocks, int32_t); P(touched_offsets, int32_t); P(touched, int64_t);
    P(touched_total, int64_t);
  }
  if (a.mode < -1 || a.mode > 3) throw py::value_error("slash: mode must be -1, 0, 1, 2 or 3");
  return a;
}
static RenderArgs to_render(const py::dict& d) {
  RenderArgs a{};
  V(rows, int64_t); V(len, int32_t); V(pitch, int64_t); P(tmpl, const uint8_t); P(out, uint8_t);
  P(ids, const int64_t);
  if (a.pitch < a.len) throw py::value_error("render_rows: pitch < len");
  const auto stamps = d["stamps"].cast<std::vector<std::tuple<int32_t, int32_t, int64_t, int64_t>>>();
  if (stamps.size() > static_cast<size_t>(kRenderMaxStamps)) throw py::value_error("render_rows: too many stamp fields");
  a.nstamp = static_cast<int32_t>(stamps.size());
  for (size_t k = 0; k < stamps.size(); ++k) {
    const auto& [pos, width, mod, add] = stamps[k];
    if (pos < 0 || width <= 0 || width > 18 || pos + width > a.len) throw py::value_error("render_rows: bad stamp field");
    a.stamp_pos[k] = pos;
    a.stamp_width[k] = width;
    a.stamp_mod[k] = mod;
    a.stamp_add[k] = add;
  }
  V(hex_pos, int32_t); V(hex_bytes, int32_t); P(hex_src, const uint8_t); V(hex_stride, int64_t);
  if (a.hex_pos >= 0 && (a.hex_src == nullptr || a.hex_pos + 2 * a.hex_bytes > a.len))
    throw py::value_error("render_rows: bad hex field");
  return a;
}
static HashManyArgs to_hash_many(const py::dict& d) {
  HashManyArgs a{};
  V(n, int64_t); P(bytes, const uint8_t); P(offsets, const int64_t); P(digest, uint32_t);
  return a;
}
static MerkleArgs to_merkle(const py::dict& d) {
  MerkleArgs a{};
  V(chains, int64_t); P(offsets, const int32_t); P(leaves, const uint32_t); P(scratch, uint32_t);
  P(root, uint32_t);
  if (d.contains("leaf_idx")) P(leaf_idx, const int64_t);
  if (d.contains("root_row")) P(root_row, const int64_t);
  if (d.contains("gate")) P(gate, const int64_t);
  return a;
}
static VerifyArgs to_verify(const py::dict& d) {
  VerifyArgs a{};
  V(deltas, int64_t); V(chains, int64_t); P(bytes, const uint8_t); P(offsets, const int64_t);
  P(stored, const uint32_t); P(parent, const uint32_t); P(has_parent, const uint8_t);
  P(chain_offsets, const int32_t); P(delta_ok, uint8_t); P(chain_ok, uint8_t);
  return a;
}
static VClockArgs to_vclock(const py::dict& d) {
  VClockArgs a{};
  V(groups, int64_t); V(A, int32_t); V(strict, int32_t); P(offsets, const int32_t); P(op, const uint8_t);
  P(path, const int32_t); P(agent, const int32_t); P(agent_col, const int32_t); P(path_clock, uint32_t);
  P(agent_clock, uint32_t); P(ok, uint8_t);
  return a;
}
static LockArgs to_locks(const py::dict& d) {
  LockArgs a{};
  V(n, int64_t); P(res_offsets, const int32_t); P(lock_agent, const int32_t); P(lock_intent, const uint8_t);
  P(req_res, const int32_t); P(req_agent, const int32_t); P(req_intent, const uint8_t); P(conflicts, int32_t);
  return a;
}
static LockGrantArgs to_lock_grant(const py::dict& d) {
  LockGrantArgs a{};
  V(segments, int64_t); P(seg_offsets, const int32_t); P(order, const int32_t); P(req_res, const int32_t);
  P(req_agent, const int32_t); P(req_intent, const uint8_t); P(table, int32_t); P(granted, uint8_t);
  return a;
}
static ChainHashArgs to_chain_hash(const py::dict& d) {
  ChainHashArgs a{};
  V(chains, int64_t); P(chain_offsets, const int32_t); P(bytes, const uint8_t); P(pre_off, const int64_t);
  P(pre_len, const int32_t); P(suf_off, const int64_t); P(suf_len, const int32_t);
  P(seed_parent, const uint32_t); P(has_seed, const uint8_t); P(digest, uint32_t);
  a.mid = d.contains("mid") ? ptr<uint32_t>(d, "mid") : nullptr;
  a.deltas = d.contains("deltas") ? d["deltas"].cast<int64_t>() : 0;
  a.uniform_len = d.contains("uniform_len") ? d["uniform_len"].cast<int32_t>() : 0;
  a.sel = d.contains("sel") ? ptr<const int64_t>(d, "sel") : nullptr;
  if (a.sel && a.uniform_len <= 0) throw py::value_error("chain_hash: sel needs uniform_len");
  return a;
}
static SagaBatchArgs to_saga(const py::dict& d) {
  SagaBatchArgs a{};
  V(sagas, int64_t); V(steps, int32_t); V(compensate, int32_t); V(now_us, int64_t);
  P(fail_attempts, const uint8_t); P(fail_kind, const uint8_t); P(comp_fail, const uint8_t);
  P(has_undo, const uint8_t); P(max_retries, const uint8_t); P(step_state, uint8_t); P(retry_count, uint8_t);
  P(step_error, uint8_t); P(started_us, int64_t); P(completed_us, int64_t); P(saga_state, uint8_t);
  P(saga_completed_us, int64_t); P(failed_step, int32_t); P(comp_failed, int32_t); P(tick, int32_t);
  P(stats, unsigned long long);
  a.now_dev = d.contains("now_dev") ? ptr<const int64_t>(d, "now_dev") : nullptr;
  return a;
}
#undef P
#undef V

template <class A>
static void bind_pair(py::module_& m, const char* name, A (*conv)(const py::dict&),
                      void (*dev)(const A&, hipStream_t), void (*host)(const A&)) {
  m.def(
      name,
      [conv, dev](const py::dict& d, uintptr_t stream) {
        A a = conv(d);
        py::gil_scoped_release nogil;
        dev(a, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("args"), py::arg("stream"));
  m.def(
      (std::string(name) + "_host").c_str(),
      [conv, host](const py::dict& d) {
        A a = conv(d);
        py::gil_scoped_release nogil;
        host(a);
      },
      py::arg("args"));
}

void register_kernels(py::module_& m) {
  bind_pair(m, "ring_gate", to_ring_gate, launch_ring_gate, ring_gate_host);
  bind_pair(m, "ring_check", to_ring_check, launch_ring_check, ring_check_host);
  bind_pair(m, "fsm", to_fsm, launch_fsm, fsm_host);
  bind_pair(m, "fanout", to_fanout, launch_fanout, fanout_host);
  bind_pair(m, "breach", to_breach, launch_breach, breach_host);
  bind_pair(m, "bucket", to_bucket, launch_bucket, bucket_host);
  bind_pair(m, "expiry", to_expiry, launch_expiry, expiry_host);
  bind_pair(m, "ledger", to_ledger, launch_ledger, ledger_host);
  bind_pair(m, "drift", to_drift, launch_drift, drift_host);
  bind_pair(m, "attribution", to_attribution, launch_attribution, attribution_host);
  bind_pair(m, "bond_tiles", to_bond_tiles, launch_bond_tiles, bond_tiles_host);
  bind_pair(m, "bond_fused", to_bond_fused, launch_bond_fused, bond_fused_host);
  bind_pair(m, "build_tiles", to_vouch_csr, launch_build_tiles, build_tiles_host);
  bind_pair(m, "sigma_eff_csr", to_vouch_csr, launch_sigma_eff_csr, sigma_eff_csr_host);
  bind_pair(m, "sigma_eff_stream", to_vouch_csr, launch_sigma_eff_stream, sigma_eff_csr_host);
  bind_pair(m, "release_bonds", to_vouch_csr, launch_release, release_host);
  bind_pair(m, "vouch_admit", to_vouch_admit, launch_vouch_admit, vouch_admit_host);
  bind_pair(m, "slash", to_slash, launch_slash, slash_host);
  bind_pair(m, "hash_many", to_hash_many, launch_hash_many, hash_many_host);
  bind_pair(m, "render_rows", to_render, launch_render_rows, render_rows_host);
  bind_pair(m, "merkle", to_merkle, launch_merkle, merkle_host);
  bind_pair(m, "verify", to_verify, launch_verify, verify_host);
  bind_pair(m, "vclock", to_vclock, launch_vclock, vclock_host);
  bind_pair(m, "locks", to_locks, launch_locks, locks_host);
  bind_pair(m, "lock_grant", to_lock_grant, launch_lock_grant, lock_grant_host);
  bind_pair(m, "saga_fused", to_saga, launch_saga_fused, saga_fused_host);
  bind_pair(m, "chain_hash", to_chain_hash, launch_chain_hash, chain_hash_host);
  m.def(
      "saga_phase",
      [](const py::dict& d, int phase, int k, uintptr_t stream) {
        SagaBatchArgs a = to_saga(d);
        py::gil_scoped_release nogil;
        launch_saga_phase(a, phase, k, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("args"), py::arg("phase"), py::arg("k"), py::arg("stream"));
  m.def(
      "saga_phase_host",
      [](const py::dict& d, int phase, int k) {
        SagaBatchArgs a = to_saga(d);
        py::gil_scoped_release nogil;
        saga_phase_host(a, phase, k);
      },
      py::arg("args"), py::arg("phase"), py::arg("k"));
  m.def(
      "spread_fold",
      [](uintptr_t spread, uintptr_t out, int k, bool accumulate, uintptr_t stream) {
        launch_spread_fold(reinterpret_cast<unsigned long long*>(spread), reinterpret_cast<unsigned long long*>(out), k,
                           accumulate, reinterpret_cast<hipStream_t>(stream));
      },
      py::arg("spread"), py::arg("out"), py::arg("k"), py::arg("accumulate"), py::arg("stream"),
      "Fold [64, k] spread counters into out[k] (add or copy) and zero them, on `stream`.");
  m.def(
      "pipeline_clock",
      [](uintptr_t cursor, int64_t base_us, int64_t base_clk, int64_t rate_khz, uintptr_t stream) {
        launch_pipeline_clock(reinterpret_cast<int64_t*>(cursor), base_us, base_clk, rate_khz,
                              reinterpret_cast<hipStream_t>(stream));
      },
      "Stamp cursor[2] (now_us) from the device wall clock on `stream`.");
  m.def(
      "pipeline_advance",
      [](uintptr_t cursor, int64_t n, int64_t capacity, uintptr_t stream) {
        launch_pipeline_advance(reinterpret_cast<int64_t*>(cursor), n, capacity,
                                reinterpret_cast<hipStream_t>(stream));
      },
      "Advance cursor slot/id bases by one batch of `n` sessions on `stream`.");
  m.def(
      "pipeline_epilogue",
      [](uintptr_t spread, uintptr_t out, int k, uintptr_t cursor, int64_t n, int64_t capacity, int64_t base_us,
         int64_t base_clk, int64_t rate_khz, uintptr_t stream) {
        launch_pipeline_epilogue(reinterpret_cast<unsigned long long*>(spread), reinterpret_cast<unsigned long long*>(out),
                                 k, reinterpret_cast<int64_t*>(cursor), n, capacity, base_us, base_clk, rate_khz,
                                 reinterpret_cast<hipStream_t>(stream));
      },
      "Captured step epilogue: fold spread counters into out (copy), advance the cursor, stamp the next time base.");
  m.def(
      "kernel_attributes",
      []() {
        std::vector<KernelEntry> ks;
        kernels_audit(ks);
        kernels_store_template(ks);
        kernels_liability(ks);
        kernels_saga(ks);
        kernels_merkle_tree(ks);
        py::list out;
        for (const auto& k : ks) {
          hipFuncAttributes fa{};
          check_hip(hipFuncGetAttributes(&fa, k.fn), k.name);
          py::dict d;
          d["name"] = k.name;
          d["vgprs"] = fa.numRegs;
          d["scratch_bytes"] = static_cast<int64_t>(fa.localSizeBytes);
          d["lds_bytes"] = static_cast<int64_t>(fa.sharedSizeBytes);
          d["max_threads"] = fa.maxThreadsPerBlock;
          out.append(d);
        }
        return out;
      },
      "Resources of the hot kernels (hipFuncGetAttributes): VGPRs, scratch, static LDS.");
  m.def("device_wall_clock", &device_wall_clock, py::arg("device"));
  m.def("device_wall_clock_rate_khz", &device_wall_clock_rate_khz, py::arg("device"));
  m.attr("PIPE_MAX_PARTICIPANTS") = kMaxParticipants;
  m.attr("PIPE_MAX_DELTAS") = kMaxDeltasPipeline;
  m.attr("PIPE_MAX_CHANGES") = kMaxChanges;
}

}  // namespace host
}  // namespace ahv
