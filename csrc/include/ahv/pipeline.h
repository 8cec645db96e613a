// Batched full governance pipeline — the device form of the reference
// benchmark's `full_governance_pipeline` (benchmarks/bench_hypervisor.py:217-239):
//
//   create_session → join(agent, σ) [ring gate K01, join admission]
//   → activate → D × DeltaEngine.capture [canonical JSON + SHA-256 chain, K08]
//   → saga create + add_step + execute_step [step FSM K13]
//   → terminate [Merkle root K09, commitment, bond release K07, GC, archive]
//
// for every session of a batch; each lane owns one session.  The per-session body
// is `pipeline_session<Sink>` below, instantiated on the device with the LDS
// WordWindowSink (ahv/wave_sink.h) and on the host with HostSink (the CPU twin
// used by tests).
#pragma once

#include "ahv/delta_emit.h"
#include "ahv/events.h"
#include "ahv/semantics.h"

namespace ahv {

constexpr int kMaxParticipants = 16;  // participant row width (max_participants ≤ 16)
constexpr int kMaxDeltasPipeline = 8;  // ⌈8/2⌉ Merkle scratch slots fit the LDS window
constexpr int kMaxChanges = 4;

// SoA device tables (one row per session slot).  All pointers are device
// pointers for the kernel, host pointers for the twin.
struct SessionTables {
  uint32_t* sess_uuid;       // [cap, 4]
  uint8_t* sess_state;       // [cap]
  uint8_t* sess_mode;        // [cap]    0 eventual, 1 strong
  int32_t* sess_creator;     // [cap]    agent id
  int64_t* sess_created_us;  // [cap]
  int64_t* sess_terminated_us;  // [cap]
  int32_t* part_count;       // [cap]
  int32_t* part_agent;       // [cap, P]
  uint8_t* part_ring;        // [cap, P]
  double* part_sigma_raw;    // [cap, P]
  double* part_sigma_eff;    // [cap, P]
  int64_t* part_joined_us;   // [cap, P]
  uint32_t* delta_hash;      // [cap, Dmax, 8]
  int32_t* delta_count;      // [cap]
  uint32_t* merkle_root;     // [cap, 8]
  uint32_t* saga_uuid;       // [cap, 4]
  uint32_t* step_uuid;       // [cap, 4]
  uint8_t* saga_state;       // [cap]
  uint8_t* step_state;       // [cap]
  int64_t* step_started_us;  // [cap]
  int64_t* step_completed_us;  // [cap]
  int64_t* committed_at_us;  // [cap]   0 = no commitment
  int32_t* gc_retained;      // [cap]
  int32_t* bonds_released;   // [cap]
  int32_t* status;           // [cap]   0 ok, else first failing rule (see PipeStatus)
};

enum PipeStatus : int32_t {
  PIPE_OK = 0,
  PIPE_BAD_HANDSHAKE = 1,
  PIPE_JOIN_REJECTED = 2,  // | join code << 8
  PIPE_BAD_ACTIVATE = 3,
  PIPE_BAD_STEP = 4,
  PIPE_BAD_TERMINATE = 5,
};

struct PipelineArgs {
  int64_t n;               // sessions in this batch
  int64_t slot_base;       // first table row
  int64_t capacity;        // table rows (slot index wraps modulo capacity)
  int32_t deltas;          // D, ≤ kMaxDeltasPipeline
  int32_t nch;             // changes per delta, ≤ kMaxChanges
  int32_t dmax;            // delta_hash row width
  int32_t max_participants;
  double min_sigma_eff;
  int64_t now_us;          // injected batch time base (N09)
  uint64_t seed;           // id generator seed
  uint64_t id_base;        // id counter base (monotone across batches)
  int32_t creator_id;      // pool id / agent id of the creator DID
  int32_t audit;           // SessionConfig.enable_audit
  const int32_t* session_agent;  // [n] agent id joining each session
  const double* agent_sigma;     // [A] σ_raw per agent id
  const int32_t* agent_did;      // [A] pool id of each agent's DID
  const ChangeIds* changes;      // [D * nch] (shared by all sessions)
  // Resident vouch slab (VouchSlab in models/tables.py), or vouch_count == null:
  // slot s owns edges [s·stride, s·stride + vouch_count[s]); terminate releases
  // the active ones (K07) and empties the slot for its next session.
  int32_t* vouch_count;          // [cap]
  int32_t vouch_stride;          // edges per slot
  uint8_t* vouch_active;         // [cap·stride] cleared on release
  int64_t* vouch_released_us;    // [cap·stride]
  int64_t gc_retention_us;       // RetentionPolicy.delta_retention_days in µs
  StrPool pool;
  SessionTables t;
  unsigned long long* stats;     // [kPipeStats] batch counters (X04), accumulated, or null
  // Device-resident cursor {slot_base, id_base, now_us} (int64[3]) or null.  When
  // set it overrides the three scalars above, so a launch captured in a hipGraph
  // stays correct on replay: the clock kernel refreshes now_us and the advance
  // kernel moves slot/id bases on the device (runtime/graphs.py, N07/N09).
  const int64_t* cursor;
  // Device event ring (N08); ev.cursor == null disables event emission.
  EventRing ev;
};

AHV_HD int64_t pipe_slot_base(const PipelineArgs& a) { return a.cursor ? a.cursor[0] : a.slot_base; }
AHV_HD uint64_t pipe_id_base(const PipelineArgs& a) {
  return a.cursor ? static_cast<uint64_t>(a.cursor[1]) : a.id_base;
}
AHV_HD int64_t pipe_now_us(const PipelineArgs& a) { return a.cursor ? a.cursor[2] : a.now_us; }

// Per-session counters reduced into PipelineArgs::stats:
// sessions, ok, participants, deltas, commitments, archived.
constexpr int kPipeStats = 6;
struct PipeCounters {
  uint32_t v[kPipeStats];
};

// Per-session body.  `i` is the batch index.
template <class Sink>
AHV_HD PipeCounters pipeline_session(const PipelineArgs& a, int64_t i, Sink& sink) {
  const int64_t slot = (pipe_slot_base(a) + i) % a.capacity;
  const SessionTables& t = a.t;
  const int64_t now = pipe_now_us(a);
  const uint64_t id_base = pipe_id_base(a);
  int32_t status = PIPE_OK;

  // ---- create_session + begin_handshake -------------------------------------
  uint32_t u[4];
  uuid4_words(a.seed, id_base + 3 * static_cast<uint64_t>(i), u);
#pragma unroll
  for (int k = 0; k < 4; ++k) t.sess_uuid[slot * 4 + k] = u[k];
  uint8_t state = SS_CREATED;
  t.sess_creator[slot] = a.creator_id;
  t.sess_created_us[slot] = now;
  t.sess_terminated_us[slot] = 0;
  t.sess_mode[slot] = 0;
  if ((session_op_allowed_from(OP_HANDSHAKE) >> state) & 1u) state = SS_HANDSHAKING;
  else status = PIPE_BAD_HANDSHAKE;

  // ---- join_session: σ resolution → ring gate (K01) → admission ----------------
  const int32_t agent = a.session_agent[i];
  const double sigma_raw = a.agent_sigma[agent];
  const double sigma_eff = sigma_raw;  // no Nexus adapter in the batched path
  const uint8_t ring = ring_from_sigma(sigma_eff, false);
  int32_t parts = 0;
  const uint8_t jc = join_check(state, false, parts, a.max_participants, sigma_eff, a.min_sigma_eff, ring);
  const int64_t prow = slot * kMaxParticipants;
  if (jc == JOIN_OK) {
    t.part_agent[prow] = agent;
    t.part_ring[prow] = ring;
    t.part_sigma_raw[prow] = sigma_raw;
    t.part_sigma_eff[prow] = sigma_eff;
    t.part_joined_us[prow] = now;
    parts = 1;
  } else if (status == PIPE_OK) {
    status = PIPE_JOIN_REJECTED | (static_cast<int32_t>(jc) << 8);
  }
  t.part_count[slot] = parts;

  // ---- activate ----------------------------------------------------------------
  if (((session_op_allowed_from(OP_ACTIVATE) >> state) & 1u) && parts > 0) state = SS_ACTIVE;
  else if (status == PIPE_OK) status = PIPE_BAD_ACTIVATE;

  // The saga and terminate-transition stages read nothing the capture stage
  // produces (their timestamps are now + D + k), so they run before it: fewer
  // values stay live across the SHA rounds (no register spill at 168 VGPRs).
  // ---- saga: create, add_step, execute_step (executor is a device no-op) ----------
  uint32_t su[4], stu[4];
  uuid4_words(a.seed, id_base + 3 * static_cast<uint64_t>(i) + 1, su);
  uuid4_words(a.seed, id_base + 3 * static_cast<uint64_t>(i) + 2, stu);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    t.saga_uuid[slot * 4 + k] = su[k];
    t.step_uuid[slot * 4 + k] = stu[k];
  }
  uint8_t saga_st = SG_RUNNING;
  uint8_t step_st = ST_PENDING;
  if ((step_transitions(step_st) >> ST_EXECUTING) & 1u) {
    step_st = ST_EXECUTING;
    t.step_started_us[slot] = now + a.deltas + 1;
  }
  if ((step_transitions(step_st) >> ST_COMMITTED) & 1u) {
    step_st = ST_COMMITTED;
    t.step_completed_us[slot] = now + a.deltas + 2;
  } else if (status == PIPE_OK) {
    status = PIPE_BAD_STEP;
  }
  t.saga_state[slot] = saga_st;
  t.step_state[slot] = step_st;

  // ---- terminate: everything except the Merkle root ---------------------------------
  // (commit timestamp, bond release K07, GC, archive and the counters read nothing the
  // capture stage produces, so they are settled here: across the SHA rounds only the
  // slot, the delta-hash row and one packed word stay live — no register spill)
  if ((session_op_allowed_from(OP_TERMINATE) >> state) & 1u) {
    state = SS_TERMINATING;
    t.sess_terminated_us[slot] = now + a.deltas + 3;
  } else if (status == PIPE_OK) {
    status = PIPE_BAD_TERMINATE;
  }
  const bool committed = a.audit && a.deltas > 0;
  const int64_t t_term = now + a.deltas + 3;
  t.committed_at_us[slot] = committed ? t_term : 0;
  int32_t released = 0;
  if (a.vouch_count) {
    const int64_t e0 = slot * a.vouch_stride;
    const int32_t ne = a.vouch_count[slot];
    for (int32_t k = 0; k < ne; ++k) {
      if (a.vouch_active[e0 + k]) {
        a.vouch_active[e0 + k] = 0;
        a.vouch_released_us[e0 + k] = t_term;
        ++released;
      }
    }
    a.vouch_count[slot] = 0;
  }
  t.bonds_released[slot] = released;
  // GC (reference audit/gc.py): deltas stamped before terminate − retention expire
  const int64_t cutoff = t_term - a.gc_retention_us;
  int32_t retained = 0;
  for (int d = 0; d < a.deltas; ++d) retained += (now + d + 1 >= cutoff) ? 1 : 0;
  t.gc_retained[slot] = retained;
  if ((session_op_allowed_from(OP_ARCHIVE) >> state) & 1u) state = SS_ARCHIVED;
  t.sess_state[slot] = state;
  t.status[slot] = status;
  t.delta_count[slot] = a.deltas;
  PipeCounters c;
  c.v[0] = 1;
  c.v[1] = status == PIPE_OK ? 1u : 0u;
  c.v[2] = static_cast<uint32_t>(parts);
  c.v[3] = static_cast<uint32_t>(a.deltas);
  c.v[4] = committed ? 1u : 0u;
  c.v[5] = state == SS_ARCHIVED ? 1u : 0u;

  // ---- D × capture: canonical JSON + SHA-256 Merkle chain (K08) -------------------
  SessionIdent sid;
  sid.str_id = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) sid.uuid[k] = u[k];
  const StrRef did = pool_ref(a.pool, a.agent_did[agent]);  // resolved once per session
  Digest prev, mid;
  uint32_t* hrow = t.delta_hash + slot * a.dmax * 8;
  const bool share_block0 = did.n >= kMidstateMinDid;  // every delta's block 0 is the same bytes
  for (int d = 0; d < a.deltas; ++d) {
    uint32_t h[8];
    const int mode = !share_block0 ? MID_OFF : (d == 0 ? MID_CAPTURE : MID_RESUME);
    emit_delta_and_hash(sink, a.pool, did, a.changes + d * a.nch, static_cast<uint32_t>(a.nch), -1,
                        static_cast<uint32_t>(d + 1), d > 0, prev, sid, now + d + 1, h, mid, mode);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      prev.v[k] = h[k];
      hrow[d * 8 + k] = h[k];
    }
  }

  // ---- terminate: Merkle root (K09) → commitment -------------------------------------
  // Leaves re-read from this session's delta_hash row (written by this same lane
  // above); interior levels in the sink's digest scratch (LDS on the device).
  uint32_t root[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (a.deltas > 0) {
    merkle_root_levels(
        sink, static_cast<uint32_t>(a.deltas),
        [&](uint32_t d, uint32_t h[8]) {
#pragma unroll
          for (int k = 0; k < 8; ++k) h[k] = hrow[d * 8 + k];
        },
        root);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) t.merkle_root[slot * 8 + k] = committed ? root[k] : 0u;
  return c;
}

// ---- lifecycle events (N08) --------------------------------------------------------
// The records the scalar Hypervisor facade publishes for the same pipeline when it
// has an event bus: created → joined → ring_assigned → activated → terminated →
// audit.committed → gc_collected → archived (fewer when a stage was refused).

AHV_HD uint32_t pipeline_event_count(const PipelineArgs& a, int64_t i, const PipeCounters& c) {
  const int64_t slot = (pipe_slot_base(a) + i) % a.capacity;
  return 1u + (c.v[2] ? 3u : 0u) + (a.t.sess_terminated_us[slot] ? 1u : 0u) + c.v[4] + 2u * c.v[5];
}

template <class Put>
AHV_HD void pipeline_events(const PipelineArgs& a, int64_t i, const PipeCounters& c, Put&& put) {
  const int64_t slot = (pipe_slot_base(a) + i) % a.capacity;
  const SessionTables& t = a.t;
  const int32_t agent = a.session_agent[i];
  const int64_t t0 = t.sess_created_us[slot];
  const int64_t te = t.sess_terminated_us[slot];
  uint32_t k = 0;
  put(k++, slot, EventRec{EV_SESSION_CREATED, -1, t0, 0});
  if (c.v[2]) {
    put(k++, slot, EventRec{EV_SESSION_JOINED, agent, t0, 0});
    put(k++, slot, EventRec{EV_RING_ASSIGNED, agent, t0, t.part_ring[slot * kMaxParticipants]});
    put(k++, slot, EventRec{EV_SESSION_ACTIVATED, -1, t0, 0});
  }
  if (te) put(k++, slot, EventRec{EV_SESSION_TERMINATED, -1, te, 0});
  if (c.v[4]) put(k++, slot, EventRec{EV_AUDIT_COMMITTED, -1, te, 0});
  if (c.v[5]) {
    put(k++, slot, EventRec{EV_AUDIT_GC_COLLECTED, -1, te, 0});
    put(k++, slot, EventRec{EV_SESSION_ARCHIVED, -1, te, 0});
  }
}

}  // namespace ahv
