// The reference pipeline (benchmarks/bench_hypervisor.py:217-239) for a batch
// of sessions that all run the same spec, written straight into the device
// store's rows — the headline path of bench.py and `Hypervisor.pipeline_batch`.
//
// One lane per session does everything the scalar API's commands do for it
// (reference core.py:94-227), in one pass and without the batched API's
// intermediate arrays (csrc/hip/store_pipeline.hip is the heterogeneous form):
//
//   create + handshake → join (K01 ring gate, admission) → activate → saga +
//   step (K13) → terminate bookkeeping (commit, GC retention, archive)
//   → D × capture: the canonical-JSON record rendered into the payload arena
//     while it is SHA-256 chained (K08), delta rows, chain head
//   → Merkle root (K09) → s_root
//
// Afterwards every session is an ordinary store session: the API's views, the
// worker's commands, verify_audit over the arena in place and checkpoints read
// these rows exactly as they read rows the per-call API wrote (one device state,
// reference core.py:92-103).
//
// Event times follow the batched API (store_pipeline.hip sp_rows): create/join/
// activate at t0, delta k at t0+1+k, the step's EXECUTING/COMMITTED at t0+D+1 /
// t0+D+2, terminate at t0+D+3.
#pragma once

#include "ahv/delta_emit.h"
#include "ahv/events.h"
#include "ahv/pipeline.h"
#include "ahv/semantics.h"
#include "ahv/store.h"

namespace ahv {

struct TemplateArgs {
  store::Tables t;
  int64_t n;                     // sessions
  const int32_t* slot;           // [n] session rows (free rows from the host allocator)
  const int32_t* gslot;          // [n] saga rows
  const int32_t* tslot;          // [n] step rows
  const int32_t* drow;           // [n·D] delta rows, session-major
  const int64_t* doff;           // [n·D] arena reservations (64-byte aligned, ≥ the padded record)
  const int32_t* session_agent;  // [n] index into the agent arrays: the agent that joins and captures
  const int32_t* agent_id;       // [A] store agent id (participant rows)
  const int32_t* agent_pool;     // [A] pool id of the agent's DID (rendered)
  const double* agent_sigma;     // [A] σ_raw (= σ_eff: no Nexus adapter in batches)
  const ChangeIds* changes;      // [D·nch] change fields per delta (shared)
  // Optional pre-rendered changes fragments (emit_changes_fragment, one per delta):
  // words [frag_off[d], …) holding frag_len[d] bytes, big-endian; null: rendered per pass
  const uint32_t* frag;
  const int32_t* frag_off;
  const int32_t* frag_len;
  StrPool pool;
  int32_t deltas;                // D ≤ kMaxDeltasPipeline
  int32_t nch;                   // changes per delta
  int32_t creator;               // store agent id of the creator DID
  int32_t maxpart;               // SessionConfig.max_participants
  double minsig;                 // SessionConfig.min_sigma_eff
  int32_t audit;                 // SessionConfig.enable_audit
  int64_t t0;                    // batch time base (µs, N09)
  uint64_t seed;                 // session ids: uuid4_words(seed, id_base + i)
  uint64_t id_base;
  int64_t gc_retention_us;       // RetentionPolicy.delta_retention_days in µs
  int32_t* status;               // [n] out (StorePipeStatus codes), or null
  unsigned long long* stats;     // [kStatSpread·kPipeStats] spread batch counters (X04), or null
  int32_t notee;                 // A/B only: digests without storing the records (AHV_TEMPLATE_AB)
  int32_t ab;                    // A/B only: 4 no Merkle root, 8 no record SHA (wrong digests), 64 per-lane tee
  // Ring mode (ring_cap > 0; GovernanceEngine's private store, which owns every row):
  // session i uses row (slot_base + i) % ring_cap for its session / saga / step rows,
  // delta rows row·dstride + d with records at off_base + (row·dstride + d)·rec_bytes,
  // and evicts whatever the row held (the slot arrays above are unused).
  int64_t ring_cap;
  int64_t slot_base;
  int32_t dstride;
  int64_t rec_bytes;
  int64_t off_base;
  uint64_t id_stride;            // session i's id counter: id_base + id_stride·i (≥ 1)
  // Device-resident {slot_base, id_base, t0} (int64[3]) or null: overrides the three
  // scalars, so a launch captured in a hipGraph stays correct on replay (N07/N09).
  const int64_t* cursor;
  EventRing ev;                  // lifecycle events (N08); ev.cursor == null: none
  uint64_t* phase_ticks;         // measurement only (or null): per-wave phase timestamps of workgroup 0
};

AHV_HD int64_t tp_slot_base(const TemplateArgs& a) { return a.cursor ? a.cursor[0] : a.slot_base; }
AHV_HD uint64_t tp_id_base(const TemplateArgs& a) { return a.cursor ? static_cast<uint64_t>(a.cursor[1]) : a.id_base; }
AHV_HD int64_t tp_t0(const TemplateArgs& a) { return a.cursor ? a.cursor[2] : a.t0; }

// Row addressing of session i (slot arrays, or the ring).
struct TemplateRows {
  int64_t s, g, ts, d0;  // session / saga / step row, index of the first delta (drow/doff or ring)
  bool ring;
  int64_t dstride, rec, off_base;
  AHV_HD int64_t drow(const TemplateArgs& a, int32_t d) const {
    return ring ? s * dstride + d : static_cast<int64_t>(a.drow[d0 + d]);
  }
  AHV_HD int64_t doff(const TemplateArgs& a, int32_t d) const {
    return ring ? off_base + (s * dstride + d) * rec : a.doff[d0 + d];
  }
};

AHV_HD TemplateRows template_rows(const TemplateArgs& a, int64_t i) {
  TemplateRows r;
  r.ring = a.ring_cap > 0;
  if (r.ring) {
    r.s = (tp_slot_base(a) + i) % a.ring_cap;
    r.g = r.s;
    r.ts = r.s;
  } else {
    r.s = a.slot[i];
    r.g = a.gslot[i];
    r.ts = a.tslot[i];
  }
  r.d0 = i * a.deltas;
  r.dstride = a.dstride;
  r.rec = a.rec_bytes;
  r.off_base = a.off_base;
  return r;
}

// Status codes (the batched API's, store_pipeline.hip).
enum TemplateStatus : int32_t { TP_OK = 0, TP_ROW_IN_USE = 1, TP_JOIN = 2, TP_ACTIVATE = 3, TP_TERMINATE = 5 };

// Bytes of a record after the opening quote of its parent digest: the quoted
// digest, the session id, the timestamp and the turn.
AHV_HD uint32_t record_suffix_len(int64_t ts_us, uint32_t turn) {
  return 66u + canon::lit_len(canon::K_SESSION) + 46u + canon::lit_len(canon::K_TS) +
         (utc_parts(ts_us).micro ? 34u : 27u) + canon::lit_len(canon::K_TURN) + canon::dec_digits(turn) +
         canon::lit_len(canon::K_CLOSE);
}

// Host twin of the device's record sink: streams the record into SHA-256 and
// into the arena at once.
struct HostTeeSink : HostSink {
  bool nohash = false;    // (device A/B knobs; the host twin always hashes and tees
  bool lane_tee = false;  //  byte by byte)
  uint8_t* dst = nullptr;
  uint32_t nb = 0;
  AHV_HD void put4(uint32_t v) {
    HostSink::put4(v);
    for (int j = 0; j < 4; ++j) dst[nb++] = static_cast<uint8_t>(v >> (24 - 8 * j));
  }
  AHV_HD void put(uint32_t v, uint32_t n) {
    HostSink::put(v, n);
    for (uint32_t j = 0; j < n; ++j) dst[nb++] = static_cast<uint8_t>(v >> (24 - 8 * j));
  }
  template <class Emit>
  AHV_HD void hash_record(Emit&& emit, uint32_t out[8], Digest&, int, uint32_t* dstw, uint32_t& len) {
    dst = reinterpret_cast<uint8_t*>(dstw);
    nb = 0;
    h.init();
    emit(*this);
    h.final(out);
    len = nb;
  }
};

// Everything of session `i` but its audit records and Merkle root: create →
// join (K01 ring gate) → activate → saga step (K13) → terminate bookkeeping.
// `u`: the session's uuid words; returns whether the terminate commits a root.
// (The caller checked that the row is free.)
AHV_HD bool template_head(const TemplateArgs& a, int64_t i, const TemplateRows& R, PipeCounters& c, uint32_t u[4]) {
  const store::Tables& t = a.t;
  const int64_t s = R.s;
  const int64_t t0 = tp_t0(a);
  const int32_t D = a.deltas;
  int32_t status = TP_OK;

  // ---- create_session + begin_handshake (OP_SESS_CREATE) ------------------------
  uuid4_words(a.seed, tp_id_base(a) + a.id_stride * static_cast<uint64_t>(i), u);
#pragma unroll
  for (int k = 0; k < 4; ++k) t.s_uuid[4 * s + k] = u[k];
  uint8_t st = SS_HANDSHAKING;
  t.s_mode[s] = 0;
  t.s_audit[s] = static_cast<uint8_t>(a.audit);
  t.s_maxpart[s] = a.maxpart;
  t.s_minsig[s] = a.minsig;
  t.s_creator[s] = a.creator;
  t.s_created[s] = t0;
  t.s_proot_n[s] = 0;

  // ---- join_session: ring gate (K01) + admission (OP_SESS_JOIN) ------------------
  const int32_t ag = a.session_agent[i];
  const double sg = a.agent_sigma[ag];
  const uint8_t ring = ring_from_sigma(sg, false);
  uint8_t code = join_check(st, false, 0, a.maxpart, sg, a.minsig, ring);
  if (code == JOIN_OK && t.cap.P < 1) code = static_cast<uint8_t>(store::JOIN_ROWS);
  const int64_t prow0 = store::prow(t, s, 0);
  int32_t pc = 0;
  if (code == JOIN_OK) {
    t.p_agent[prow0] = a.agent_id[ag];
    t.p_ring[prow0] = ring;
    t.p_sraw[prow0] = sg;
    t.p_seff[prow0] = sg;
    t.p_joined[prow0] = t0;
    pc = 1;
  } else {
    status = TP_JOIN;
  }
  t.s_pcount[s] = pc;
  t.s_pactive[s] = pc;

  // ---- activate ----------------------------------------------------------------------
  if (st == SS_HANDSHAKING && pc > 0) st = SS_ACTIVE;
  else if (status == TP_OK) status = TP_ACTIVATE;

  // ---- saga create + add_step + execute_step (K13; the executor is a no-op) ----------
  const int64_t g = R.g;
  const int64_t ts = R.ts;
  t.g_state[g] = SG_RUNNING;
  t.g_created[g] = t0;
  t.g_completed[g] = 0;
  t.g_nsteps[g] = 1;
  t.t_saga[ts] = static_cast<int32_t>(g);
  t.t_undo[ts] = 0;
  t.t_maxretry[ts] = 0;
  t.t_retry[ts] = 0;
  uint8_t step = ST_PENDING;
  if ((step_transitions(step) >> ST_EXECUTING) & 1u) step = ST_EXECUTING;
  if ((step_transitions(step) >> ST_COMMITTED) & 1u) step = ST_COMMITTED;
  t.t_state[ts] = step;
  t.t_started[ts] = t0 + D + 1;
  t.t_completed[ts] = t0 + D + 2;

  // ---- terminate: everything but the Merkle root ---------------------------------------
  // (settled before the SHA loop: only the slot, the delta rows and the digests stay live
  // across the rounds)
  const int64_t tt = t0 + D + 3;
  bool committed = false;
  t.s_released[s] = 0;  // batched sessions post no bonds
  if ((session_op_allowed_from(OP_TERMINATE) >> st) & 1u) {
    t.s_terminated[s] = tt;
    committed = a.audit && D > 0;
    int32_t retained = 0;
    for (int32_t k = 0; k < D; ++k) retained += (t0 + 1 + k >= tt - a.gc_retention_us) ? 1 : 0;
    t.s_retained[s] = retained;
    if (committed && pc) t.p_active[prow0] = store::P_ACTIVE | store::P_COMMITTED;
    else if (pc) t.p_active[prow0] = store::P_ACTIVE;
    st = SS_ARCHIVED;
  } else {
    t.s_terminated[s] = 0;
    t.s_retained[s] = 0;
    if (pc) t.p_active[prow0] = store::P_ACTIVE;
    if (status == TP_OK) status = TP_TERMINATE;
  }
  t.s_committed[s] = committed ? tt : 0;
  t.s_commit_n[s] = committed ? D : 0;
  t.s_dcount[s] = D;
  t.s_dlast[s] = D > 0 ? static_cast<int32_t>(R.drow(a, D - 1)) : -1;
  t.s_state[s] = st;
  if (a.status) a.status[i] = status;
  c.v[1] = status == TP_OK ? 1u : 0u;
  c.v[2] = static_cast<uint32_t>(pc);
  c.v[3] = static_cast<uint32_t>(D);
  c.v[4] = committed ? 1u : 0u;
  c.v[5] = st == SS_ARCHIVED ? 1u : 0u;

  return committed;
}

// Per-session body (`i` = batch index).
template <class Sink>
AHV_HD PipeCounters template_session(const TemplateArgs& a, int64_t i, Sink& sink) {
  const store::Tables& t = a.t;
  PipeCounters c{};
  c.v[0] = 1;
  const TemplateRows R = template_rows(a, i);
  const int64_t s = R.s;
  if (!R.ring && t.s_state[s] != store::kFree8) {  // a live row is never overwritten
    if (a.status) a.status[i] = TP_ROW_IN_USE;
    return c;
  }
  const int64_t t0 = tp_t0(a);
  const int32_t D = a.deltas;
  uint32_t u[4];
  const bool committed = template_head(a, i, R, c, u);
  const int32_t ag = a.session_agent[i];

  // ---- D × capture: record into the arena + SHA-256 chain (K08) ------------------------
  SessionIdent sid;
  sid.str_id = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) sid.uuid[k] = u[k];
  const StrRef did = pool_ref(a.pool, a.agent_pool[ag]);
  const bool share_block0 = did.n >= kMidstateMinDid;  // every record of the session starts with the same 64 bytes
  Digest prev, mid;
#pragma unroll
  for (int k = 0; k < 8; ++k) prev.v[k] = 0;
  const StrPool pool = a.pool;  // captured by value below (not the whole argument block)
  const uint32_t nch = static_cast<uint32_t>(a.nch);
  // Row / arena loads of delta d+1 are issued before delta d's record stores: a load
  // waited for behind stores waits for the stores too (vmcnt counts both), so nothing
  // is loaded after the first record's stores until the block-0 copies at the end.
  int32_t dr_next = D > 0 ? static_cast<int32_t>(R.drow(a, 0)) : -1;  // delta rows fit int32 (cap.D)
  int64_t off_next = D > 0 ? R.doff(a, 0) : 0;
  int32_t dr_prev = -1;
  for (int32_t d = 0; d < D; ++d) {
    const int64_t dr = dr_next;
    const int64_t off = off_next;
    if (d + 1 < D) {
      dr_next = static_cast<int32_t>(R.drow(a, d + 1));
      off_next = R.doff(a, d + 1);
    }
    uint32_t* dst = a.notee ? nullptr : reinterpret_cast<uint32_t*>(t.payload + off);
    const uint32_t turn = static_cast<uint32_t>(d + 1);
    const int64_t tsd = t0 + 1 + d;
    const int mode = !share_block0 ? MID_OFF : (d == 0 ? MID_CAPTURE : MID_RESUME);
    const ChangeIds* ch = a.changes + d * nch;
    const uint32_t* fw = a.frag ? a.frag + frag_word(reinterpret_cast<const uint32_t*>(a.frag_off), d) : nullptr;
    const uint32_t fn = a.frag ? frag_word(reinterpret_cast<const uint32_t*>(a.frag_len), d) : 0u;
    uint32_t h[8];
    uint32_t len = 0;
    sink.nohash = (a.ab & 8) != 0;
    sink.lane_tee = (a.ab & 64) != 0;
    sink.hash_record([=](Sink& k) {
      emit_delta_payload(k, pool, did, ch, nch, -1, turn, d > 0, prev, sid, tsd, fw, fn);
    }, h, mid, mode, dst, len);
    t.d_sess[dr] = static_cast<int32_t>(s);
    t.d_turn[dr] = static_cast<int32_t>(turn);
    t.d_prev[dr] = dr_prev;
    t.d_ts[dr] = tsd;
    t.d_off[dr] = off;
    t.d_len[dr] = static_cast<int32_t>(len);
    t.d_hole[dr] = d > 0 ? static_cast<int32_t>(len - record_suffix_len(tsd, turn)) : -1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      t.d_hash[8 * dr + k] = h[k];
      prev.v[k] = h[k];
    }
    dr_prev = static_cast<int32_t>(dr);
  }
  // Records resumed from the midstate did not re-emit block 0: it is the first
  // record's, copied once all the stores are out (one wait, shared with the Merkle
  // leaves' reads below).
  if (share_block0 && !a.notee && D > 1) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(t.payload + R.doff(a, 0));
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    for (int32_t d = 1; d < D; ++d) {
      // re-read per record (L1/L2 hits): 16 words held across the loop were spilled
      // to scratch at the kernel's register cap
      const uint4 c0 = s4[0], c1 = s4[1], c2 = s4[2], c3 = s4[3];
      uint4* dst = reinterpret_cast<uint4*>(t.payload + R.doff(a, d));
      dst[0] = c0;
      dst[1] = c1;
      dst[2] = c2;
      dst[3] = c3;
    }
#else
    for (int32_t d = 1; d < D; ++d) {
      uint32_t* dst = reinterpret_cast<uint32_t*>(t.payload + R.doff(a, d));
      for (int q = 0; q < 16; ++q) dst[q] = src[q];
    }
#endif
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) t.s_head[8 * s + k] = prev.v[k];

  // ---- terminate: Merkle root (K09) → commitment ---------------------------------------
  uint32_t root[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (committed && !(a.ab & 4)) {
    merkle_root_levels(
        sink, static_cast<uint32_t>(D),
        [&](uint32_t d, uint32_t hh[8]) {
          const int64_t dr = R.drow(a, static_cast<int32_t>(d));
#pragma unroll
          for (int k = 0; k < 8; ++k) hh[k] = t.d_hash[8 * dr + k];
        },
        root);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) t.s_root[8 * s + k] = root[k];
  return c;
}

// ---- lifecycle events (N08) ----------------------------------------------------------
// The records the scalar Hypervisor publishes for the same pipeline when it has an
// event bus: created → joined → ring_assigned → activated → terminated →
// audit.committed → gc_collected → archived (fewer when a stage was refused).
AHV_HD uint32_t template_event_count(const PipeCounters& c, bool terminated) {
  return 1u + (c.v[2] ? 3u : 0u) + (terminated ? 1u : 0u) + c.v[4] + 2u * c.v[5];
}

template <class Put>
AHV_HD void template_events(const TemplateArgs& a, int64_t i, const PipeCounters& c, Put&& put) {
  const store::Tables& t = a.t;
  const int64_t s = template_rows(a, i).s;
  const int32_t agent = a.agent_id[a.session_agent[i]];
  const int64_t t0 = t.s_created[s];
  const int64_t te = t.s_terminated[s];
  const int64_t prow = store::prow(t, s, 0);
  uint32_t k = 0;
  put(k++, s, EventRec{EV_SESSION_CREATED, -1, t0, 0});
  if (c.v[2]) {
    put(k++, s, EventRec{EV_SESSION_JOINED, agent, t0, 0});
    put(k++, s, EventRec{EV_RING_ASSIGNED, agent, t0, t.p_ring[prow]});
    put(k++, s, EventRec{EV_SESSION_ACTIVATED, -1, t0, 0});
  }
  if (te) put(k++, s, EventRec{EV_SESSION_TERMINATED, -1, te, 0});
  if (c.v[4]) put(k++, s, EventRec{EV_AUDIT_COMMITTED, -1, te, 0});
  if (c.v[5]) {
    put(k++, s, EventRec{EV_AUDIT_GC_COLLECTED, -1, te, 0});
    put(k++, s, EventRec{EV_SESSION_ARCHIVED, -1, te, 0});
  }
}

}  // namespace ahv
