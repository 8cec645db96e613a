// Batched governance pipeline over the *store's* tables (one device state).
//
// `Hypervisor.run_pipelines` runs the reference pipeline (benchmarks/
// bench_hypervisor.py:217-239) — generalised to heterogeneous sessions: several
// joins per session with per-agent σ (reference core.py:106-185), per-delta
// change lists, and saga steps with pre-resolved outcomes, retries and reverse-
// order compensation (saga/orchestrator.py:77-198) — for thousands of sessions
// at once, writing ordinary store rows: afterwards every session is a normal
// device session of the public API (views, reads, verify, terminate all work on
// it), unlike the standalone engine tables of models/engine.py.
//
// Three launches (render_first = 2, the default), all over rows the host allocator
// handed out (free rows; a row that is not free is refused and reported, never
// overwritten):
//
//   store_pipe_render_rows_kernel  two kinds of block, interleaved:
//     render  lane per delta: the canonical-JSON record (the shared emitters of
//             ahv/delta_emit.h) written into the payload arena, parent digest left
//             as a hole; the lane checks its session row itself
//     rows    lane per session: create (+ handshake), joins through the K01 ring
//             gate and join admission, activate, saga/step FSM (K13) with retries
//             and compensation (K14), terminate → commit → GC → archive
//             bookkeeping, chain links of its delta rows
//   store_pipe_prefix_kernel       lane per delta: SHA-256 of the record's blocks
//                                  before the parent hole (all of a turn-1 record)
//   store_pipe_chain_kernel        lane per session: the serial SHA-256 chain (K08):
//                                  each record's parent hole filled with the previous
//                                  digest, then compressed from the prefix midstate;
//                                  digests and chain head; then the Merkle root (K09)
//                                  of a committed chain into s_root (chain_roots)
//
// (render_first = 1: render alone, then store_pipe_prefix_rows_kernel — the rows blocks
// beside the prefix SHA blocks; render_first = 0: rows, render, prefix as passes of their
// own; chain_roots = 0: the K09 kernel reads the resident digests afterwards —
// store_pipeline.py.)
// Lanes take records / sessions in descending-work order (render_order,
// chain_order) so a wave's lanes finish together.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "ahv/delta_emit.h"
#include "ahv/launch.h"
#include "ahv/semantics.h"
#include "ahv/store.h"

namespace py = pybind11;

namespace ahv {
namespace {

using store::Tables;
using store::kFree8;

// Per-batch specification (host-built int32/int64/fp64 arrays on the device).
struct StorePipeArgs {
  Tables t;
  int64_t n;                    // sessions
  StrPool pool;                 // escaped strings: DIDs, change fields
  const int32_t* slot;          // [n] session rows
  const uint32_t* uuid;         // [n, 4] session id words
  const int64_t* t0;            // [n] base timestamp (µs) of each session
  const int32_t* creator;       // [n] creator agent id
  const int32_t* maxpart;       // [n]
  const double* minsig;         // [n]
  const uint8_t* flags;         // [n] bit0 audit, bit1 strong mode, bit2 activate, bit3 terminate, bit4 compensate
  const int32_t* join_off;      // [n+1]
  const int32_t* join_agent;    // [J] agent ids
  const double* join_sigma;     // [J] σ_raw (= σ_eff: no Nexus in batches)
  uint8_t* join_ring;           // [J] out: assigned ring
  uint8_t* join_code;           // [J] out: JoinCode (0 = admitted)
  const int32_t* delta_off;     // [n+1]
  const int32_t* drow;          // [Dn] delta rows
  const int32_t* dagent_pool;   // [Dn] pool id of the delta's agent DID
  const int32_t* dch_off;       // [Dn+1] change ranges
  const ChangeIds* changes;     // [C]
  const int64_t* doff;          // [Dn] arena offsets (64-aligned)
  const int32_t* dcap;          // [Dn] bytes reserved at doff
  const int32_t* gslot;         // [n] saga row (-1: no saga)
  const int32_t* step_off;      // [n+1]
  const int32_t* tslot;         // [T] step rows
  const uint8_t* step_undo;     // [T]
  const int32_t* step_retries;  // [T] max_retries
  const uint8_t* step_fail;     // [T] attempts that fail before success (≥ 1 + retries: the step fails)
  int64_t gc_retention_us;
  int32_t* status;              // [n] out: 0 ok, else first refused stage (StorePipeStatus)
  uint32_t* mid;                // [Dn, 8] SHA-256 state after a record's parent-independent blocks, or null
  int32_t* mid_blocks;          // [Dn] blocks `mid` covers (all of them for a turn-1 record: its digest)
  int32_t prefix_in_render;     // 1: the render lane compresses its record's prefix; 0: store_pipe_prefix_kernel
  const int32_t* chain_order;   // [n] sessions by descending SHA work (chain kernel lane order), or null
  const int32_t* render_order;  // [Dn] deltas by descending record size (render kernel lane order), or null
  const int32_t* prefix_order;  // [Dn] deltas grouped by prefix SHA work (prefix kernel lane order), or null
  int32_t max_nch;              // most changes of any record
  int32_t wide_only;            // lane renderer: only records with more than coop::kCoopChanges changes
  // record heads (`{"agent_did": …, "changes": […], "delta_id": "delta:`) rendered once
  // per distinct (agent, changes) of the batch (frag_pack), or null: emitted per record
  const int32_t* dfrag;         // [Dn] head of each delta
  const uint8_t* frag_bytes;    // heads, each 16-byte aligned and zero-padded
  const int64_t* frag_off;      // [F]
  const int32_t* frag_len;      // [F]
  // 1: render before rows (the render lane checks its session row itself), rows
  // blocks interleaved with the prefix SHA blocks in one launch (store_pipe_prefix_rows_kernel);
  // 2: rows blocks interleaved with the render blocks instead (store_pipe_render_rows_kernel),
  // the prefix pass on its own
  int32_t render_first;
  // 1: the chain lane folds its session's digests into the Merkle root (K09) as it
  // produces them and writes s_root of a committed row (needs `mid`: its scratch)
  int32_t chain_roots;
};

enum StorePipeStatus : int32_t {
  SP_OK = 0,
  SP_ROW_IN_USE = 1,
  SP_JOIN = 2,        // at least one join refused (its code in join_code)
  SP_ACTIVATE = 3,
  SP_STEP_FAILED = 4, // a step failed (after its retries)
  SP_TERMINATE = 5,
  SP_RENDER = 6,      // a record did not fit its reservation
};

// Event times of session i: created/joins/activate at t0, delta k at t0+1+k,
// step attempt a of step j at t0+D+1+2·(A_j+a) / +1, terminate after the last.
AHV_HD int64_t sp_delta_ts(const StorePipeArgs& a, int64_t i, int32_t k) { return a.t0[i] + 1 + k; }

AHV_HD void sp_rows(const StorePipeArgs& a, int64_t i) {
  const Tables& t = a.t;
  const int64_t s = a.slot[i];
  if (s < 0 || s >= t.cap.S || t.s_state[s] != kFree8) {
    a.status[i] = SP_ROW_IN_USE;
    return;
  }
  int32_t status = SP_OK;
  const int64_t t0 = a.t0[i];
  const uint8_t fl = a.flags[i];
  // create + begin_handshake (OP_SESS_CREATE)
  uint8_t st = SS_HANDSHAKING;
  t.s_mode[s] = (fl & 2u) ? 1 : 0;
  t.s_audit[s] = fl & 1u;
  t.s_maxpart[s] = a.maxpart[i];
  t.s_minsig[s] = a.minsig[i];
  t.s_creator[s] = a.creator[i];
  t.s_created[s] = t0;
  t.s_terminated[s] = 0;
  t.s_committed[s] = 0;
  t.s_commit_n[s] = 0;
  t.s_released[s] = 0;
  t.s_retained[s] = 0;
  t.s_proot_n[s] = 0;
  for (int k = 0; k < 4; ++k) t.s_uuid[4 * s + k] = a.uuid[4 * i + k];
  for (int k = 0; k < 8; ++k) {
    t.s_head[8 * s + k] = 0;
    t.s_root[8 * s + k] = 0;
  }
  // joins, in order: K01 ring gate + admission (OP_SESS_JOIN semantics).  The
  // duplicate check compares the session's earlier admitted joins (a bit mask over
  // its first 64 joins, in registers) instead of reading back the participant rows
  // just stored: a read after a store waits out a full memory round trip.
  int32_t pc = 0, active = 0;
  const int32_t j0 = a.join_off[i], j1 = a.join_off[i + 1];
  const int32_t maxpart = a.maxpart[i];
  const double minsig = a.minsig[i];
  uint64_t admitted = 0;
  for (int32_t j = j0; j < j1; ++j) {
    const int32_t agent = a.join_agent[j];
    const double sg = a.join_sigma[j];
    const uint8_t ring = ring_from_sigma(sg, false);
    bool dup = false;
    for (int32_t q = j0; q < j; ++q) {
      const bool adm = q - j0 < 64 ? ((admitted >> (q - j0)) & 1u) != 0 : a.join_code[q] == JOIN_OK;
      dup = dup || (adm && a.join_agent[q] == agent);
    }
    uint8_t code = join_check(st, dup, active, maxpart, sg, minsig, ring);
    if (code == JOIN_OK && pc >= t.cap.P) code = static_cast<uint8_t>(store::JOIN_ROWS);
    a.join_ring[j] = ring;
    a.join_code[j] = code;
    if (code == JOIN_OK) {
      const int64_t row = store::prow(t, s, pc);
      t.p_agent[row] = agent;
      t.p_ring[row] = ring;
      t.p_active[row] = 1;
      t.p_sraw[row] = sg;
      t.p_seff[row] = sg;
      t.p_joined[row] = t0;
      if (j - j0 < 64) admitted |= uint64_t(1) << (j - j0);
      ++pc;
      ++active;
    } else if (status == SP_OK) {
      status = SP_JOIN;
    }
  }
  t.s_pcount[s] = pc;
  t.s_pactive[s] = active;
  if (fl & 4u) {  // activate: HANDSHAKING with ≥ 1 participant row
    if (st == SS_HANDSHAKING && pc > 0) st = SS_ACTIVE;
    else if (status == SP_OK) status = SP_ACTIVATE;
  }
  // delta rows: chain links (records and digests come from the render/chain kernels)
  const int32_t d0 = a.delta_off[i], d1 = a.delta_off[i + 1];
  const int32_t nd = d1 - d0;
  t.s_dcount[s] = nd;
  t.s_dlast[s] = nd > 0 ? a.drow[d1 - 1] : -1;
  int64_t tnext = t0 + 1 + nd;
  // saga: steps executed in order with their pre-resolved outcomes (K13), retries
  // reset to PENDING between attempts as the reference does (orchestrator.py:124/134).
  // Each step's state is settled in registers and stored once; the committed steps
  // (first 64) are a bit mask for the compensation pass.
  const int32_t g = a.gslot[i];
  if (g >= 0) {
    const int32_t k0 = a.step_off[i], k1 = a.step_off[i + 1];
    t.g_state[g] = SG_RUNNING;
    t.g_created[g] = t0;
    t.g_completed[g] = 0;
    t.g_nsteps[g] = k1 - k0;
    bool failed = false;
    uint64_t committed = 0;
    for (int32_t k = k0; k < k1; ++k) {
      const int32_t ts = a.tslot[k];
      uint8_t sst = ST_PENDING;
      int32_t rt = 0;
      int64_t started = 0, completed = 0;
      if (!failed) {  // the caller stops at the first failed step
        const int32_t attempts = 1 + a.step_retries[k];
        const int32_t fails = a.step_fail[k];
        for (int32_t at = 0; at < attempts; ++at) {
          rt = at;
          started = tnext++;
          if (at >= fails) {
            sst = ST_COMMITTED;
            completed = tnext++;
            break;
          }
          completed = tnext++;
          sst = at < attempts - 1 ? ST_PENDING : ST_FAILED;
        }
        if (sst == ST_FAILED) {
          failed = true;
          if (status == SP_OK) status = SP_STEP_FAILED;
        }
      }
      t.t_saga[ts] = g;
      t.t_state[ts] = sst;
      t.t_undo[ts] = a.step_undo[k];
      t.t_maxretry[ts] = a.step_retries[k];
      t.t_retry[ts] = rt;
      t.t_started[ts] = started;
      t.t_completed[ts] = completed;
      if (sst == ST_COMMITTED && k - k0 < 64) committed |= uint64_t(1) << (k - k0);
    }
    if (failed && (fl & 16u)) {  // compensate: committed steps in reverse (K14)
      int32_t comp_failed = 0;
      for (int32_t k = k1 - 1; k >= k0; --k) {
        const int32_t ts = a.tslot[k];
        const bool was = k - k0 < 64 ? ((committed >> (k - k0)) & 1u) != 0 : t.t_state[ts] == ST_COMMITTED;
        if (!was) continue;
        if (!a.step_undo[k]) {
          t.t_state[ts] = ST_COMPENSATION_FAILED;  // "No Undo_API available" (set directly, no stamp)
          ++comp_failed;
          continue;
        }
        t.t_state[ts] = ST_COMPENSATED;  // COMPENSATING → COMPENSATED
        t.t_completed[ts] = tnext++;
      }
      t.g_state[g] = comp_failed ? SG_ESCALATED : SG_COMPLETED;
      t.g_completed[g] = tnext++;
    }
  }
  // terminate → Merkle root (K09, afterwards) → commit → bond release → GC → archive
  if (fl & 8u) {
    if ((session_op_allowed_from(OP_TERMINATE) >> st) & 1u) {
      const int64_t tt = tnext++;
      t.s_terminated[s] = tt;
      if ((fl & 1u) && nd > 0) {
        t.s_committed[s] = tt;
        t.s_commit_n[s] = nd;
        for (int32_t k = 0; k < pc; ++k) t.p_active[store::prow(t, s, k)] = store::P_ACTIVE | store::P_COMMITTED;
      }
      int32_t retained = 0;
      for (int32_t k = 0; k < nd; ++k) retained += sp_delta_ts(a, i, k) >= tt - a.gc_retention_us ? 1 : 0;
      t.s_retained[s] = retained;
      t.s_released[s] = 0;  // batched sessions post no bonds
      st = SS_ARCHIVED;
    } else if (status == SP_OK) {
      status = SP_TERMINATE;
    }
  }
  t.s_state[s] = st;
  // a record that overflowed its reservation outranks the other stages' codes
  // (render ran first: its SP_RENDER is already in status)
  if (a.render_first == 2) {  // the render pass runs beside this one: the larger code wins (SP_RENDER)
#if defined(__HIP_DEVICE_COMPILE__)
    atomicMax(&a.status[i], status);
#else
    a.status[i] = a.status[i] > status ? a.status[i] : status;
#endif
  } else if (!a.render_first || a.status[i] != SP_RENDER) {
    a.status[i] = status;
  }
}

// The render-first layout: the session row is free for this batch (the rows pass
// checks the same and has not written s_state yet when the render lanes run).
AHV_HD bool sp_row_in_use(const StorePipeArgs& a, int64_t i) {
  const int64_t s = a.slot[i];
  return s < 0 || s >= a.t.cap.S || a.t.s_state[s] != kFree8;
}

// Bytes of one record, written straight to the arena (records start 64-byte
// aligned, reservations are whole 64-byte lines).  Big-endian chunks from the
// emitters → little-endian memory words, staged four at a time so the arena sees
// one 16-byte store per 16 bytes (a quarter of the store instructions of a word
// sink; each lane writes its own record, so every store is its own cache line).
AHV_HD void store4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
  *reinterpret_cast<uint4*>(p) = make_uint4(a, b, c, d);
#else
  p[0] = a;
  p[1] = b;
  p[2] = c;
  p[3] = d;
#endif
}

// kFlat (default): put() and word() are straight-line — the word completion and
// the 16-byte chunk completion are selects, and the one branch left per put is
// the chunk's store.  The staged form (kFlat = false, AHV_SP_SINK=staged) branches
// on both, and every divergent branch costs the wave exec-mask bookkeeping (the
// r6 ISA of the render kernel: ≈ 4 SALU mask / branch instructions per put).
template <bool kFlat>
struct ArenaSinkT {
  uint32_t* dst;
  uint32_t cap_w;
  uint32_t nw = 0;   // words in memory (a multiple of 4 until flush)
  uint32_t nq = 0;   // staged words (0..3), in q0..q2 (named: no runtime-indexed array)
  uint32_t q0 = 0, q1 = 0, q2 = 0;
  uint32_t acc = 0;  // pending bytes in memory order
  uint32_t nb = 0;   // pending byte count
  AHV_HD bool seg(uint32_t) { return true; }
  AHV_HD bool any(bool b) const { return b; }
  template <class T>
  AHV_HD void launder(T&) const {}
  AHV_HD uint32_t pos() const { return 4 * (nw + nq) + nb; }
  // Stage w when `take`; a completed chunk is stored if it lies inside the
  // reservation (past it the record overflows, SP_RENDER: its bytes are void).
  AHV_HD void stage(uint32_t w, bool take) {
    const bool done = take && nq == 3;
    if (done && nw + 4 <= cap_w) store4(dst + nw, q0, q1, q2, w);
    q0 = take && nq == 0 ? w : q0;
    q1 = take && nq == 1 ? w : q1;
    q2 = take && nq == 2 ? w : q2;
    nw += done ? 4u : 0u;
    nq = take ? (nq + 1) & 3u : nq;
  }
  AHV_HD void word(uint32_t w) {
    if (kFlat) {
      stage(w, true);
      return;
    }
    if (nq == 3) {
      if (nw + 4 <= cap_w) {
        store4(dst + nw, q0, q1, q2, w);
      } else {  // past the reservation: the record overflows (SP_RENDER); keep what fits
        if (nw < cap_w) dst[nw] = q0;
        if (nw + 1 < cap_w) dst[nw + 1] = q1;
        if (nw + 2 < cap_w) dst[nw + 2] = q2;
      }
      nw += 4;
      nq = 0;
      return;
    }
    q0 = nq == 0 ? w : q0;
    q1 = nq == 1 ? w : q1;
    q2 = nq == 2 ? w : q2;
    ++nq;
  }
  AHV_HD void byte(uint32_t b) {
    acc |= (b & 0xffu) << (8 * nb);
    if (++nb == 4) {
      word(acc);
      acc = 0;
      nb = 0;
    }
  }
  // The top n ≤ 4 bytes of v appended after the nb pending bytes with one funnel
  // shift (at most one word completes), not n byte steps: n and nb differ per
  // lane, and a per-byte loop made every lane of a wave run the longest one.
  AHV_HD void put(uint32_t v, uint32_t n) {
    const uint32_t m = n >= 4 ? 0xffffffffu : (1u << (8 * n)) - 1u;
    const uint32_t tot = nb + n;
    if (kFlat) {
      const uint32_t vv = bswap32(v) & m;
      const uint32_t sh = 8 * nb;  // 0..24
      const uint32_t lo = acc | (vv << sh);
      const uint32_t hi = nb ? vv >> (32u - sh) : 0u;
      const bool full = tot >= 4;
      stage(lo, full);
      acc = full ? hi : lo;
      nb = full ? tot - 4 : tot;
      return;
    }
    const uint64_t x = static_cast<uint64_t>(acc) | (static_cast<uint64_t>(bswap32(v) & m) << (8 * nb));
    if (tot >= 4) {
      word(static_cast<uint32_t>(x));
      acc = static_cast<uint32_t>(x >> 32);
      nb = tot - 4;
    } else {
      acc = static_cast<uint32_t>(x);
      nb = tot;
    }
  }
  AHV_HD void put4(uint32_t v) { put(v, 4); }
  AHV_HD void flush() {
    if (nb) {
      word(acc);
      acc = 0;
      nb = 0;
    }
    if (nq > 0 && nw < cap_w) dst[nw] = q0;
    if (nq > 1 && nw + 1 < cap_w) dst[nw + 1] = q1;
    if (nq > 2 && nw + 2 < cap_w) dst[nw + 2] = q2;
    nw += nq;
    nq = 0;
  }
};

// Lane per delta g (session `i`, turn k+1): render the record; the parent digest
// is rendered as 66 placeholder bytes whose offset is recorded (d_hole).
// Block `b` of the SHA-256 message of a `len`-byte record at w32 (big-endian
// words, 0x80 terminator and bit length in the last of its `nblk` blocks).
// The raw (little-endian) words of block b: 16-byte loads of the chunks that start
// inside the record (reservations are whole 64-byte lines, so a chunk that starts
// before `len` lies inside them), zeros past it.
AHV_HD void sp_block_raw(const uint32_t* w32, uint64_t len, uint64_t b, uint32_t raw[16]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint64_t o = 64 * b + 16 * c;
    uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;
    if (o < len) {
#if defined(__HIP_DEVICE_COMPILE__)
      const uint4 v = *reinterpret_cast<const uint4*>(w32 + o / 4);
      x0 = v.x;
      x1 = v.y;
      x2 = v.z;
      x3 = v.w;
#else
      x0 = w32[o / 4];
      x1 = w32[o / 4 + 1];
      x2 = w32[o / 4 + 2];
      x3 = w32[o / 4 + 3];
#endif
    }
    raw[4 * c] = x0;
    raw[4 * c + 1] = x1;
    raw[4 * c + 2] = x2;
    raw[4 * c + 3] = x3;
  }
}

// Message words of block b from its raw words: big-endian, the 0x80 terminator and
// the bit length in the last of the record's `nblk` blocks.
AHV_HD void sp_block_words(const uint32_t raw[16], uint64_t len, uint64_t nblk, uint64_t b, uint32_t blk[16]) {
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const uint64_t o = 64 * b + 4 * w;
    uint32_t x = 0;
    if (o + 4 <= len) {
      x = bswap32(raw[w]);
    } else if (o < len) {
      x = bswap32(raw[w]) & (0xffffffffu << (8 * (4 - (len - o))));
    }
    if (o <= len && len < o + 4) x |= 0x80u << (8 * (3 - (len - o)));
    if (b == nblk - 1 && w == 14) x |= static_cast<uint32_t>((len * 8) >> 32);
    if (b == nblk - 1 && w == 15) x |= static_cast<uint32_t>(len * 8);
    blk[w] = x;
  }
}

AHV_HD void sp_block(const uint32_t* w32, uint64_t len, uint64_t nblk, uint64_t b, uint32_t blk[16]) {
  uint32_t raw[16];
  sp_block_raw(w32, len, b, raw);
  sp_block_words(raw, len, nblk, b, blk);
}

AHV_HD void sp_prefix(const StorePipeArgs& a, int64_t g);

// A pool string's (pointer, length) with unconditional loads (an absent string, id −1,
// reads entry 0 — a record's agent DID is always in the pool — and reports length −1).
AHV_HD StrRef pool_ref_flat(const StrPool& pool, int32_t id) {
  const int32_t j = id < 0 ? 0 : id;
  const int64_t off = pool.off[j];
  const int32_t len = pool.len[j];
  return StrRef{pool.bytes + off, id < 0 ? -1 : len};
}

// kHoist: the loads whose values are needed only later — the session id words, the
// base time, the agent DID's pool entry, each change's four pool entries and the next
// change's ids — are issued ahead of the stores that precede their use, so the lane does
// not wait for a load after every string it emits (AHV_SP_HOIST=0: in line).
template <bool kFlat = true, bool kHoist = true>
AHV_HD void sp_render(const StorePipeArgs& a, int64_t i, int32_t g) {
  const Tables& t = a.t;
  const int32_t k = g - a.delta_off[i];
  const int32_t d = a.drow[g];
  const int64_t s = a.slot[i];
  uint32_t uw[4] = {0, 0, 0, 0};
  int64_t ts = 0;
  StrRef agent{nullptr, -1};
  if (kHoist) {
#pragma unroll
    for (int q = 0; q < 4; ++q) uw[q] = a.uuid[4 * i + q];
    ts = sp_delta_ts(a, i, k);
  }
  ArenaSinkT<kFlat> snk;
  snk.dst = reinterpret_cast<uint32_t*>(t.payload + a.doff[g]);
  snk.cap_w = static_cast<uint32_t>(a.dcap[g]) / 4;
  const ChangeIds* ch = a.changes + a.dch_off[g];
  const uint32_t nch = static_cast<uint32_t>(a.dch_off[g + 1] - a.dch_off[g]);
  const uint32_t turn = static_cast<uint32_t>(k + 1);
  if (a.dfrag != nullptr) {
    // the head, pre-rendered: whole 16-byte chunks straight into the record (both
    // 16-aligned), its last partial chunk into the sink, which continues after it
    const int32_t f = a.dfrag[g];
    const uint32_t hl = static_cast<uint32_t>(a.frag_len[f]);
    const U4* src = reinterpret_cast<const U4*>(a.frag_bytes + a.frag_off[f]);
    const uint32_t full = hl / 16;
    for (uint32_t c = 0; c < full; ++c) {
      const U4 v = src[c];
      if (4 * c + 4 <= snk.cap_w) store4(snk.dst + 4 * c, v.a, v.b, v.c, v.d);
    }
    snk.nw = 4 * full;
    const uint32_t rem = hl - 16 * full;
    if (rem) {
      const U4 v = src[full];  // zero-padded past the head
      const uint32_t nwd = rem / 4, nb = rem % 4;
      if (nwd > 0) snk.word(v.a);
      if (nwd > 1) snk.word(v.b);
      if (nwd > 2) snk.word(v.c);
      if (nb) {
        snk.acc = nwd == 0 ? v.a : nwd == 1 ? v.b : nwd == 2 ? v.c : v.d;
        snk.nb = nb;
      }
    }
  } else if (kHoist) {
    agent = pool_ref_flat(a.pool, a.dagent_pool[g]);
    ChangeIds nx = nch > 0 ? ch[0] : ChangeIds{-1, -1, -1, -1};
    emit_lit(snk, canon::K_OPEN_AGENT);
    emit_str_ref(snk, agent);
    emit_lit(snk, canon::K_CHANGES);
    for (uint32_t c = 0; c < nch; ++c) {
      const StrRef rc = pool_ref_flat(a.pool, nx.content_hash), ro = pool_ref_flat(a.pool, nx.op);
      const StrRef rp = pool_ref_flat(a.pool, nx.path), rv = pool_ref_flat(a.pool, nx.previous_hash);
      if (c + 1 < nch) nx = ch[c + 1];
      if (c) emit_lit(snk, canon::K_CH_SEP);
      emit_lit(snk, canon::K_CH_OPEN);
      emit_str_ref(snk, rc);
      emit_lit(snk, canon::K_CH_OP);
      emit_str_ref(snk, ro);
      emit_lit(snk, canon::K_CH_PATH);
      emit_str_ref(snk, rp);
      emit_lit(snk, canon::K_CH_PREV);
      emit_str_ref(snk, rv);
      emit_lit(snk, canon::K_CH_CLOSE);
    }
    emit_lit(snk, canon::K_DELTA_ID);
    emit_lit(snk, canon::K_DELTA_PFX);
  } else {
    emit_lit(snk, canon::K_OPEN_AGENT);
    emit_str_ref(snk, pool_ref(a.pool, a.dagent_pool[g]));
    emit_lit(snk, canon::K_CHANGES);
    for (uint32_t c = 0; c < nch; ++c) {
      if (c) emit_lit(snk, canon::K_CH_SEP);
      emit_lit(snk, canon::K_CH_OPEN);
      emit_pool_str(snk, a.pool, ch[c].content_hash);
      emit_lit(snk, canon::K_CH_OP);
      emit_pool_str(snk, a.pool, ch[c].op);
      emit_lit(snk, canon::K_CH_PATH);
      emit_pool_str(snk, a.pool, ch[c].path);
      emit_lit(snk, canon::K_CH_PREV);
      emit_pool_str(snk, a.pool, ch[c].previous_hash);
      emit_lit(snk, canon::K_CH_CLOSE);
    }
    emit_lit(snk, canon::K_DELTA_ID);
    emit_lit(snk, canon::K_DELTA_PFX);
  }
  emit_uint(snk, turn);
  emit_char(snk, 0x22u);
  emit_lit(snk, canon::K_PARENT);
  int32_t hole = -1;
  if (turn > 1) {
    hole = static_cast<int32_t>(snk.pos());
    for (int b = 0; b < 16; ++b) snk.put4(0x22222222u);  // 66-byte placeholder: the chain kernel
    snk.put(0x22220000u, 2);                              // writes the quoted digest into it
  } else {
    emit_lit(snk, canon::K_NULL);
  }
  emit_lit(snk, canon::K_SESSION);
  emit_session_uuid_quoted(snk, kHoist ? uw : a.uuid + 4 * i);
  emit_lit(snk, canon::K_TS);
  emit_iso_quoted(snk, kHoist ? ts : sp_delta_ts(a, i, k));
  emit_lit(snk, canon::K_TURN);
  emit_uint(snk, turn);
  emit_lit(snk, canon::K_CLOSE);
  const uint32_t len = snk.pos();
  snk.flush();
  t.d_sess[d] = static_cast<int32_t>(s);
  t.d_turn[d] = static_cast<int32_t>(turn);
  t.d_prev[d] = k > 0 ? a.drow[g - 1] : -1;
  t.d_ts[d] = sp_delta_ts(a, i, k);
  t.d_off[d] = a.doff[g];
  t.d_len[d] = static_cast<int32_t>(len);
  t.d_hole[d] = hole;
  if (len > static_cast<uint32_t>(a.dcap[g])) a.status[i] = SP_RENDER;
  if (a.mid && a.prefix_in_render) sp_prefix(a, g);  // the record is still hot in this lane's cache lines
}

// K08 split (lane per record; in the render pass or its own pass): the blocks before the parent hole
// (sort_keys puts agent_did, changes and delta_id first) — or the whole record
// of turn 1 — do not depend on the chain, so they are compressed here in
// parallel over records, and the serial chain pass resumes from this state.
// Kept out of the render pass: the SHA rounds are uniform control flow, the
// rendering is not (its lanes diverge on string lengths and field kinds).
// kPipe: block b+1's four 16-byte loads are issued before block b is compressed, so a
// lane's next block is in flight while it runs 64 rounds (the prefix blocks lie wholly
// inside the record: no padding to apply).  AHV_SP_PREFIX_PIPE=0: load, then compress.
template <bool kPipe>
AHV_HD void sp_prefix_t(const StorePipeArgs& a, int64_t g) {
  const Tables& t = a.t;
  const int32_t d = a.drow[g];
  const uint32_t len = static_cast<uint32_t>(t.d_len[d]);
  if (len > static_cast<uint32_t>(a.dcap[g])) {  // overflowed its reservation (SP_RENDER)
    a.mid_blocks[g] = 0;
    return;
  }
  const int32_t hole = t.d_hole[d];
  const uint64_t nblk = (static_cast<uint64_t>(len) + 9 + 63) / 64;
  const uint64_t pb = hole >= 0 ? static_cast<uint64_t>(hole) / 64 : nblk;
  uint32_t h[8];
  sha256_init(h);
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(t.payload + a.doff[g]);
  if (kPipe && hole >= 0) {
    const U4* src = reinterpret_cast<const U4*>(w32);
    U4 n0{0u, 0u, 0u, 0u}, n1 = n0, n2 = n0, n3 = n0;
    if (pb > 0) {
      n0 = src[0];
      n1 = src[1];
      n2 = src[2];
      n3 = src[3];
    }
    for (uint64_t b = 0; b < pb; ++b) {
      const U4 c0 = n0, c1 = n1, c2 = n2, c3 = n3;
      if (b + 1 < pb) {
        n0 = src[4 * (b + 1)];
        n1 = src[4 * (b + 1) + 1];
        n2 = src[4 * (b + 1) + 2];
        n3 = src[4 * (b + 1) + 3];
      }
      const uint32_t blk[16] = {bswap32(c0.a), bswap32(c0.b), bswap32(c0.c), bswap32(c0.d),
                                bswap32(c1.a), bswap32(c1.b), bswap32(c1.c), bswap32(c1.d),
                                bswap32(c2.a), bswap32(c2.b), bswap32(c2.c), bswap32(c2.d),
                                bswap32(c3.a), bswap32(c3.b), bswap32(c3.c), bswap32(c3.d)};
      sha256_compress(h, blk);
    }
  } else {
    for (uint64_t b = 0; b < pb; ++b) {
      uint32_t blk[16];
      sp_block(w32, len, nblk, b, blk);
      sha256_compress(h, blk);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) a.mid[8 * g + k] = h[k];
  a.mid_blocks[g] = static_cast<int32_t>(pb);
}

AHV_HD void sp_prefix(const StorePipeArgs& a, int64_t g) { sp_prefix_t<true>(a, g); }

// Lane per session: the SHA-256 chain over its records (K08).
template <bool kPipe = true>
AHV_HD void sp_chain(const StorePipeArgs& a, int64_t i) {
  const Tables& t = a.t;
  const int64_t s = a.slot[i];
  uint32_t prev[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int32_t g = a.delta_off[i]; g < a.delta_off[i + 1]; ++g) {
    const int32_t d = a.drow[g];
    uint8_t* rec = t.payload + t.d_off[d];
    const uint64_t len = static_cast<uint64_t>(t.d_len[d]);
    const int32_t hole = t.d_hole[d];
    if (hole >= 0) {  // '"' + hex(prev) + '"' into the record
#pragma unroll
      for (int q = 0; q < 8; ++q) {
#pragma unroll
        for (int e = 0; e < 8; ++e) rec[hole + 1 + 8 * q + e] = static_cast<uint8_t>(hex_nibble((prev[q] >> (28 - 4 * e)) & 15u));
      }
    }
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(rec);
    uint32_t h[8];
    const uint64_t nblk = (len + 9 + 63) / 64;
    const uint64_t pb = a.mid ? static_cast<uint64_t>(a.mid_blocks[g]) : 0;  // compressed by the render pass
    if (pb > 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = a.mid[8 * static_cast<int64_t>(g) + k];
    } else {
      sha256_init(h);
    }
    if (kPipe) {  // block b+1's loads in flight while block b compresses
      uint32_t nx[16];
      if (pb < nblk) sp_block_raw(w32, len, pb, nx);
      for (uint64_t b = pb; b < nblk; ++b) {
        uint32_t raw[16], blk[16];
#pragma unroll
        for (int w = 0; w < 16; ++w) raw[w] = nx[w];
        if (b + 1 < nblk) sp_block_raw(w32, len, b + 1, nx);
        sp_block_words(raw, len, nblk, b, blk);
        sha256_compress(h, blk);
      }
    } else {
      for (uint64_t b = pb; b < nblk; ++b) {
        uint32_t blk[16];
        sp_block(w32, len, nblk, b, blk);
        sha256_compress(h, blk);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      t.d_hash[8 * static_cast<int64_t>(d) + k] = h[k];
      prev[k] = h[k];
    }
  }
  if (a.delta_off[i + 1] > a.delta_off[i]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) t.s_head[8 * s + k] = prev[k];
  }
}

// K09 in the chain lane: the session's Merkle root over the digests its chain just
// produced (still in this lane's cache lines), as a binary counter whose ≤ ⌊log2 n⌋+1
// partial subtrees are parked in the session's own `mid` rows — spent by then: a
// record's row is read before its digest exists, and slot L ≤ log2(k+1) ≤ k.  Same
// tree as merkle_kernel (reference audit/delta.py:117-134, odd node duplicated).
struct MidStash {
  uint32_t* rows;
  AHV_HD void stash(int j, const uint32_t d[8]) {
    for (int k = 0; k < 8; ++k) rows[j * 8 + k] = d[k];
  }
  AHV_HD void load(int j, uint32_t d[8]) const {
    for (int k = 0; k < 8; ++k) d[k] = rows[j * 8 + k];
  }
  AHV_HD void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) const {
    uint32_t t[8];
    merkle_node(l, r, t);
    for (int k = 0; k < 8; ++k) out[k] = t[k];
  }
};

AHV_HD void sp_chain_root(const StorePipeArgs& a, int64_t i) {
  const Tables& t = a.t;
  const int64_t s = a.slot[i];
  const int32_t d0 = a.delta_off[i], d1 = a.delta_off[i + 1];
  if (d1 <= d0 || t.s_committed[s] == 0) return;  // no root: s_root stays as the rows pass zeroed it
  MidStash ms{a.mid + 8 * static_cast<int64_t>(d0)};
  uint32_t r[8];
  merkle_root_counter(
      ms, static_cast<uint32_t>(d1 - d0),
      [&](uint32_t k, uint32_t h[8]) {
        const int64_t d = a.drow[d0 + static_cast<int32_t>(k)];
        for (int q = 0; q < 8; ++q) h[q] = t.d_hash[8 * d + q];
      },
      r);
  for (int k = 0; k < 8; ++k) t.s_root[8 * s + k] = r[k];
}

__global__ __launch_bounds__(256) void store_pipe_rows_kernel(StorePipeArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.n) sp_rows(a, i);
}

// lane per record (records in render_order: similar sizes per wave)
template <bool kPipe>
__global__ __launch_bounds__(256) void store_pipe_prefix_kernel(StorePipeArgs a, const int32_t* dsess, int64_t nd) {
  const int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (x < nd) {
    // lanes of a wave hash records with the same number of parent-independent blocks
    // (prefix_order: turn-1 records, whole record, first, then by reserved size)
    const int64_t g = a.prefix_order ? a.prefix_order[x] : a.render_order ? a.render_order[x] : x;
    if (a.status[dsess[g]] != SP_ROW_IN_USE) sp_prefix_t<kPipe>(a, g);
    else a.mid_blocks[g] = 0;
  }
}

// lane per delta; `dsess` maps a delta to its session
template <bool kFlat, bool kHoist>
__global__ __launch_bounds__(256) void store_pipe_render_kernel(StorePipeArgs a, const int32_t* dsess, int64_t nd) {
  const int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (x < nd) {
    const int64_t g = a.render_order ? a.render_order[x] : x;  // records of similar size per wave
    const int64_t i = dsess[g];
    if (a.render_first) {
      if (sp_row_in_use(a, i)) a.status[i] = SP_ROW_IN_USE;  // (every lane of the session writes the same)
      else sp_render<kFlat, kHoist>(a, i, static_cast<int32_t>(g));
    } else if (a.status[i] != SP_ROW_IN_USE && (!a.wide_only || a.dch_off[g + 1] - a.dch_off[g] > 4)) {
      sp_render<kFlat, kHoist>(a, i, static_cast<int32_t>(g));
    }
  }
}

// Render-first layout: the rows pass (memory-latency bound: 672 VALU per lane, r6
// PMC) and the prefix SHA pass (VALU bound) in one grid, their blocks interleaved
// in proportion, so each CU runs both kinds of wave side by side and the rows'
// memory waits hide under SHA issue instead of taking their own 215 µs pass.
// Neither reads what the other writes: prefix reads the records and status codes
// the render pass left (SP_ROW_IN_USE, written there for in-use rows); rows writes
// the session / participant / saga rows and the other codes, never SP_ROW_IN_USE
// for a row that is free.
__global__ __launch_bounds__(256) void store_pipe_prefix_rows_kernel(StorePipeArgs a, const int32_t* dsess, int64_t nd,
                                                                     uint32_t nrows_blk, uint32_t nblk) {
  const uint64_t b = blockIdx.x;
  const uint64_t r0 = b * nrows_blk / nblk, r1 = (b + 1) * nrows_blk / nblk;  // rows blocks before / through b
  if (r1 > r0) {
    const int64_t i = static_cast<int64_t>(r0) * blockDim.x + threadIdx.x;
    if (i < a.n) sp_rows(a, i);
    return;
  }
  const int64_t x = static_cast<int64_t>(b - r0) * blockDim.x + threadIdx.x;
  if (x < nd) {
    const int64_t g = a.prefix_order ? a.prefix_order[x] : a.render_order ? a.render_order[x] : x;
    if (a.status[dsess[g]] != SP_ROW_IN_USE) sp_prefix(a, g);
    else a.mid_blocks[g] = 0;
  }
}

// render_first = 2: the rows blocks interleaved with the render blocks (both wait on
// memory most of the time: rows on its scattered row writes, render on its string loads).
// Status codes meet through atomicMax (SP_RENDER, the largest, wins).
template <bool kHoist>
__global__ __launch_bounds__(256) void store_pipe_render_rows_kernel(StorePipeArgs a, const int32_t* dsess, int64_t nd,
                                                                     uint32_t nrows_blk, uint32_t nblk) {
  const uint64_t b = blockIdx.x;
  const uint64_t r0 = b * nrows_blk / nblk, r1 = (b + 1) * nrows_blk / nblk;
  if (r1 > r0) {
    const int64_t i = static_cast<int64_t>(r0) * blockDim.x + threadIdx.x;
    if (i < a.n) sp_rows(a, i);
    return;
  }
  const int64_t x = static_cast<int64_t>(b - r0) * blockDim.x + threadIdx.x;
  if (x < nd) {
    const int64_t g = a.render_order ? a.render_order[x] : x;
    const int64_t i = dsess[g];
    if (sp_row_in_use(a, i)) a.status[i] = SP_ROW_IN_USE;
    else sp_render<true, kHoist>(a, i, static_cast<int32_t>(g));
  }
}

// A lane's chain is serial and its length varies per session (0..k deltas of
// varying size): lanes take sessions in descending-work order (chain_order), so
// the 64 chains of a wave are about equally long and the wave does not idle most
// lanes while its longest chain finishes.
template <bool kPipe>
__global__ __launch_bounds__(64) void store_pipe_chain_kernel(StorePipeArgs a) {
  const int64_t x = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (x >= a.n) return;
  const int64_t i = a.chain_order ? a.chain_order[x] : x;
  if (a.status[i] != SP_ROW_IN_USE) {
    sp_chain<kPipe>(a, i);
    if (a.chain_roots) sp_chain_root(a, i);
  }
}

// ------------------------------------------------- wave-cooperative renderer
//
// store_pipe_render_kernel gives each lane a whole record: its emission branches
// on field kinds, null values and string lengths, so the wave runs every lane's
// path and half its lanes idle (r3 PMC: 48 % lane utilisation).  Here 16 lanes
// render one record:
//
//   1. layout — the record is a fixed schema of 18 + 18·nch pieces (literals,
//      quotes, pool string bodies, "null", the 66-byte parent placeholder and the
//      generated turn / session-uuid / timestamp text); lane j resolves pieces
//      j, j+16, … to (source, length) in LDS — a handful of uniform selects — and
//      the group prefix-sums the lengths (one 16-lane shuffle scan);
//   2. assembly — lane j builds output words j, j+16, … : each word is 1–2
//      funnel-shifted reads of the piece(s) covering its 4 bytes, found by a short
//      forward walk over the piece offsets; the 16 lanes store 64 contiguous bytes
//      per instruction.
//
// A wave renders its 64 records (in render_order: similar shapes together) 64/G
// at a time; store_pipe_prefix_kernel then compresses each record's parent-
// independent blocks one record per lane (uniform SHA control flow).
// Same bytes as sp_render (the CPU twin), checked by the batch tests' digests.
namespace coop {

constexpr int kCoopChanges = 4;      // records with more changes take the lane renderer
constexpr int kMaxPieces = 18 + 18 * kCoopChanges;
constexpr int kGenBytes = 128;       // generated text: turn digits, "session:…", "…timestamp…"

enum Lit : int {
  L_OPEN_AGENT, L_CHANGES, L_CH_OPEN, L_CH_OP, L_CH_PATH, L_CH_PREV, L_CH_CLOSE, L_CH_SEP, L_DELTA_ID,
  L_DELTA_PFX, L_PARENT, L_SESSION, L_TS, L_TURN, L_CLOSE, L_NULL, L_QUOTE, L_HOLE, L_COUNT
};

struct Lits {
  uint8_t b[352] = {};
  uint16_t off[L_COUNT] = {};
  uint16_t len[L_COUNT] = {};
  template <size_t N>
  constexpr void add(size_t& p, int i, const char (&v)[N]) {
    off[i] = static_cast<uint16_t>(p);
    len[i] = static_cast<uint16_t>(N - 1);
    for (size_t k = 0; k + 1 < N; ++k) b[p++] = static_cast<uint8_t>(v[k]);
    p = (p + 3) & ~size_t(3);
  }
  constexpr Lits() {
    size_t p = 0;
    add(p, L_OPEN_AGENT, canon::K_OPEN_AGENT);
    add(p, L_CHANGES, canon::K_CHANGES);
    add(p, L_CH_OPEN, canon::K_CH_OPEN);
    add(p, L_CH_OP, canon::K_CH_OP);
    add(p, L_CH_PATH, canon::K_CH_PATH);
    add(p, L_CH_PREV, canon::K_CH_PREV);
    add(p, L_CH_CLOSE, canon::K_CH_CLOSE);
    add(p, L_CH_SEP, canon::K_CH_SEP);
    add(p, L_DELTA_ID, canon::K_DELTA_ID);
    add(p, L_DELTA_PFX, canon::K_DELTA_PFX);
    add(p, L_PARENT, canon::K_PARENT);
    add(p, L_SESSION, canon::K_SESSION);
    add(p, L_TS, canon::K_TS);
    add(p, L_TURN, canon::K_TURN);
    add(p, L_CLOSE, canon::K_CLOSE);
    add(p, L_NULL, canon::K_NULL);
    add(p, L_QUOTE, "\"");
    off[L_HOLE] = static_cast<uint16_t>(p);  // the parent placeholder: 66 quote bytes
    len[L_HOLE] = 66;
    for (int k = 0; k < 66; ++k) b[p++] = 0x22;
  }
};

// in global memory (a constexpr device object indexed at run time would be
// copied into per-lane scratch)
__device__ Lits kLits = Lits();

// Generated text of one record, in LDS: [0,16) turn digits, [16,64) the quoted
// session id, [64,128) the quoted timestamp.
struct GenSink {
  uint8_t* p;
  uint32_t n;
  __device__ bool seg(uint32_t) { return true; }
  __device__ bool any(bool b) const { return b; }
  template <class T>
  __device__ void launder(T&) const {}
  __device__ void put(uint32_t v, uint32_t k) {
    for (uint32_t j = 0; j < k; ++j) p[n++] = static_cast<uint8_t>(v >> (24 - 8 * j));
  }
  __device__ void put4(uint32_t v) { put(v, 4); }
};

struct Group {  // one record's layout (LDS)
  const uint8_t* src[kMaxPieces];
  uint32_t off[kMaxPieces + 1];
  uint32_t len[kMaxPieces];
  uint8_t gen[kGenBytes];
};

__device__ __forceinline__ uint32_t lit_len(int i) { return kLits.len[i]; }
__device__ __forceinline__ const uint8_t* lit_src(int i) { return kLits.b + kLits.off[i]; }

// Piece q of record g: (source, length).  `nch` changes; str triple = ( '"', body, '"' )
// or ( -, "null", - ).
__device__ __forceinline__ void piece(const StorePipeArgs& a, int64_t g, uint32_t nch, uint32_t turn, const Group& G, int q,
                      const uint8_t*& src, uint32_t& len) {
  int lit = -1;
  int32_t sid = -2;  // pool id of a string triple's value (-1 null)
  int part = 0;      // 0 open quote, 1 body, 2 close quote
  const int tail = 5 + 18 * static_cast<int>(nch);
  if (q < 5) {
    switch (q) {
      case 0: lit = L_OPEN_AGENT; break;
      case 4: lit = L_CHANGES; break;
      default: sid = a.dagent_pool[g]; part = q - 1; break;
    }
  } else if (q < tail) {
    const int c = (q - 5) / 18;
    const int k = (q - 5) - 18 * c;
    const ChangeIds ch = a.changes[a.dch_off[g] + c];
    switch (k) {
      case 0: lit = c ? L_CH_SEP : -2; break;
      case 1: lit = L_CH_OPEN; break;
      case 5: lit = L_CH_OP; break;
      case 9: lit = L_CH_PATH; break;
      case 13: lit = L_CH_PREV; break;
      case 17: lit = L_CH_CLOSE; break;
      default: {
        const int f = (k - 2) / 4;  // 0 content_hash, 1 op, 2 path, 3 previous_hash
        part = (k - 2) - 4 * f;
        sid = f == 0 ? ch.content_hash : f == 1 ? ch.op : f == 2 ? ch.path : ch.previous_hash;
        break;
      }
    }
  } else {
    const uint32_t td = canon::dec_digits(turn);
    switch (q - tail) {
      case 0: lit = L_DELTA_ID; break;
      case 1: lit = L_DELTA_PFX; break;
      case 2: case 11: src = G.gen; len = td; return;
      case 3: lit = L_QUOTE; break;
      case 4: lit = L_PARENT; break;
      case 5: lit = turn > 1 ? L_HOLE : L_NULL; break;
      case 6: lit = L_SESSION; break;
      case 7: src = G.gen + 16; len = 46; return;
      case 8: lit = L_TS; break;
      case 9: src = G.gen + 64; len = G.off[kMaxPieces]; return;  // its length, stashed by the generator
      case 10: lit = L_TURN; break;
      case 12: lit = L_CLOSE; break;
      default: lit = -2; break;
    }
  }
  if (lit == -2) {  // an empty slot
    src = kLits.b;
    len = 0;
    return;
  }
  if (lit >= 0) {
    src = lit_src(lit);
    len = lit_len(lit);
    return;
  }
  if (sid < 0) {  // null: ( -, "null", - )
    src = part == 1 ? lit_src(L_NULL) : kLits.b;
    len = part == 1 ? 4u : 0u;
    return;
  }
  if (part == 1) {
    src = a.pool.bytes + a.pool.off[sid];
    len = static_cast<uint32_t>(a.pool.len[sid]);
  } else {
    src = lit_src(L_QUOTE);
    len = 1;
  }
}

// `t` ≤ 4 bytes at `p` (any alignment) as a little-endian word (bytes past `t` zero);
// reads only the aligned words that hold them.
__device__ __forceinline__ uint32_t read_bytes(const uint8_t* p, uint32_t t) {
  const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(ad & ~uintptr_t(3));
  const uint32_t sh = static_cast<uint32_t>(ad & 3u);
  const uint32_t lo = w[0];
  const uint32_t hi = sh + t > 4u ? w[1] : 0u;
  const uint32_t x = __builtin_amdgcn_alignbit(hi, lo, 8u * sh);
  return t >= 4u ? x : (x & ((1u << (8u * t)) - 1u));
}

}  // namespace coop

// G lanes per record (16, 8 or 4; AHV_SP_COOP_G), one wave per workgroup: the
// wave's 64 records take 64/G rounds of 64/G… records at a time.
template <int kGroup>
__global__ __launch_bounds__(64) void store_pipe_render_coop_kernel(StorePipeArgs a, const int32_t* dsess,
                                                                    int64_t nd) {
  using namespace coop;
  constexpr int kNG = 64 / kGroup;  // groups per wave
  __shared__ Group groups[kNG];
  const int lane = static_cast<int>(threadIdx.x);
  const int gl = lane & (kGroup - 1);  // lane within the group
  const int gq = lane / kGroup;        // group within the wave
  Group& G = groups[gq];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * 64;  // this wave's 64 records
  const Tables& t = a.t;
  for (int it = 0; it < 64 / kNG; ++it) {
    const int64_t x = base + kNG * it + gq;
    const bool live = x < nd;
    const int64_t g = live ? (a.render_order ? a.render_order[x] : x) : 0;
    const int64_t i = live ? dsess[g] : 0;
    bool on = live && a.status[i] != SP_ROW_IN_USE;
    const int32_t k = on ? static_cast<int32_t>(g - a.delta_off[i]) : 0;
    const uint32_t turn = static_cast<uint32_t>(k + 1);
    uint32_t nch = on ? static_cast<uint32_t>(a.dch_off[g + 1] - a.dch_off[g]) : 0u;
    if (on && nch > static_cast<uint32_t>(kCoopChanges)) {  // rare: the lane renderer's (wide_only pass)
      on = false;
      nch = 0;
    }
    const int np = 18 + 18 * static_cast<int>(nch);
    // generated text (three lanes of the group, in parallel)
    if (on && gl < 3) {
      GenSink gs{G.gen, 0};
      if (gl == 0) {
        emit_uint(gs, turn);
      } else if (gl == 1) {
        gs.n = 16;
        emit_session_uuid_quoted(gs, a.uuid + 4 * i);
      } else {
        gs.n = 64;
        emit_iso_quoted(gs, sp_delta_ts(a, i, k));
        G.off[kMaxPieces] = gs.n - 64;  // the timestamp's length (read by piece 9 of the tail)
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // layout: lane gl resolves pieces gl, gl+16, …; sums its own contiguous chunk after
    uint32_t mine = 0;
    if (on) {
      for (int q = gl; q < np; q += kGroup) {
        const uint8_t* sp;
        uint32_t ln;
        piece(a, g, nch, turn, G, q, sp, ln);
        G.src[q] = sp;
        G.len[q] = ln;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int per = (np + kGroup - 1) / kGroup;
    const int q0 = gl * per;
    const int q1 = q0 + per < np ? q0 + per : np;
    if (on)
      for (int q = q0; q < q1; ++q) mine += G.len[q];
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < kGroup; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, kGroup);
      if (gl >= o) incl += y;
    }
    const uint32_t L = __shfl(incl, kGroup - 1, kGroup);
    if (on) {
      uint32_t run = incl - mine;
      for (int q = q0; q < q1; ++q) {
        G.off[q] = run;
        run += G.len[q];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // assembly: output word w = gl + 16·j (64 contiguous bytes per group store)
    const int32_t d = on ? a.drow[g] : 0;
    const uint32_t cap = on ? static_cast<uint32_t>(a.dcap[g]) : 0u;
    const uint32_t lim = L < cap ? L : cap;  // an overflowing record keeps what fits (SP_RENDER)
    uint32_t* dst = reinterpret_cast<uint32_t*>(t.payload + (on ? a.doff[g] : 0));
    int p = 0;
    for (uint32_t w = static_cast<uint32_t>(gl); on && 4 * w < lim; w += kGroup) {
      uint32_t pos = 4 * w;
      const uint32_t end = pos + 4 < L ? pos + 4 : L;
      while (p < np - 1 && G.off[p] + G.len[p] <= pos) ++p;
      uint32_t out = 0;
      uint32_t sh = 0;
      while (pos < end) {
        const uint32_t in = pos - G.off[p];
        const uint32_t rem = G.len[p] - in;
        const uint32_t take = rem < end - pos ? rem : end - pos;
        out |= read_bytes(G.src[p] + in, take) << sh;
        sh += 8 * take;
        pos += take;
        if (pos < end) {
          ++p;
          while (p < np - 1 && G.len[p] == 0) ++p;
        }
      }
      if (4 * w + 4 <= cap) dst[w] = out;
    }
    if (on && gl == 0) {
      t.d_sess[d] = static_cast<int32_t>(a.slot[i]);
      t.d_turn[d] = static_cast<int32_t>(turn);
      t.d_prev[d] = k > 0 ? a.drow[g - 1] : -1;
      t.d_ts[d] = sp_delta_ts(a, i, k);
      t.d_off[d] = a.doff[g];
      t.d_len[d] = static_cast<int32_t>(L);
      t.d_hole[d] = turn > 1 ? static_cast<int32_t>(G.off[5 + 18 * static_cast<int>(nch) + 5]) : -1;
      if (L > cap) a.status[i] = SP_RENDER;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // the group's LDS layout is rewritten next iteration
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // (the parent-independent blocks: store_pipe_prefix_kernel, one record per lane)
}

template <class T>
T* P(const py::dict& d, const char* k) {
  return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}

StorePipeArgs to_args(const Tables& t, const py::dict& d) {
  StorePipeArgs a{};
  a.t = t;
  a.n = d["n"].cast<int64_t>();
  a.pool = StrPool{P<const uint8_t>(d, "pool_bytes"), P<const int64_t>(d, "pool_off"), P<const int32_t>(d, "pool_len")};
  a.slot = P<const int32_t>(d, "slot");
  a.uuid = P<const uint32_t>(d, "uuid");
  a.t0 = P<const int64_t>(d, "t0");
  a.creator = P<const int32_t>(d, "creator");
  a.maxpart = P<const int32_t>(d, "maxpart");
  a.minsig = P<const double>(d, "minsig");
  a.flags = P<const uint8_t>(d, "flags");
  a.join_off = P<const int32_t>(d, "join_off");
  a.join_agent = P<const int32_t>(d, "join_agent");
  a.join_sigma = P<const double>(d, "join_sigma");
  a.join_ring = P<uint8_t>(d, "join_ring");
  a.join_code = P<uint8_t>(d, "join_code");
  a.delta_off = P<const int32_t>(d, "delta_off");
  a.drow = P<const int32_t>(d, "drow");
  a.dagent_pool = P<const int32_t>(d, "dagent_pool");
  a.dch_off = P<const int32_t>(d, "dch_off");
  a.changes = P<const ChangeIds>(d, "changes");
  a.doff = P<const int64_t>(d, "doff");
  a.dcap = P<const int32_t>(d, "dcap");
  a.gslot = P<const int32_t>(d, "gslot");
  a.step_off = P<const int32_t>(d, "step_off");
  a.tslot = P<const int32_t>(d, "tslot");
  a.step_undo = P<const uint8_t>(d, "step_undo");
  a.step_retries = P<const int32_t>(d, "step_retries");
  a.step_fail = P<const uint8_t>(d, "step_fail");
  a.gc_retention_us = d["gc_retention_us"].cast<int64_t>();
  a.status = P<int32_t>(d, "status");
  a.chain_order = d.contains("chain_order") ? P<const int32_t>(d, "chain_order") : nullptr;
  a.mid = d.contains("mid") ? P<uint32_t>(d, "mid") : nullptr;
  a.mid_blocks = d.contains("mid_blocks") ? P<int32_t>(d, "mid_blocks") : nullptr;
  a.prefix_in_render = d.contains("prefix_in_render") ? d["prefix_in_render"].cast<int32_t>() : 1;
  a.render_order = d.contains("render_order") ? P<const int32_t>(d, "render_order") : nullptr;
  a.prefix_order = d.contains("prefix_order") ? P<const int32_t>(d, "prefix_order") : nullptr;
  a.max_nch = d.contains("max_nch") ? d["max_nch"].cast<int32_t>() : 1 << 30;
  a.wide_only = 0;
  // only with the prefix pass of its own and the lane renderer (the layout it reorders)
  a.render_first = d.contains("render_first") && a.mid != nullptr && !a.prefix_in_render
                       ? d["render_first"].cast<int32_t>()
                       : 0;
  a.chain_roots = d.contains("chain_roots") && d["chain_roots"].cast<int32_t>() != 0 && a.mid != nullptr;
  if (d.contains("dfrag")) {
    a.dfrag = P<const int32_t>(d, "dfrag");
    a.frag_bytes = P<const uint8_t>(d, "frag_bytes");
    a.frag_off = P<const int64_t>(d, "frag_off");
    a.frag_len = P<const int32_t>(d, "frag_len");
  }
  return a;
}

// AHV_SP_RENDER=coop: the wave-cooperative renderer with AHV_SP_COOP_G lanes per
// record (16, 8 or 4); default: the lane-per-record renderer (0).
static int render_coop() {
  static const int v = [] {
    const char* e = std::getenv("AHV_SP_RENDER");
    if (e == nullptr || std::string(e) != "coop") return 0;
    const char* g = std::getenv("AHV_SP_COOP_G");
    const int n = g ? std::atoi(g) : 16;
    return n == 8 || n == 4 ? n : 16;
  }();
  return v;
}

// AHV_SP_SINK=staged: the lane renderer's branching arena sink (A/B); default flat.
static bool sink_flat() {
  static const bool v = [] {
    const char* e = std::getenv("AHV_SP_SINK");
    return e == nullptr || std::string(e) != "staged";
  }();
  return v;
}

using RenderFn = void (*)(StorePipeArgs, const int32_t*, int64_t);

// (Register budgets for 5 / 6 waves per SIMD, __launch_bounds__(256, W), spill the
// render lane to scratch and ran slower: 1.99 / 2.03 vs 1.93 ms per 1 M-session step;
// the chain kernel held to 4 / 5 waves: 1.95 / 1.99 ms — profiles/r6/hetero_sink_waves_ab_r6ah.txt.)
// AHV_SP_HOIST=0: the render lanes' loads in line (A/B).  (Also loading each string's first
// 16-byte chunk ahead measured no better: profiles/r6/hetero_hoist_levels_ab_r6ay.txt.)
static bool hoist() {
  static const bool v = [] {
    const char* e = std::getenv("AHV_SP_HOIST");
    return e == nullptr || std::string(e) != "0";
  }();
  return v;
}

static RenderFn render_fn() {
  if (!sink_flat()) return static_cast<RenderFn>(store_pipe_render_kernel<false, false>);
  return hoist() ? static_cast<RenderFn>(store_pipe_render_kernel<true, true>)
                 : static_cast<RenderFn>(store_pipe_render_kernel<true, false>);
}

static RenderFn prefix_fn() {
  static const RenderFn f = [] {
    const char* e = std::getenv("AHV_SP_PREFIX_PIPE");
    return (e != nullptr && std::string(e) == "0") ? static_cast<RenderFn>(store_pipe_prefix_kernel<false>)
                                                   : static_cast<RenderFn>(store_pipe_prefix_kernel<true>);
  }();
  return f;
}

using ChainFn = void (*)(StorePipeArgs);

// AHV_SP_CHAIN_PIPE=0: the chain lanes load each block, then compress it (A/B)
static ChainFn chain_fn() {
  static const ChainFn f = [] {
    const char* e = std::getenv("AHV_SP_CHAIN_PIPE");
    return (e != nullptr && std::string(e) == "0") ? static_cast<ChainFn>(store_pipe_chain_kernel<false>)
                                                   : static_cast<ChainFn>(store_pipe_chain_kernel<true>);
  }();
  return f;
}

using RowsFn = void (*)(StorePipeArgs, const int32_t*, int64_t, uint32_t, uint32_t);

static RowsFn render_rows_fn() {
  return hoist() ? static_cast<RowsFn>(store_pipe_render_rows_kernel<true>)
                 : static_cast<RowsFn>(store_pipe_render_rows_kernel<false>);
}

}  // namespace

// Launch the kernels (rows, render, prefix, chain) on `stream` (device) or run the twin (host tables).
void store_pipeline_run(const Tables& t, bool gpu, const py::dict& d, uintptr_t stream) {
  StorePipeArgs a = to_args(t, d);
  const int32_t* dsess = P<const int32_t>(d, "dsess");
  const int64_t nd = d["nd"].cast<int64_t>();
  if (gpu && render_coop()) a.render_first = 0;
  if (!gpu && a.render_first) {  // the device's order: render (own row check), rows, prefix, chain
    for (int64_t g = 0; g < nd; ++g) {
      const int64_t i = dsess[g];
      if (sp_row_in_use(a, i)) a.status[i] = SP_ROW_IN_USE;
      else sp_render(a, i, static_cast<int32_t>(g));
    }
    for (int64_t i = 0; i < a.n; ++i) sp_rows(a, i);
    for (int64_t g = 0; g < nd; ++g) {
      if (a.status[dsess[g]] != SP_ROW_IN_USE) sp_prefix(a, g);
      else a.mid_blocks[g] = 0;
    }
    for (int64_t i = 0; i < a.n; ++i)
      if (a.status[i] != SP_ROW_IN_USE) {
        sp_chain(a, i);
        if (a.chain_roots) sp_chain_root(a, i);
      }
    return;
  }
  if (!gpu) {
    for (int64_t i = 0; i < a.n; ++i) sp_rows(a, i);
    for (int64_t g = 0; g < nd; ++g)
      if (a.status[dsess[g]] != SP_ROW_IN_USE) sp_render(a, dsess[g], static_cast<int32_t>(g));
    if (a.mid && !a.prefix_in_render)
      for (int64_t g = 0; g < nd; ++g) {
        if (a.status[dsess[g]] != SP_ROW_IN_USE) sp_prefix(a, g);
        else a.mid_blocks[g] = 0;
      }
    for (int64_t i = 0; i < a.n; ++i)
      if (a.status[i] != SP_ROW_IN_USE) {
        sp_chain(a, i);
        if (a.chain_roots) sp_chain_root(a, i);
      }
    return;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  py::gil_scoped_release nogil;
  if (a.n > 0 && a.render_first == 2) {
    const unsigned rb = static_cast<unsigned>((a.n + 255) / 256), pb = static_cast<unsigned>((nd + 255) / 256);
    hipLaunchKernelGGL(render_rows_fn(), dim3(rb + pb), dim3(256), 0, st, a, dsess, nd, rb, rb + pb);
    if (nd > 0) hipLaunchKernelGGL(prefix_fn(), dim3(pb), dim3(256), 0, st, a, dsess, nd);
    hipLaunchKernelGGL(chain_fn(), dim3(static_cast<unsigned>((a.n + 63) / 64)), dim3(64), 0, st, a);
  } else if (a.n > 0 && a.render_first) {
    const unsigned rb = static_cast<unsigned>((a.n + 255) / 256), pb = static_cast<unsigned>((nd + 255) / 256);
    if (nd > 0)
      hipLaunchKernelGGL(render_fn(), dim3(pb), dim3(256), 0, st, a, dsess, nd);
    hipLaunchKernelGGL(store_pipe_prefix_rows_kernel, dim3(rb + pb), dim3(256), 0, st, a, dsess, nd, rb, rb + pb);
    hipLaunchKernelGGL(chain_fn(), dim3(static_cast<unsigned>((a.n + 63) / 64)), dim3(64), 0, st, a);
  } else if (a.n > 0) {
    hipLaunchKernelGGL(store_pipe_rows_kernel, dim3(static_cast<unsigned>((a.n + 255) / 256)), dim3(256), 0, st, a);
    if (nd > 0) {
      const int cg = render_coop();
      const dim3 cgrid(static_cast<unsigned>((nd + 63) / 64));
      if (cg == 16)
        hipLaunchKernelGGL(store_pipe_render_coop_kernel<16>, cgrid, dim3(64), 0, st, a, dsess, nd);
      else if (cg == 8)
        hipLaunchKernelGGL(store_pipe_render_coop_kernel<8>, cgrid, dim3(64), 0, st, a, dsess, nd);
      else if (cg == 4)
        hipLaunchKernelGGL(store_pipe_render_coop_kernel<4>, cgrid, dim3(64), 0, st, a, dsess, nd);
      if (cg && a.max_nch > coop::kCoopChanges) {  // records past the cooperative layout: one lane each
        StorePipeArgs w = a;
        w.wide_only = 1;
        w.prefix_in_render = 0;
        hipLaunchKernelGGL(render_fn(), dim3(static_cast<unsigned>((nd + 255) / 256)), dim3(256), 0, st,
                           w, dsess, nd);
      }
      if (!cg)
        hipLaunchKernelGGL(render_fn(), dim3(static_cast<unsigned>((nd + 255) / 256)), dim3(256), 0, st,
                           a, dsess, nd);
      if (a.mid && (cg || !a.prefix_in_render))
        hipLaunchKernelGGL(prefix_fn(), dim3(static_cast<unsigned>((nd + 255) / 256)), dim3(256), 0, st,
                           a, dsess, nd);
    }
    hipLaunchKernelGGL(chain_fn(), dim3(static_cast<unsigned>((a.n + 63) / 64)), dim3(64), 0, st, a);
  }
  check_hip(hipGetLastError(), "store_pipeline");
}

}  // namespace ahv
