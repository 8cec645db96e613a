// Device-authoritative governance state store and its command
// processor, written once for the gfx950 worker and the CPU twin.
//
// The public `Hypervisor` API (reference core.py:69-227, liability/vouching.py:
// 61-184, liability/slashing.py:63-143, audit/delta.py:85-152, saga/
// state_machine.py + orchestrator.py) runs as a stream of small commands against
// SoA tables resident in HBM:
//
//   sessions   lifecycle state, config, participant rows (ring, σ_raw, σ_eff),
//              audit chain head, Merkle root, commitment, GC/bond counters
//   deltas     arena of audit deltas (session, turn, parent link, timestamp,
//              SHA-256 digest, canonical-JSON payload bytes = the on-disk record)
//   vouches    bond edges in creation order, linked per liability session
//   sagas/steps  saga and step FSM rows (K13), timestamps, retry counters
//
// A command is one 512-byte slot (64 little-endian u64 words) in a ring the
// host writes through the PCIe BAR (fine-grained device memory); a resident
// single-wave worker (csrc/hip/store_worker.hip) polls the ring, executes the
// command with `store_exec` and writes a 512-byte result slot into pinned host
// memory.  The host twin (csrc/host/py_store.cpp, device='cpu') calls
// `store_exec` directly on host-memory tables, so one body defines the
// semantics for both.  Strings never reach the device: DIDs and session ids are
// interned ids, error texts are formatted on the host from returned codes.
//
// Slot layout:  w[0] seq (written last), w[1] op | words-in-use << 32, w[2]
// checksum (xor of w[1], w[3..63]), w[3..15] = a[0..12] scalar args, w[16..63] =
// 384 inline payload bytes (index lists, score pairs).  Only the words in use are
// written; the worker reads the others as zero.  Larger variable data lives in the staging
// area (fine-grained device memory), addressed by (offset, length) args.
#pragma once

#include "ahv/hd.h"
#include "ahv/semantics.h"
#include "ahv/sha256.h"

namespace ahv {
namespace store {

constexpr int kSlotWords = 64;

// Command-slot checksum term of word k (w[2] = XOR of slot_mix(w[k], k) over k = 1
// and k ≥ 3).  Write-combined 32-byte chunks of a slot can reach the device in any
// order, so the worker may read a slot half new, half from its previous occupant;
// the checksum rejects that read.  A plain XOR of the words did not: two captures
// differ in their record length and parent-hole offset by the same amount (the
// suffix after the hole has a fixed length), and those two word changes cancelled
// in the XOR about once per few thousand torn reads — the worker then hashed a
// record with another capture's length and hole.  Each word is multiplied by its
// own odd constant first, so correlated changes of different words do not cancel.
AHV_HD uint64_t slot_mix(uint64_t w, uint64_t k) { return w * (0x9E3779B97F4A7C15ull + 2ull * k); }
constexpr int kArgs = 13;
constexpr int kInlineWords = 48;  // w[16..63]
constexpr int kResWords = 64;     // result slot: r[0] seq, r[1] status, r[2..63] values

enum Op : uint32_t {
  OP_NOP = 0,
  OP_STOP = 1,
  OP_FLUSH = 2,    // release: make table writes visible to other agents (torch, kernels)
  OP_ACQUIRE = 3,  // acquire: see rows other kernels wrote (batched pipeline)
  OP_FREE_ROWS = 4,  // return rows to the free state (host allocator reclaim; drains the hash engine)

  OP_SESS_CREATE = 10,
  OP_SESS_JOIN = 11,
  OP_SESS_LEAVE = 12,
  OP_SESS_ACTIVATE = 13,
  OP_SESS_TERMINATE = 14,
  OP_SESS_ARCHIVE = 15,
  OP_SESS_UPDATE_RING = 16,
  OP_SESS_SET_MODE = 17,
  OP_SESS_READ = 18,
  OP_SESS_SET_SIGMA = 19,
  OP_SESS_CLOSE = 20,  // Hypervisor.terminate_session: terminate+root+commit+release+GC+archive
  OP_SESS_HANDSHAKE = 21,
  OP_SESS_READ_MANY = 22,  // headers (+ participant rows) of many sessions in one command

  OP_DELTA_CAPTURE = 30,
  OP_DELTA_MERKLE = 31,
  OP_DELTA_VERIFY = 32,
  OP_DELTA_READ = 33,

  OP_VOUCH = 40,
  OP_SIGMA_EFF = 41,
  OP_EXPOSURE = 42,
  OP_RELEASE_BOND = 43,
  OP_RELEASE_SESSION = 44,
  OP_VOUCH_LIST = 45,
  OP_EDGE_READ = 46,
  OP_SLASH = 47,
  OP_V_RETIRE = 48,  // unlink a liability session's edge list and free its rows (after close)

  OP_SAGA_CREATE = 60,
  OP_STEP_ADD = 61,
  OP_STEP_TRANSITION = 62,
  OP_STEP_SET = 63,
  OP_SAGA_TRANSITION = 64,
  OP_SAGA_READ = 65,
  OP_SAGA_PLAN = 66,
  OP_STEP_READ = 67,
};

// Status codes in r[1] (0 = ok).  Op-specific codes are small positive ints.
enum Status : uint64_t {
  ST_OK = 0,
  ST_BAD_STATE = 1,
  ST_NOT_FOUND = 2,
  ST_BAD_ARG = 90,
  ST_SCRATCH = 91,   // scratch too small for this request
  ST_BAD_OP = 99,
};

// Vouch rejection codes (VouchingEngine.vouch check order).
enum VouchCode : uint64_t { V_OK = 0, V_SELF = 1, V_LOW_SIGMA = 2, V_CYCLE = 3, V_EXPOSURE = 4, V_FULL = 5 };

// Join codes extend semantics.h JoinCode.
constexpr uint64_t JOIN_ROWS = 5;  // participant row table exhausted
constexpr uint64_t JOIN_NOT_MINE = 6;  // the row holds another session (creation stamp differs)
constexpr uint64_t ACT_NOT_MINE = 4;   // activate: the row holds another session

// Row lifecycle.  A row is FREE until a create command claims it and FREE again
// after the host allocator reclaims it (OP_FREE_ROWS); creates refuse a row that
// is not free (ST_BAD_STATE), so an allocator bug can never overwrite live state.
// Markers: s_state / g_state / t_state = kFree8, d_sess / e_vsess = -1.
constexpr uint8_t kFree8 = 255;
enum RowKind : uint64_t { RK_S = 0, RK_G = 1, RK_T = 2, RK_E = 3, RK_D = 4, RK_V = 5 };

// --------------------------------------------------------------- tables

// X-macro: (name, element type, extent) where extent names a capacity:
// S sessions, SP participant rows (participant-major: row k·S + s, see prow),
// S8/S4 session×digest/uuid words,
// D deltas, D8 delta×digest words, E vouch edges, V liability sessions,
// G sagas, T steps, SCR scratch bytes (cap X).
#define AHV_STORE_COLUMNS(X)       \
  X(s_state, uint8_t, S)           \
  X(s_mode, uint8_t, S)            \
  X(s_audit, uint8_t, S)           \
  X(s_maxpart, int32_t, S)         \
  X(s_minsig, double, S)           \
  X(s_creator, int32_t, S)         \
  X(s_created, int64_t, S)         \
  X(s_terminated, int64_t, S)      \
  X(s_pcount, int32_t, S)          \
  X(s_pactive, int32_t, S)         \
  X(s_dcount, int32_t, S)          \
  X(s_dlast, int32_t, S)           \
  X(s_committed, int64_t, S)       \
  X(s_commit_n, int32_t, S)        \
  X(s_released, int32_t, S)        \
  X(s_retained, int32_t, S)        \
  X(s_uuid, uint32_t, S4)          \
  X(s_head, uint32_t, S8)          \
  X(s_root, uint32_t, S8)          \
  X(s_proot, uint32_t, S8)         \
  X(s_proot_n, int32_t, S)         \
  X(s_proot_last, int32_t, S)      \
  X(p_agent, int32_t, SP)          \
  X(p_ring, uint8_t, SP)           \
  X(p_active, uint8_t, SP)         \
  X(p_sraw, double, SP)            \
  X(p_seff, double, SP)            \
  X(p_joined, int64_t, SP)         \
  X(d_sess, int32_t, D)            \
  X(d_turn, int32_t, D)            \
  X(d_prev, int32_t, D)            \
  X(d_ts, int64_t, D)              \
  X(d_off, int64_t, D)             \
  X(d_len, int32_t, D)             \
  X(d_hole, int32_t, D)            \
  X(d_hash, uint32_t, D8)          \
  X(e_voucher, int32_t, E)         \
  X(e_vouchee, int32_t, E)         \
  X(e_vsess, int32_t, E)           \
  X(e_next, int32_t, E)            \
  X(e_active, uint8_t, E)          \
  X(e_bonded, double, E)           \
  X(e_pct, double, E)              \
  X(e_expiry, int64_t, E)          \
  X(e_released, int64_t, E)        \
  X(e_created, int64_t, E)         \
  X(v_head, int32_t, V)            \
  X(v_tail, int32_t, V)            \
  X(g_state, uint8_t, G)           \
  X(g_created, int64_t, G)         \
  X(g_completed, int64_t, G)       \
  X(g_nsteps, int32_t, G)          \
  X(t_saga, int32_t, T)            \
  X(t_state, uint8_t, T)           \
  X(t_undo, uint8_t, T)            \
  X(t_started, int64_t, T)         \
  X(t_completed, int64_t, T)       \
  X(t_retry, int32_t, T)           \
  X(t_maxretry, int32_t, T)        \
  X(scratch, uint8_t, SCR)

struct Caps {
  int64_t S, P, D, E, V, G, T, X, B;  // B = payload arena bytes
};

struct Tables {
#define AHV_DECL(name, type, ext) type* name;
  AHV_STORE_COLUMNS(AHV_DECL)
#undef AHV_DECL
  uint8_t* payload;  // [B] canonical-JSON audit records (fine-grained device memory)
  const uint8_t* staging;  // host-written variable-length inputs
  Caps cap;
};

// ------------------------------------------------------ execution context

// SIMT context: the worker runs one wave (lane 0..63); the host twin is one lane.
// `lds` is a word buffer in LDS on the device (a thread-local array on the host)
// used to stage audit payloads as big-endian SHA message words.
constexpr int kLdsWords = 4096;  // 16 KiB: payloads up to 16 KiB − 72 B hash from LDS
constexpr int kKwStride = 65;    // words per schedule row: odd stride, the 64 lanes' rows hit distinct banks

struct Lanes {
  int lane;
  int n;
  uint32_t* lds;
  uint32_t* kw = nullptr;  // [n][kKwStride] per-lane K+W schedule rows (hash-engine wave), or null
  // worker command wave: session + 1 whose provisional Merkle root the hash-engine
  // wave is computing (LDS, 0 = none); a close / Merkle command waits on it only
  // right before it reads that root (null: host twin, nothing to wait for)
  const uint32_t* tree_busy = nullptr;
  AHV_HD bool leader() const { return lane == 0; }
  AHV_HD void wait_tree(int64_t s) const {
#if defined(__HIP_DEVICE_COMPILE__)
    if (tree_busy == nullptr) return;
    const uint32_t want = static_cast<uint32_t>(s) + 1u;
    while (__hip_atomic_load(tree_busy, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == want)
      __builtin_amdgcn_s_sleep(1);
#else
    (void)s;
#endif
  }
  // Lanes of ONE wave exchange data through LDS / global memory: a wave-level
  // barrier with wavefront-scope fences (the worker runs two waves with
  // different roles, so a workgroup barrier here would deadlock).
  AHV_HD void sync() const {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
  }
};

// A capture whose digest is computed by the hash-engine wave (worker) or right
// away (host twin): everything but the SHA-256 is recorded by the command wave.
struct HashJob {
  uint64_t seq;
  int64_t s, d, off, len, hole;
  int64_t prev;        // parent delta index (-1 for turn 1)
  int32_t mid_blocks;  // leading blocks already compressed into `mid` (0: none)
  uint32_t mid[8];     // SHA-256 state after those blocks (they precede the parent hole)
  // Speculated chain link (worker): the host wrote its predicted parent digest into
  // the hole (`spec`), so a helper wave may hash the whole record before the parent
  // is final (`full`: `sdig` is the digest of the record as stored, `ppar` the
  // parent digest its hole holds).  The hash engine takes `sdig` only when `ppar`
  // equals the parent digest it computed; otherwise it splices and re-hashes.
  int32_t spec;
  int32_t full;
  uint32_t sdig[8];
  uint32_t ppar[8];
};

enum ExecResult : int { EXEC_STOP = 0, EXEC_DONE = 1, EXEC_DEFERRED = 2 };

// Commands that read or reset state the hash engine may still be writing
// (delta digests, chain heads) or that publish table state wholesale; the
// command wave drains the hash queue before executing them.
AHV_HD bool needs_drain(uint32_t op);
// Commands that read the audit state of ONE session (a0): the command wave waits
// only until no queued capture of that session is pending — captures of other
// sessions keep hashing alongside (many pipelines in flight never serialise on
// the engine).
AHV_HD bool session_drain(uint32_t op);

// Result / bulk-output stores.  On the device these land in pinned host memory,
// so they are system-scope stores (vector stores that bypass the caches).
AHV_HD void out64(uint64_t* p, uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  *p = v;
#endif
}

// Loads of host-written fine-grained memory (payload arena, staging area): the
// host writes these bytes through the BAR between commands, so the device must
// not serve them from a cache line it filled earlier — system-scope loads bypass
// L1/L2 (one round trip to HBM each; they are issued in parallel).
AHV_HD uint32_t ld32f(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __hip_atomic_load(static_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  return *static_cast<const uint32_t*>(p);
#endif
}
AHV_HD uint64_t ld64f(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __hip_atomic_load(static_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
  return *static_cast<const uint64_t*>(p);
#endif
}

AHV_HD uint64_t dbits(double d) {
  union { double d; uint64_t u; } x;
  x.d = d;
  return x.u;
}
AHV_HD double bitsd(uint64_t u) {
  union { double d; uint64_t u; } x;
  x.u = u;
  return x.d;
}

struct Cmd {
  uint32_t op;
  uint64_t a[kArgs];
  const uint64_t* inl;  // inline payload words (kInlineWords)
};

// Broadcast a value from lane 0 (device: readfirstlane-style shuffle).
template <class T>
AHV_HD T bcast(const Lanes& L, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    u = __shfl(u, 0);
    T r;
    __builtin_memcpy(&r, &u, 8);
    return r;
  } else {
    return static_cast<T>(__shfl(static_cast<int>(v), 0));
  }
#else
  (void)L;
  return v;
#endif
}

// ------------------------------------------------------------- helpers

AHV_HD void load8(const uint32_t* src, uint32_t d[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = src[k];
}
AHV_HD void store8(uint32_t* dst, const uint32_t d[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) dst[k] = d[k];
}

// SHA-256 of `n` bytes at `p` (any alignment) on one lane; big-endian word
// assembly four bytes at a time.
AHV_HD void sha256_mem(const uint8_t* p, uint64_t n, uint32_t out[8]) {
  sha256_init(out);
  uint32_t blk[16];
  uint64_t i = 0;
  while (n - i >= 64) {
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const uint8_t* q = p + i + 4 * w;
      blk[w] = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | uint32_t(q[3]);
    }
    sha256_compress(out, blk);
    i += 64;
  }
  // tail + padding (one or two blocks)
  uint8_t tail[128];
  const uint64_t r = n - i;
  for (uint64_t k = 0; k < r; ++k) tail[k] = p[i + k];
  tail[r] = 0x80;
  const uint64_t padded = (r + 9 <= 64) ? 64 : 128;
  for (uint64_t k = r + 1; k < padded; ++k) tail[k] = 0;
  const uint64_t bits = n * 8;
  for (int k = 0; k < 8; ++k) tail[padded - 1 - k] = static_cast<uint8_t>(bits >> (8 * k));
  for (uint64_t b = 0; b < padded; b += 64) {
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      const uint8_t* q = tail + b + 4 * w;
      blk[w] = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | uint32_t(q[3]);
    }
    sha256_compress(out, blk);
  }
}

// SHA-256 of `n` bytes of fine-grained memory at 4-byte-aligned `p`.
AHV_HD void sha256_fine(const uint8_t* p, uint64_t n, uint32_t out[8]) {
  sha256_init(out);
  uint32_t blk[16];
  const uint64_t nblk = (n + 9 + 63) / 64;
  for (uint64_t b = 0; b < nblk; ++b) {
    for (int w = 0; w < 16; ++w) {
      const uint64_t o = 64 * b + 4 * w;
      uint32_t x = 0;
      if (o + 4 <= n) {
        x = bswap32(ld32f(p + o));
      } else if (o < n) {
        x = bswap32(ld32f(p + o)) & (0xffffffffu << (8 * (4 - (n - o))));
      }
      if (o <= n && n < o + 4) x |= 0x80u << (8 * (3 - (n - o)));
      if (b == nblk - 1 && w == 14) x |= static_cast<uint32_t>((n * 8) >> 32);
      if (b == nblk - 1 && w == 15) x |= static_cast<uint32_t>(n * 8);
      blk[w] = x;
    }
    sha256_compress(out, blk);
  }
}

AHV_HD void hex_digest(const uint32_t d[8], uint8_t out[64]) {
  for (int i = 0; i < 8; ++i) {
    for (int j = 0; j < 8; ++j) {
      const uint32_t nib = (d[i] >> (28 - 4 * j)) & 15u;
      out[8 * i + j] = static_cast<uint8_t>(hex_nibble(nib));
    }
  }
}

// Live vouch: active and not expired at `now` (VouchRecord.is_live, reference
// vouching.py:34-38 + the `_active_vouches_for` filter).
AHV_HD bool edge_live(const Tables& t, int32_t e, int64_t now) {
  return t.e_active[e] && (t.e_expiry[e] < 0 || now <= t.e_expiry[e]);
}

// p_active bits: P_ACTIVE — the participant is in the session now (SSO leave
// clears it); P_COMMITTED — it was active when the session's Merkle root was
// committed (the commitment record's participant_dids, reference core.py:209-214:
// the list is taken at terminate, so a later leave must not change it).
constexpr uint8_t P_ACTIVE = 1u;
constexpr uint8_t P_COMMITTED = 2u;

// Participant row k of session s.  The participant columns are participant-major
// ([k][session]): the k-th rows of consecutive sessions are adjacent, so the
// batched pipelines' first-participant writes from 64 lanes are contiguous.
AHV_HD int64_t prow(const Tables& t, int64_t s, int64_t k) { return k * t.cap.S + s; }

AHV_HD void mark_committed_participants(const Tables& t, int64_t s) {
  const int32_t n = t.s_pcount[s];
  for (int32_t k = 0; k < n; ++k) {
    const int64_t row = prow(t, s, k);
    if (t.p_active[row] & P_ACTIVE) t.p_active[row] = P_ACTIVE | P_COMMITTED;
  }
}

// Participant row of `agent` in session `s` (all rows, active or not), or -1.
// Creation stamp of row s: the low 64 bits of the id words its create wrote (a
// uuid4's low half always has the variant bits set, so it is never 0).
AHV_HD uint64_t row_stamp(const Tables& t, int64_t s) {
  return (static_cast<uint64_t>(t.s_uuid[4 * s + 2]) << 32) | t.s_uuid[4 * s + 3];
}

AHV_HD int32_t find_part(const Tables& t, int64_t s, int32_t agent) {
  const int32_t n = t.s_pcount[s];
  for (int32_t k = 0; k < n; ++k)
    if (t.p_agent[prow(t, s, k)] == agent) return k;
  return -1;
}

// An int32 index list argument: ≤ 96 entries inline in the command, else in
// the staging area at `off`.
struct IndexList {
  const int32_t* p;
  bool fine;
  AHV_HD int32_t operator[](uint64_t i) const {
    return fine ? static_cast<int32_t>(ld32f(p + i)) : p[i];
  }
};

AHV_HD IndexList index_list(const Tables& t, const Cmd& c, uint64_t n, uint64_t off) {
  if (n <= 2 * kInlineWords) return IndexList{reinterpret_cast<const int32_t*>(c.inl), false};
  return IndexList{reinterpret_cast<const int32_t*>(t.staging + off), true};
}

// Merkle root (reference audit/delta.py:117-134) over `n` digests in `lv`
// (scratch, n*8 words), level by level with odd duplication; SIMT across the
// lanes within a level (the worker is a single wave, so a barrier inside the
// lane-strided loop is wave-uniform).  Parent i overwrites slot i: within a
// pass every lane reads its two children before any lane writes, and the slots
// a pass writes ([p·n, (p+1)·n)) lie below every child slot of later passes.
// The root is left in lv[0..7].
AHV_HD void merkle_inplace(const Lanes& L, uint32_t* lv, int64_t n) {
  while (n > 1) {
    const int64_t m = (n + 1) / 2;
    for (int64_t i0 = 0; i0 < m; i0 += L.n) {
      const int64_t i = i0 + L.lane;
      uint32_t o[8];
      if (i < m) {
        uint32_t l[8], r[8];
        load8(lv + 16 * i, l);
        if (2 * i + 1 < n) load8(lv + 16 * i + 8, r);
        else load8(lv + 16 * i, r);
        merkle_node(l, r, o);
      }
      L.sync();
      if (i < m) store8(lv + 8 * i, o);
      L.sync();
    }
    n = m;
  }
}

// Stage `n` payload bytes at `src` (64-byte aligned) into `w` as big-endian
// SHA-256 message words and append the SHA padding.  Returns the number of
// 64-byte blocks, or -1 when the message needs more than `cap` words.  All
// lanes participate (lane-strided loads of the host-written arena).
AHV_HD int64_t stage_words(const Lanes& L, const uint8_t* src, uint64_t n, uint32_t* w, int64_t cap) {
  const uint64_t nblk = (n + 9 + 63) / 64;
  if (static_cast<int64_t>(nblk * 16) > cap) return -1;
  const uint64_t nw = nblk * 16;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src);
  for (uint64_t i = L.lane; i < nw; i += L.n) {
    uint32_t x = 0;
    const uint64_t b = 4 * i;
    if (b + 4 <= n) {
      x = bswap32(ld32f(s32 + i));
    } else if (b < n) {
      const uint32_t raw = bswap32(ld32f(s32 + i));
      const uint32_t keep = static_cast<uint32_t>(n - b);  // 1..3 leading bytes
      x = raw & (0xffffffffu << (8 * (4 - keep)));
    }
    if (b <= n && n < b + 4) x |= 0x80u << (8 * (3 - (n - b)));  // padding marker
    if (i == nw - 2) x |= static_cast<uint32_t>((n * 8) >> 32);
    if (i == nw - 1) x |= static_cast<uint32_t>(n * 8);
    w[i] = x;
  }
  L.sync();
  return static_cast<int64_t>(nblk);
}

// Splice the quoted hex of `head` ('"', 64 lowercase hex digits, '"' = 66
// bytes) into the staged words `w` at byte `hole`, and into the arena record
// `src` so the stored record is complete.  All lanes participate.
AHV_HD void splice_parent(const Lanes& L, uint8_t* src, uint32_t* w, int64_t hole, const uint32_t* head) {
  for (int k = L.lane; k < 66; k += L.n) {
    uint32_t ch;
    if (k == 0 || k == 65) {
      ch = 0x22u;
    } else {
      const int nib = k - 1;
      ch = hex_nibble((head[nib >> 3] >> (28 - 4 * (nib & 7))) & 15u);
    }
    const uint64_t b = static_cast<uint64_t>(hole) + k;
    src[b] = static_cast<uint8_t>(ch);
    if (w) reinterpret_cast<uint8_t*>(w)[(b & ~uint64_t(3)) | (3 - (b & 3))] = static_cast<uint8_t>(ch);
  }
  L.sync();
}

// stage_words + splice_parent into L.lds (the whole window).  A record larger
// than the window (-1) is hashed from the arena, so the parent is spliced there
// only — before the caller's sha256_fine reads it.
AHV_HD int64_t stage_message(const Lanes& L, uint8_t* src, uint64_t n, int64_t hole, const uint32_t* head) {
  const int64_t nblk = stage_words(L, src, n, L.lds, kLdsWords);
  if (hole >= 0) splice_parent(L, src, nblk >= 0 ? L.lds : nullptr, hole, head);
  return nblk;
}

AHV_HD void sha256_lds_blocks(const uint32_t* w, int64_t nblk, uint32_t out[8]) {
  sha256_init(out);
  for (int64_t b = 0; b < nblk; ++b) sha256_compress(out, w + 16 * b);
}

// Message schedule of one block with the round constants folded in: kw[t] =
// K[t] + W[t] for t < 64 (the half of a compression that does not depend on the
// chaining state).
AHV_HD void sha256_expand_kw(const uint32_t* blk, uint32_t* kw) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    w[i] = blk[i];
    kw[i] = w[i] + sha256_k(i);
  }
#pragma unroll
  for (int i = 16; i < 64; ++i) {
    const uint32_t x = w[(i + 1) & 15];
    const uint32_t y = w[(i + 14) & 15];
    const uint32_t s0 = xor3(rotr32(x, 7), rotr32(x, 18), x >> 3);
    const uint32_t s1 = xor3(rotr32(y, 17), rotr32(y, 19), y >> 10);
    const uint32_t wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
    w[i & 15] = wi;
    kw[i] = wi + sha256_k(i);
  }
}

// 3-input add: one v_add3_u32.  LLVM forms it in sha256_compress but not in
// the K+W round loop below (~2.5 extra VALU per round on the single-lane,
// issue-bound serial path), so it is spelled out there.
AHV_HD uint32_t add3u(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return a + b + c;
#endif
}

// The 64 rounds of a compression over a precomputed K+W row.  h + kw[i] does
// not depend on the previous round (h is e from three rounds back), so the
// round's critical path is Σ1 → add3 → add.
AHV_HD void sha256_rounds_kw(uint32_t st[8], const uint32_t* kw) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
  // K+W words are read 8 rounds ahead through a small register ring: the LDS
  // latency hides behind the rounds without holding all 64 words live (the
  // worker kernel sits at the VGPR limit, where the compiler otherwise waits on
  // every read).
  uint32_t q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = kw[i];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint32_t kwi = q[i & 7];
    if (i + 8 < 64) q[i & 7] = kw[i + 8];
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t t1 = add3u(h + kwi, S1, sha_ch(e, f, g));
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t na = add3u(t1, S0, sha_maj(a, b, c));
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = na;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256 of `nblk` staged blocks by one wave: the lanes expand up to L.n block
// schedules at once (one block per lane, SIMT), then the leader runs only the
// rounds — the serial part shrinks by the schedule's third.  Without schedule
// rows (host twin) the plain serial form.  The digest is valid on the leader.
// With `from` the compression resumes from that state (blocks `w` follow it).
AHV_HD void sha256_lds_blocks_par(const Lanes& L, const uint32_t* w, int64_t nblk, uint32_t out[8],
                                  const uint32_t* from = nullptr) {
  if (L.kw == nullptr || L.n < 2) {
    if (L.leader()) {
      if (from) {
        for (int k = 0; k < 8; ++k) out[k] = from[k];
        for (int64_t b = 0; b < nblk; ++b) sha256_compress(out, w + 16 * b);
      } else {
        sha256_lds_blocks(w, nblk, out);
      }
    }
    return;
  }
  if (L.leader()) {
    if (from) {
      for (int k = 0; k < 8; ++k) out[k] = from[k];
    } else {
      sha256_init(out);
    }
  }
  for (int64_t b0 = 0; b0 < nblk; b0 += L.n) {
    const int64_t b = b0 + L.lane;
    if (b < nblk) sha256_expand_kw(w + 16 * b, L.kw + kKwStride * L.lane);
    L.sync();
    if (L.leader()) {
      const int64_t m = nblk - b0 < L.n ? nblk - b0 : L.n;
      for (int64_t j = 0; j < m; ++j) sha256_rounds_kw(out, L.kw + kKwStride * j);
    }
    L.sync();
  }
}

// Midstate of the blocks of a captured record that lie entirely before its
// `"parent_hash": ` hole — they do not depend on the parent digest (sort_keys
// puts agent_did, changes and delta_id first), so the command
// wave compresses them while the hash engine is still busy with the parent.
// At most `max_blocks`; returns the count (0: nothing to do).  Valid on the leader.
AHV_HD int32_t capture_prefix(const Lanes& L, const Tables& t, const HashJob& j, uint32_t* w, int64_t cap_words,
                              int32_t max_blocks, uint32_t mid[8]) {
  if (j.hole < 64) return 0;
  int64_t pb = j.hole / 64;
  if (pb > max_blocks) pb = max_blocks;
  if (pb * 16 > cap_words) return 0;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(t.payload + j.off);
  for (int64_t i = L.lane; i < pb * 16; i += L.n) w[i] = bswap32(ld32f(s32 + i));
  L.sync();
  sha256_lds_blocks_par(L, w, pb, mid);
  L.sync();
  return static_cast<int32_t>(pb);
}

// Provisional Merkle root (hash-engine wave, while it would otherwise idle):
// after the capture of delta `d` of session `s` — the chain's n-th, n ≤ 64 —
// the root of the n leaves is computed ahead of time into s_proot, tagged with
// (n, d).  Terminate / compute_merkle_root use it when their leaf list is
// exactly that chain (same count, same last delta) and skip the tree.  The
// leaves come from walking d_prev back from d; the levels run SIMT: lanes
// 2i, 2i+1 expand the schedules of node i's two hex blocks (K+W rows), lane i
// then runs only the rounds, plus the constant 128-byte padding block (its
// schedule folds at compile time).  `abort()` is polled between levels (a new
// capture is queued: its digest comes first); returns false when abandoned or
// when the chain is not the expected one.  `lv`: 8·64 words of LDS.
// `cached` (or null): the chain's n leaf digests, in order, already at hand (the
// hash engine keeps the chain it is extending in LDS) — no walk over d_prev.
template <class Abort>
AHV_HD bool merkle_provisional(const Lanes& L, const Tables& t, int64_t s, int64_t d, int64_t n, uint32_t* lv,
                               const Abort& abort, const uint32_t* cached = nullptr) {
  if (n < 1 || n > 64 || L.kw == nullptr) return false;
  int ok = 1;
  if (cached) {
    for (int64_t i = L.lane; i < 8 * n; i += L.n) lv[i] = cached[i];
  } else if (L.leader()) {
    int64_t k = d;
    for (int64_t i = n - 1; i >= 0; --i) {
      if (k < 0 || k >= t.cap.D || t.d_sess[k] != s || t.d_turn[k] != i + 1) {
        ok = 0;
        break;
      }
      load8(t.d_hash + 8 * k, lv + 8 * i);
      k = t.d_prev[k];
    }
  }
  if (!bcast(L, ok)) return false;
  L.sync();
  int64_t m = n;
  while (m > 1) {
    const int64_t half = (m + 1) / 2;
    if (L.lane < 2 * half) {
      const int64_t node = L.lane >> 1;
      int64_t child = 2 * node + (L.lane & 1);
      if (child >= m) child = 2 * node;  // odd level: the last node pairs with itself
      uint32_t blk[16];
      digest_to_hex_words(lv + 8 * child, blk);
      sha256_expand_kw(blk, L.kw + kKwStride * L.lane);
    }
    L.sync();
    uint32_t o[8];
    if (L.lane < half) {
      sha256_init(o);
      sha256_rounds_kw(o, L.kw + kKwStride * (2 * L.lane));
      sha256_rounds_kw(o, L.kw + kKwStride * (2 * L.lane + 1));
      sha256_compress_pad_only(o, 128u);
    }
    L.sync();
    if (L.lane < half) store8(lv + 8 * L.lane, o);
    L.sync();
    m = half;
    if (m > 1 && bcast(L, abort() ? 1 : 0)) return false;
  }
  if (L.leader()) {
    store8(t.s_proot + 8 * s, lv);
    t.s_proot_last[s] = static_cast<int32_t>(d);
    t.s_proot_n[s] = static_cast<int32_t>(n);
  }
  return true;
}

// ------------------------------------------------------------- session ops

AHV_HD void exec_sess(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r, uint8_t* bulk) {
  if (!L.leader()) return;
  const int64_t s = static_cast<int64_t>(c.a[0]);
  if (s < 0 || s >= t.cap.S || (c.op != OP_SESS_CREATE && c.op != OP_SESS_READ && t.s_state[s] == kFree8)) {
    if (L.leader()) out64(r + 1, ST_BAD_ARG);
    return;
  }
  switch (c.op) {
    case OP_SESS_CREATE: {
      if (t.s_state[s] != kFree8) {  // the row still holds a session: never overwrite it
        out64(r + 2, t.s_state[s]);
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.s_state[s] = SS_HANDSHAKING;  // create + begin_handshake (Hypervisor.create_session)
      t.s_mode[s] = static_cast<uint8_t>(c.a[3]);
      t.s_audit[s] = static_cast<uint8_t>(c.a[6]);
      t.s_maxpart[s] = static_cast<int32_t>(c.a[4]);
      t.s_minsig[s] = bitsd(c.a[5]);
      t.s_creator[s] = static_cast<int32_t>(c.a[1]);
      t.s_created[s] = static_cast<int64_t>(c.a[2]);
      t.s_terminated[s] = 0;
      t.s_pcount[s] = 0;
      t.s_pactive[s] = 0;
      t.s_dcount[s] = 0;
      t.s_dlast[s] = -1;
      t.s_committed[s] = 0;
      t.s_commit_n[s] = 0;
      t.s_released[s] = 0;
      t.s_retained[s] = 0;
      t.s_proot_n[s] = 0;  // no provisional Merkle root (a reused slot must not inherit one)
      t.s_uuid[4 * s + 0] = static_cast<uint32_t>(c.a[7] >> 32);
      t.s_uuid[4 * s + 1] = static_cast<uint32_t>(c.a[7]);
      t.s_uuid[4 * s + 2] = static_cast<uint32_t>(c.a[8] >> 32);
      t.s_uuid[4 * s + 3] = static_cast<uint32_t>(c.a[8]);
      for (int k = 0; k < 8; ++k) {
        t.s_head[8 * s + k] = 0;
        t.s_root[8 * s + k] = 0;
      }
      if (c.a[9]) t.s_state[s] = SS_CREATED;  // bare SharedSessionObject (no handshake yet)
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_HANDSHAKE: {
      const uint8_t st = t.s_state[s];
      if (st != SS_CREATED) {
        out64(r + 2, st);
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.s_state[s] = SS_HANDSHAKING;
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_JOIN: {
      // a1 agent, a2 σ_raw, a3 σ_eff, a4 flags (bit0 trustworthy, bit1 explicit ring), a5 ring, a6 now,
      // a7 creation stamp the host sent with its create (0: unchecked) — a host that posts
      // before it has seen its create's result: a row holding another session (the create
      // was refused) refuses the join instead of being changed (JOIN_NOT_MINE).  The stamp
      // is the low 64 bits of the session's id words (row_stamp), not a clock value: two
      // creates in the same microsecond (or under a pinned clock) still differ.
      if (c.a[7] && row_stamp(t, s) != c.a[7]) {
        out64(r + 1, JOIN_NOT_MINE);
        return;
      }
      const int32_t agent = static_cast<int32_t>(c.a[1]);
      const double sraw = bitsd(c.a[2]);
      const double seff = bitsd(c.a[3]);
      const uint8_t st = t.s_state[s];
      uint8_t ring = (c.a[4] & 2u) ? static_cast<uint8_t>(c.a[5]) : ring_from_sigma(seff, false);  // K01
      if (!(c.a[4] & 2u) && !(c.a[4] & 1u)) ring = RING3;  // untrustworthy history → sandbox
      const bool dup = find_part(t, s, agent) >= 0;
      const int32_t active = t.s_pactive[s];
      uint64_t code = join_check(st, dup, active, t.s_maxpart[s], seff, t.s_minsig[s], ring);
      if (code == JOIN_OK && t.s_pcount[s] >= t.cap.P) code = JOIN_ROWS;
      if (code == JOIN_OK) {
        const int64_t row = prow(t, s, t.s_pcount[s]);
        t.p_agent[row] = agent;
        t.p_ring[row] = ring;
        t.p_active[row] = 1;
        t.p_sraw[row] = sraw;
        t.p_seff[row] = seff;
        t.p_joined[row] = static_cast<int64_t>(c.a[6]);
        t.s_pcount[s] += 1;
        t.s_pactive[s] = active + 1;
      }
      out64(r + 2, ring);
      out64(r + 3, st);
      out64(r + 4, static_cast<uint64_t>(active));
      out64(r + 5, static_cast<uint64_t>(t.s_maxpart[s]));
      out64(r + 6, dbits(t.s_minsig[s]));
      out64(r + 1, code);
      return;
    }
    case OP_SESS_LEAVE: {
      const int32_t k = find_part(t, s, static_cast<int32_t>(c.a[1]));
      if (k < 0) {
        out64(r + 1, ST_NOT_FOUND);
        return;
      }
      const int64_t row = prow(t, s, k);
      if (t.p_active[row] & P_ACTIVE) {  // a commit-time membership bit (P_COMMITTED) stays
        t.p_active[row] = static_cast<uint8_t>(t.p_active[row] & ~P_ACTIVE);
        t.s_pactive[s] -= 1;
      }
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_UPDATE_RING:
    case OP_SESS_SET_SIGMA: {
      const int32_t k = find_part(t, s, static_cast<int32_t>(c.a[1]));
      if (k < 0) {
        out64(r + 1, ST_NOT_FOUND);
        return;
      }
      const int64_t row = prow(t, s, k);
      if (c.op == OP_SESS_UPDATE_RING) {
        t.p_ring[row] = static_cast<uint8_t>(c.a[2]);
      } else {
        t.p_seff[row] = bitsd(c.a[2]);
        if (c.a[3] & 1u) t.p_ring[row] = static_cast<uint8_t>(c.a[4]);
      }
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_SET_MODE:
      t.s_mode[s] = static_cast<uint8_t>(c.a[1]);
      out64(r + 1, ST_OK);
      return;
    case OP_SESS_ACTIVATE: {
      if (c.a[1] && row_stamp(t, s) != c.a[1]) {  // a1: creation stamp (see OP_SESS_JOIN)
        out64(r + 1, ACT_NOT_MINE);
        return;
      }
      const uint8_t st = t.s_state[s];
      out64(r + 2, st);
      if (st != SS_HANDSHAKING) {
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      if (t.s_pcount[s] == 0) {  // counts inactive rows too (reference session/__init__.py:81)
        out64(r + 1, 3);
        return;
      }
      t.s_state[s] = SS_ACTIVE;
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_TERMINATE: {
      const uint8_t st = t.s_state[s];
      out64(r + 2, st);
      if (!((session_op_allowed_from(OP_TERMINATE) >> st) & 1u)) {
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.s_state[s] = SS_TERMINATING;
      t.s_terminated[s] = static_cast<int64_t>(c.a[1]);
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_ARCHIVE: {
      const uint8_t st = t.s_state[s];
      out64(r + 2, st);
      if (st != SS_TERMINATING) {
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.s_state[s] = SS_ARCHIVED;
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SESS_READ: {
      // header → r[2..], participant rows → bulk at a[1] (stride 40 bytes)
      out64(r + 2, t.s_state[s]);
      out64(r + 3, t.s_mode[s]);
      out64(r + 4, static_cast<uint64_t>(t.s_pcount[s]));
      out64(r + 5, static_cast<uint64_t>(t.s_pactive[s]));
      out64(r + 6, static_cast<uint64_t>(t.s_created[s]));
      out64(r + 7, static_cast<uint64_t>(t.s_terminated[s]));
      out64(r + 8, static_cast<uint64_t>(t.s_dcount[s]));
      out64(r + 9, static_cast<uint64_t>(t.s_maxpart[s]));
      out64(r + 10, dbits(t.s_minsig[s]));
      out64(r + 11, t.s_audit[s]);
      out64(r + 12, static_cast<uint64_t>(t.s_committed[s]));
      out64(r + 13, static_cast<uint64_t>(t.s_commit_n[s]));
      out64(r + 14, static_cast<uint64_t>(static_cast<int64_t>(t.s_creator[s])));
      out64(r + 15, static_cast<uint64_t>(t.s_released[s]));
      out64(r + 16, static_cast<uint64_t>(t.s_retained[s]));
      for (int k = 0; k < 4; ++k) out64(r + 17 + k, (uint64_t(t.s_uuid[4 * s + k])));
      for (int k = 0; k < 8; ++k) out64(r + 21 + k, uint64_t(t.s_root[8 * s + k]));
      for (int k = 0; k < 8; ++k) out64(r + 29 + k, uint64_t(t.s_head[8 * s + k]));
      if (bulk) {
        uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[1]);
        const int32_t n = t.s_pcount[s];
        for (int32_t k = 0; k < n; ++k) {
          const int64_t row = prow(t, s, k);
          out64(b + 5 * k + 0, static_cast<uint64_t>(static_cast<int64_t>(t.p_agent[row])));
          out64(b + 5 * k + 1, uint64_t(t.p_ring[row]) | (uint64_t(t.p_active[row]) << 8));
          out64(b + 5 * k + 2, dbits(t.p_sraw[row]));
          out64(b + 5 * k + 3, dbits(t.p_seff[row]));
          out64(b + 5 * k + 4, static_cast<uint64_t>(t.p_joined[row]));
        }
      }
      out64(r + 1, ST_OK);
      return;
    }
    default:
      out64(r + 1, ST_BAD_OP);  // an unassigned code in the session range
      break;
  }
}

// Collect a session's delta digests into scratch (in capture order) from the
// arena indices the host recorded at capture time; every index is validated
// against the chain (owner session, turn, count).  Returns the count or -1.
AHV_HD int64_t gather_leaves(const Lanes& L, const Tables& t, int64_t s, const IndexList& idx, int64_t n,
                             uint32_t* lv, int64_t cutoff, int64_t* expired_out) {
  int bad = 0;
  int64_t expired = 0;
  for (int64_t i = L.lane; i < n; i += L.n) {
    const int32_t d = idx[i];
    if (d < 0 || d >= t.cap.D || t.d_sess[d] != s || t.d_turn[d] != i + 1) {
      bad = 1;
      continue;
    }
    load8(t.d_hash + 8 * static_cast<int64_t>(d), lv + 8 * i);
    if (t.d_ts[d] < cutoff) ++expired;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  bad = __any(bad) ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) expired += __shfl_xor(expired, o);
#endif
  L.sync();
  if (expired_out) *expired_out = expired;
  return bad ? -1 : n;
}

// ------------------------------------------------------------- vouch ops

// K07: release every still-active edge of liability session `v` (reference
// vouching.py:176-184); returns the count.
AHV_HD int32_t release_vsess(const Tables& t, int32_t v, int64_t now) {
  int32_t n = 0;
  if (v < 0 || v >= t.cap.V) return 0;
  for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e]) {
    if (t.e_active[e]) {
      t.e_active[e] = 0;
      t.e_released[e] = now;
      ++n;
    }
  }
  return n;
}

// Does voucher→vouchee close a cycle among the live edges of `v`?  Non-parity:
// true reachability; parity: the reference BFS that also flags diamonds (Q05).
// Work arrays in scratch; returns 2 when scratch is too small.
AHV_HD int creates_cycle(const Tables& t, int32_t v, int32_t voucher, int32_t vouchee, int64_t now, bool parity) {
  int32_t* from = reinterpret_cast<int32_t*>(t.scratch);
  const int64_t cap = t.cap.X / 16;
  int32_t* to = from + cap;
  int32_t* q = to + cap;
  int32_t* seen = q + cap;
  int64_t m = 0;
  for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e]) {
    if (!edge_live(t, e, now)) continue;
    if (m >= cap) return 2;
    from[m] = t.e_voucher[e];
    to[m] = t.e_vouchee[e];
    ++m;
  }
  for (int64_t i = 0; i < m; ++i)
    if (from[i] == vouchee && to[i] == voucher) return 1;
  int64_t qh = 0, qt = 0, ns = 0;
  auto is_seen = [&](int32_t a) {
    for (int64_t k = 0; k < ns; ++k)
      if (seen[k] == a) return true;
    return false;
  };
  if (parity) {
    seen[ns++] = voucher;
    q[qt++] = vouchee;
    while (qh < qt) {
      const int32_t cur = q[qh++];
      if (is_seen(cur)) return 1;
      if (ns >= cap) return 2;
      seen[ns++] = cur;
      for (int64_t i = 0; i < m; ++i) {
        if (from[i] != cur || is_seen(to[i])) continue;
        if (qt >= cap) return 2;
        q[qt++] = to[i];
      }
    }
    return 0;
  }
  seen[ns++] = vouchee;
  q[qt++] = vouchee;
  while (qh < qt) {
    const int32_t cur = q[qh++];
    for (int64_t i = 0; i < m; ++i) {
      if (from[i] != cur) continue;
      const int32_t nx = to[i];
      if (nx == voucher) return 1;
      if (!is_seen(nx)) {
        if (ns >= cap || qt >= cap) return 2;
        seen[ns++] = nx;
        q[qt++] = nx;
      }
    }
  }
  return 0;
}

AHV_HD double exposure_of(const Tables& t, int32_t v, int32_t voucher, int64_t now) {
  double cur = 0.0;
  for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e])
    if (t.e_voucher[e] == voucher && edge_live(t, e, now)) cur += t.e_bonded[e];
  return cur;
}

// Slash working set in scratch: (agent, σ) score pairs, then the clip list.
struct Scores {
  int32_t* agent;
  double* sigma;
  int64_t n, cap;
  AHV_HD int64_t find(int32_t a) const {
    for (int64_t k = 0; k < n; ++k)
      if (agent[k] == a) return k;
    return -1;
  }
  AHV_HD double get(int32_t a) const {
    const int64_t k = find(a);
    return k < 0 ? 0.0 : sigma[k];
  }
  AHV_HD bool set(int32_t a, double v) {
    int64_t k = find(a);
    if (k < 0) {
      if (n >= cap) return false;
      k = n++;
      agent[k] = a;
    }
    sigma[k] = v;
    return true;
  }
};

AHV_HD bool has_live_vouchers(const Tables& t, int32_t v, int32_t agent, int64_t now) {
  for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e])
    if (t.e_vouchee[e] == agent && edge_live(t, e, now)) return true;
  return false;
}

// K06 — SlashingEngine.slash with its cascade (reference slashing.py:63-143),
// pre-order like the recursion: one record per slash (frame) followed by its
// clips, then the children of each clip in clip order (a child is eligible when
// its σ after the clip is < SIGMA_FLOOR + 0.01 and it still has live vouchers
// *at that moment*, i.e. after earlier siblings' subtrees released bonds).
// Output u64 words: per frame [vouchee, depth, nclips, σ_before bits] then per
// clip [voucher, before bits, after bits, edge].  Clips are mirrored in scratch
// (clip_v/clip_a) so the descent never reads back the host-memory output.
// Returns words written, or -1 when an output/scratch bound is hit.
AHV_HD int64_t slash_cascade(const Tables& t, int32_t v, int32_t root, double root_sigma, double w, int64_t now,
                             Scores& sc, int32_t* clip_v, double* clip_a, int64_t clip_cap, uint64_t* out,
                             int64_t out_cap, int start_depth) {
  constexpr int kDepth = 3;  // MAX_CASCADE_DEPTH 2 → frames at depth 0..2
  struct Frame {
    int64_t base;  // first clip of this frame in clip_v/clip_a
    int32_t nclips, next;
  } fr[kDepth];
  int64_t wpos = 0, ncl = 0;
  if (start_depth < 0) start_depth = 0;
  if (start_depth > kDepth - 1) start_depth = kDepth - 1;
  int depth = start_depth;
  int32_t vouchee = root;
  double before = root_sigma;
  for (;;) {
    if (wpos + 4 > out_cap) return -1;
    const int64_t hdr = wpos;
    out64(out + hdr + 0, static_cast<uint64_t>(static_cast<int64_t>(vouchee)));
    out64(out + hdr + 1, static_cast<uint64_t>(depth));
    out64(out + hdr + 3, dbits(before));
    wpos += 4;
    if (!sc.set(vouchee, 0.0)) return -1;
    const int64_t base = ncl;
    for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e]) {
      if (t.e_vouchee[e] != vouchee || !edge_live(t, e, now)) continue;
      const int32_t vr = t.e_voucher[e];
      const double b = sc.get(vr);
      double a = b * (1.0 - w);
      if (a < 0.05) a = 0.05;  // clip_sigma: max(σ·(1−ω), SIGMA_FLOOR)
      if (!sc.set(vr, a) || ncl >= clip_cap || wpos + 4 > out_cap) return -1;
      out64(out + wpos + 0, static_cast<uint64_t>(static_cast<int64_t>(vr)));
      out64(out + wpos + 1, dbits(b));
      out64(out + wpos + 2, dbits(a));
      out64(out + wpos + 3, static_cast<uint64_t>(static_cast<int64_t>(e)));
      wpos += 4;
      clip_v[ncl] = vr;
      clip_a[ncl] = a;
      ++ncl;
      t.e_active[e] = 0;  // release_bond
      t.e_released[e] = now;
    }
    out64(out + hdr + 2, static_cast<uint64_t>(ncl - base));
    fr[depth].base = base;
    fr[depth].nclips = static_cast<int32_t>(ncl - base);
    fr[depth].next = 0;
    bool descended = false;
    for (;;) {
      if (depth < kDepth - 1) {
        Frame& f = fr[depth];
        while (f.next < f.nclips) {
          const int64_t k = f.base + f.next;
          f.next += 1;
          if (clip_a[k] < 0.05 + 0.01 && has_live_vouchers(t, v, clip_v[k], now)) {
            vouchee = clip_v[k];
            before = clip_a[k];
            depth += 1;
            descended = true;
            break;
          }
        }
        if (descended) break;
      }
      if (depth == start_depth) return wpos;
      depth -= 1;
    }
  }
}

AHV_HD void exec_vouch(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r, uint8_t* bulk) {
  if (!L.leader()) return;
  switch (c.op) {
    case OP_VOUCH: {
      // a0 vsess, a1 voucher, a2 vouchee, a3 σ bits, a4 pct bits (NaN = default),
      // a5 expiry µs (-1 none), a6 now, a7 max_exposure bits, a8 parity, a9 edge index
      const int32_t v = static_cast<int32_t>(c.a[0]);
      const int32_t vr = static_cast<int32_t>(c.a[1]), ve = static_cast<int32_t>(c.a[2]);
      const double sigma = bitsd(c.a[3]);
      const int64_t now = static_cast<int64_t>(c.a[6]);
      const int64_t e = static_cast<int64_t>(c.a[9]);
      if (v < 0 || v >= t.cap.V || e < 0 || e >= t.cap.E) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      if (t.e_vsess[e] != -1) {  // edge row in use
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      if (vr == ve) {
        out64(r + 1, V_SELF);
        return;
      }
      if (sigma < 0.50) {
        out64(r + 1, V_LOW_SIGMA);
        return;
      }
      const int cyc = creates_cycle(t, v, vr, ve, now, c.a[8] != 0);
      if (cyc == 2) {
        out64(r + 1, ST_SCRATCH);
        return;
      }
      if (cyc) {
        out64(r + 1, V_CYCLE);
        return;
      }
      double pct = bitsd(c.a[4]);
      if (pct != pct) pct = 0.20;  // DEFAULT_BOND_PCT
      pct = pct < 0.0 ? 0.0 : (pct > 1.0 ? 1.0 : pct);
      const double bonded = sigma * pct;
      const double current = exposure_of(t, v, vr, now);
      const double limit = sigma * bitsd(c.a[7]);
      out64(r + 2, dbits(current));
      out64(r + 3, dbits(bonded));
      out64(r + 4, dbits(limit));
      out64(r + 5, dbits(pct));
      if (current + bonded > limit) {
        out64(r + 1, V_EXPOSURE);
        return;
      }
      t.e_voucher[e] = vr;
      t.e_vouchee[e] = ve;
      t.e_vsess[e] = v;
      t.e_next[e] = -1;
      t.e_active[e] = 1;
      t.e_bonded[e] = bonded;
      t.e_pct[e] = pct;
      t.e_expiry[e] = static_cast<int64_t>(c.a[5]);
      t.e_released[e] = -1;
      t.e_created[e] = now;
      const int32_t tail = t.v_tail[v];
      if (tail < 0) t.v_head[v] = static_cast<int32_t>(e);
      else t.e_next[tail] = static_cast<int32_t>(e);
      t.v_tail[v] = static_cast<int32_t>(e);
      out64(r + 1, V_OK);
      return;
    }
    case OP_SIGMA_EFF: {
      // a0 vsess, a1 vouchee, a2 σ bits, a3 ω bits, a4 now — sum in creation order (K03 scalar path)
      const int32_t v = static_cast<int32_t>(c.a[0]);
      const int32_t ve = static_cast<int32_t>(c.a[1]);
      const int64_t now = static_cast<int64_t>(c.a[4]);
      double contrib = 0.0;
      if (v >= 0 && v < t.cap.V)
        for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e])
          if (t.e_vouchee[e] == ve && edge_live(t, e, now)) contrib += t.e_bonded[e];
      double s = bitsd(c.a[2]) + bitsd(c.a[3]) * contrib;
      if (s > 1.0) s = 1.0;
      out64(r + 2, dbits(s));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_EXPOSURE: {
      const int32_t v = static_cast<int32_t>(c.a[0]);
      const double x = (v >= 0 && v < t.cap.V)
                           ? exposure_of(t, v, static_cast<int32_t>(c.a[1]), static_cast<int64_t>(c.a[2]))
                           : 0.0;
      out64(r + 2, dbits(x));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_RELEASE_BOND: {
      const int64_t e = static_cast<int64_t>(c.a[0]);
      if (e < 0 || e >= t.cap.E) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      t.e_active[e] = 0;
      t.e_released[e] = static_cast<int64_t>(c.a[1]);
      out64(r + 1, ST_OK);
      return;
    }
    case OP_RELEASE_SESSION: {
      const int32_t n = release_vsess(t, static_cast<int32_t>(c.a[0]), static_cast<int64_t>(c.a[1]));
      out64(r + 2, static_cast<uint64_t>(n));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_VOUCH_LIST: {
      // a0 vsess, a1 filter (0 all, 1 live by vouchee a2, 2 live by voucher a2, 3 live), a3 now,
      // a4 bulk offset, a5 bulk capacity (edges), a6 matches to skip (paging).
      // Rows: [edge, voucher, vouchee, active, bonded, pct, expiry, released];
      // r[2] = total matches (the host pages until it has them all).
      const int32_t v = static_cast<int32_t>(c.a[0]);
      const int64_t now = static_cast<int64_t>(c.a[3]);
      const int32_t who = static_cast<int32_t>(c.a[2]);
      const int64_t skip = static_cast<int64_t>(c.a[6]);
      uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[4]);
      int64_t n = 0;
      if (v >= 0 && v < t.cap.V) {
        for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e]) {
          const bool live = edge_live(t, e, now);
          bool keep = true;
          switch (c.a[1]) {
            case 1: keep = live && t.e_vouchee[e] == who; break;
            case 2: keep = live && t.e_voucher[e] == who; break;
            case 3: keep = live; break;
            default: break;
          }
          if (!keep) continue;
          if (n >= skip && n - skip < static_cast<int64_t>(c.a[5])) {
            uint64_t* row = b + 8 * (n - skip);
            out64(row + 0, static_cast<uint64_t>(static_cast<int64_t>(e)));
            out64(row + 1, static_cast<uint64_t>(static_cast<int64_t>(t.e_voucher[e])));
            out64(row + 2, static_cast<uint64_t>(static_cast<int64_t>(t.e_vouchee[e])));
            out64(row + 3, uint64_t(t.e_active[e]));
            out64(row + 4, dbits(t.e_bonded[e]));
            out64(row + 5, dbits(t.e_pct[e]));
            out64(row + 6, static_cast<uint64_t>(t.e_expiry[e]));
            out64(row + 7, static_cast<uint64_t>(t.e_released[e]));
          }
          ++n;
        }
      }
      out64(r + 2, static_cast<uint64_t>(n));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_EDGE_READ: {
      const int64_t e = static_cast<int64_t>(c.a[0]);
      if (e < 0 || e >= t.cap.E) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      out64(r + 2, t.e_active[e]);
      out64(r + 3, static_cast<uint64_t>(t.e_released[e]));
      out64(r + 4, dbits(t.e_bonded[e]));
      out64(r + 5, dbits(t.e_pct[e]));
      out64(r + 6, static_cast<uint64_t>(t.e_expiry[e]));
      out64(r + 7, static_cast<uint64_t>(static_cast<int64_t>(t.e_voucher[e])));
      out64(r + 8, static_cast<uint64_t>(static_cast<int64_t>(t.e_vouchee[e])));
      out64(r + 9, static_cast<uint64_t>(static_cast<int64_t>(t.e_vsess[e])));
      out64(r + 10, static_cast<uint64_t>(t.e_created[e]));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SLASH: {
      // a0 vsess, a1 vouchee, a2 σ_before bits, a3 ω bits, a4 now, a5 nscores (pairs in staging at a6),
      // a7 bulk offset of the record stream, a8 its capacity (words), a9 bulk offset of the scores out
      const int32_t v = static_cast<int32_t>(c.a[0]);
      const int64_t now = static_cast<int64_t>(c.a[4]);
      const int64_t ns = static_cast<int64_t>(c.a[5]);
      const int64_t cap = t.cap.X / 24;  // scratch: agents i32, σ f64, clip agents i32, clip σ f64
      Scores sc;
      sc.agent = reinterpret_cast<int32_t*>(t.scratch);
      sc.sigma = reinterpret_cast<double*>(t.scratch + 8 * cap);
      int32_t* clip_v = reinterpret_cast<int32_t*>(t.scratch + 16 * cap);
      double* clip_a = reinterpret_cast<double*>(t.scratch + 16 * cap + 8 * (cap / 2));
      sc.cap = cap;
      sc.n = 0;
      if (ns > cap || v < 0 || v >= t.cap.V) {
        out64(r + 1, ST_SCRATCH);
        return;
      }
      const uint64_t* pairs = reinterpret_cast<const uint64_t*>(t.staging + c.a[6]);
      for (int64_t k = 0; k < ns; ++k) {
        sc.agent[k] = static_cast<int32_t>(ld64f(pairs + 2 * k));
        sc.sigma[k] = bitsd(ld64f(pairs + 2 * k + 1));
      }
      sc.n = ns;
      uint64_t* out = reinterpret_cast<uint64_t*>(bulk + c.a[7]);
      const int64_t words = slash_cascade(t, v, static_cast<int32_t>(c.a[1]), bitsd(c.a[2]), bitsd(c.a[3]), now,
                                          sc, clip_v, clip_a, cap / 2, out, static_cast<int64_t>(c.a[8]),
                                          static_cast<int>(c.a[10]));
      if (words < 0) {
        out64(r + 1, ST_SCRATCH);
        return;
      }
      uint64_t* so = reinterpret_cast<uint64_t*>(bulk + c.a[9]);
      for (int64_t k = 0; k < sc.n; ++k) {
        out64(so + 2 * k, static_cast<uint64_t>(static_cast<int64_t>(sc.agent[k])));
        out64(so + 2 * k + 1, dbits(sc.sigma[k]));
      }
      out64(r + 2, static_cast<uint64_t>(words));
      out64(r + 3, static_cast<uint64_t>(sc.n));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_V_RETIRE: {
      // a0 vsess, a1 bulk offset, a2 capacity (edges).  Every edge of the list —
      // all released by the close that precedes this — is reported as
      // [edge, active, released µs] and returned to the free state; the list is
      // emptied (later vouches in the same session start a new list).  Nothing
      // changes when the list is longer than the capacity (ST_SCRATCH + count).
      const int32_t v = static_cast<int32_t>(c.a[0]);
      if (v < 0 || v >= t.cap.V) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      int64_t n = 0;
      for (int32_t e = t.v_head[v]; e >= 0; e = t.e_next[e]) ++n;
      out64(r + 2, static_cast<uint64_t>(n));
      if (n > static_cast<int64_t>(c.a[2])) {
        out64(r + 1, ST_SCRATCH);
        return;
      }
      uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[1]);
      int64_t k = 0;
      for (int32_t e = t.v_head[v]; e >= 0;) {
        const int32_t nx = t.e_next[e];
        out64(b + 3 * k + 0, static_cast<uint64_t>(static_cast<int64_t>(e)));
        out64(b + 3 * k + 1, uint64_t(t.e_active[e]));
        out64(b + 3 * k + 2, static_cast<uint64_t>(t.e_released[e]));
        t.e_active[e] = 0;
        t.e_vsess[e] = -1;
        t.e_next[e] = -1;
        ++k;
        e = nx;
      }
      t.v_head[v] = -1;
      t.v_tail[v] = -1;
      out64(r + 1, ST_OK);
      return;
    }
    default:
      out64(r + 1, ST_BAD_OP);
      break;
  }
}

// OP_FREE_ROWS: a0 kind (RowKind), a1 n, a2 staging offset of the row list.
// The host reclaims a row only once no API object refers to it any more; the
// command marks it free so the next create may claim it.  Runs after the hash
// engine has drained (needs_drain), so no queued capture still writes a freed
// delta row or the chain head of a freed session.
AHV_HD void exec_free_rows(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r) {
  const uint64_t kind = c.a[0];
  const uint64_t n = c.a[1];
  const IndexList idx = index_list(t, c, n, c.a[2]);
  int bad = 0;
  for (uint64_t i = L.lane; i < n; i += L.n) {
    const int64_t x = idx[i];
    switch (kind) {
      case RK_S:
        if (x < 0 || x >= t.cap.S) { bad = 1; break; }
        t.s_state[x] = kFree8;
        t.s_proot_n[x] = 0;
        t.s_dlast[x] = -1;
        t.s_dcount[x] = 0;
        break;
      case RK_G:
        if (x < 0 || x >= t.cap.G) { bad = 1; break; }
        t.g_state[x] = kFree8;
        break;
      case RK_T:
        if (x < 0 || x >= t.cap.T) { bad = 1; break; }
        t.t_state[x] = kFree8;
        t.t_saga[x] = -1;
        break;
      case RK_E:
        if (x < 0 || x >= t.cap.E) { bad = 1; break; }
        t.e_active[x] = 0;
        t.e_vsess[x] = -1;
        t.e_next[x] = -1;
        break;
      case RK_D:
        if (x < 0 || x >= t.cap.D) { bad = 1; break; }
        t.d_sess[x] = -1;
        t.d_turn[x] = 0;
        t.d_prev[x] = -1;
        t.d_hole[x] = -1;
        break;
      case RK_V:
        if (x < 0 || x >= t.cap.V) { bad = 1; break; }
        t.v_head[x] = -1;
        t.v_tail[x] = -1;
        break;
      default:
        bad = 1;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  bad = __any(bad) ? 1 : 0;
#endif
  L.sync();
  if (L.leader()) out64(r + 1, bad ? ST_BAD_ARG : ST_OK);
}

// OP_SESS_READ_MANY: a0 n, a1 staging offset of the slot list, a2 bulk offset,
// a3 participant rows too (1) or headers only (0).  One lane per session.
// Header row (kHdrWords u64): [state | mode<<8 | audit<<16, pcount | pactive<<32,
// created, terminated, dcount | commit_n<<32, maxpart, minsig bits, committed,
// creator, released | retained<<32, uuid (2 words), root (4 words), head (4 words)].
// With participants, session i's rows follow all headers at stride cap.P × 5 words
// (the OP_SESS_READ participant layout).
constexpr int kHdrWords = 20;

AHV_HD void exec_read_many(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r, uint8_t* bulk) {
  const uint64_t n = c.a[0];
  const IndexList idx = index_list(t, c, n, c.a[1]);
  uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[2]);
  const bool parts = c.a[3] != 0;
  uint64_t* pb = b + kHdrWords * n;
  int bad = 0;
  for (uint64_t i = L.lane; i < n; i += L.n) {
    const int64_t s = idx[i];
    uint64_t* h = b + kHdrWords * i;
    if (s < 0 || s >= t.cap.S) {
      bad = 1;
      continue;
    }
    out64(h + 0, uint64_t(t.s_state[s]) | (uint64_t(t.s_mode[s]) << 8) | (uint64_t(t.s_audit[s]) << 16));
    out64(h + 1, uint64_t(static_cast<uint32_t>(t.s_pcount[s])) | (uint64_t(static_cast<uint32_t>(t.s_pactive[s])) << 32));
    out64(h + 2, static_cast<uint64_t>(t.s_created[s]));
    out64(h + 3, static_cast<uint64_t>(t.s_terminated[s]));
    out64(h + 4, uint64_t(static_cast<uint32_t>(t.s_dcount[s])) | (uint64_t(static_cast<uint32_t>(t.s_commit_n[s])) << 32));
    out64(h + 5, static_cast<uint64_t>(static_cast<int64_t>(t.s_maxpart[s])));
    out64(h + 6, dbits(t.s_minsig[s]));
    out64(h + 7, static_cast<uint64_t>(t.s_committed[s]));
    out64(h + 8, static_cast<uint64_t>(static_cast<int64_t>(t.s_creator[s])));
    out64(h + 9, uint64_t(static_cast<uint32_t>(t.s_released[s])) | (uint64_t(static_cast<uint32_t>(t.s_retained[s])) << 32));
    for (int k = 0; k < 2; ++k)
      out64(h + 10 + k, (uint64_t(t.s_uuid[4 * s + 2 * k]) << 32) | uint64_t(t.s_uuid[4 * s + 2 * k + 1]));
    for (int k = 0; k < 4; ++k) {
      out64(h + 12 + k, (uint64_t(t.s_root[8 * s + 2 * k]) << 32) | uint64_t(t.s_root[8 * s + 2 * k + 1]));
      out64(h + 16 + k, (uint64_t(t.s_head[8 * s + 2 * k]) << 32) | uint64_t(t.s_head[8 * s + 2 * k + 1]));
    }
    if (parts) {
      uint64_t* p = pb + 5 * t.cap.P * i;
      const int32_t np = t.s_pcount[s];
      for (int32_t k = 0; k < np; ++k) {
        const int64_t row = prow(t, s, k);
        out64(p + 5 * k + 0, static_cast<uint64_t>(static_cast<int64_t>(t.p_agent[row])));
        out64(p + 5 * k + 1, uint64_t(t.p_ring[row]) | (uint64_t(t.p_active[row]) << 8));
        out64(p + 5 * k + 2, dbits(t.p_sraw[row]));
        out64(p + 5 * k + 3, dbits(t.p_seff[row]));
        out64(p + 5 * k + 4, static_cast<uint64_t>(t.p_joined[row]));
      }
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  bad = __any(bad) ? 1 : 0;
#endif
  L.sync();
  if (L.leader()) out64(r + 1, bad ? ST_BAD_ARG : ST_OK);
}

// ------------------------------------------------------------- saga ops

AHV_HD void exec_saga(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r, uint8_t* bulk) {
  if (!L.leader()) return;
  switch (c.op) {
    case OP_SAGA_CREATE: {
      const int64_t g = static_cast<int64_t>(c.a[0]);
      if (g < 0 || g >= t.cap.G) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      if (t.g_state[g] != kFree8) {
        out64(r + 2, t.g_state[g]);
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.g_state[g] = SG_RUNNING;
      t.g_created[g] = static_cast<int64_t>(c.a[1]);
      t.g_completed[g] = 0;
      t.g_nsteps[g] = 0;
      out64(r + 1, ST_OK);
      return;
    }
    case OP_STEP_ADD: {
      const int64_t g = static_cast<int64_t>(c.a[0]), st = static_cast<int64_t>(c.a[1]);
      if (g < 0 || g >= t.cap.G || st < 0 || st >= t.cap.T) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      if (t.t_state[st] != kFree8 || t.g_state[g] == kFree8) {
        out64(r + 2, t.t_state[st]);
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.t_saga[st] = static_cast<int32_t>(g);
      t.t_state[st] = ST_PENDING;
      t.t_undo[st] = static_cast<uint8_t>(c.a[2]);
      t.t_maxretry[st] = static_cast<int32_t>(c.a[3]);
      t.t_retry[st] = 0;
      t.t_started[st] = 0;
      t.t_completed[st] = 0;
      t.g_nsteps[g] += 1;
      out64(r + 1, ST_OK);
      return;
    }
    case OP_STEP_TRANSITION: {
      // a0 step, a1 to-state, a2 now, a3 retry count (≥0 sets retry_count first)
      const int64_t st = static_cast<int64_t>(c.a[0]);
      if (st < 0 || st >= t.cap.T) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      const uint8_t to = static_cast<uint8_t>(c.a[1]);
      const uint8_t from = t.t_state[st];
      if (static_cast<int64_t>(c.a[3]) >= 0) t.t_retry[st] = static_cast<int32_t>(c.a[3]);
      out64(r + 2, from);
      if (!((step_transitions(from) >> to) & 1u)) {  // K13
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.t_state[st] = to;
      if (to == ST_EXECUTING) t.t_started[st] = static_cast<int64_t>(c.a[2]);
      else if (step_stamps_completed(to)) t.t_completed[st] = static_cast<int64_t>(c.a[2]);
      out64(r + 1, ST_OK);
      return;
    }
    case OP_STEP_SET: {
      // direct write outside the FSM (reference orchestrator.py:124/134 retry reset, :167 no-undo)
      const int64_t st = static_cast<int64_t>(c.a[0]);
      if (st < 0 || st >= t.cap.T) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      t.t_state[st] = static_cast<uint8_t>(c.a[1]);
      if (static_cast<int64_t>(c.a[2]) >= 0) t.t_retry[st] = static_cast<int32_t>(c.a[2]);
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SAGA_TRANSITION: {
      const int64_t g = static_cast<int64_t>(c.a[0]);
      if (g < 0 || g >= t.cap.G) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      const uint8_t to = static_cast<uint8_t>(c.a[1]);
      const uint8_t from = t.g_state[g];
      out64(r + 2, from);
      if (!((saga_transitions(from) >> to) & 1u)) {
        out64(r + 1, ST_BAD_STATE);
        return;
      }
      t.g_state[g] = to;
      if (saga_terminal(to)) t.g_completed[g] = static_cast<int64_t>(c.a[2]);
      out64(r + 1, ST_OK);
      return;
    }
    case OP_STEP_READ: {
      const int64_t st = static_cast<int64_t>(c.a[0]);
      if (st < 0 || st >= t.cap.T) {
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      out64(r + 2, t.t_state[st]);
      out64(r + 3, static_cast<uint64_t>(static_cast<int64_t>(t.t_retry[st])));
      out64(r + 4, static_cast<uint64_t>(t.t_started[st]));
      out64(r + 5, static_cast<uint64_t>(t.t_completed[st]));
      out64(r + 6, static_cast<uint64_t>(static_cast<int64_t>(t.t_saga[st])));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_SAGA_READ:
    case OP_SAGA_PLAN: {
      // a0 saga, a1 nsteps, a2 staging offset of step indices (if > inline), a3 bulk offset
      const int64_t g = static_cast<int64_t>(c.a[0]);
      const uint64_t n = c.a[1];
      const IndexList idx = index_list(t, c, n, c.a[2]);
      uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[3]);
      bool bad = g < 0 || g >= t.cap.G;
      for (uint64_t k = 0; k < n && !bad; ++k) bad = idx[k] < 0 || idx[k] >= t.cap.T;
      if (bad) {  // row indices come from API objects: validated like every other row argument
        out64(r + 1, ST_BAD_ARG);
        return;
      }
      out64(r + 2, t.g_state[g]);
      out64(r + 3, static_cast<uint64_t>(t.g_created[g]));
      out64(r + 4, static_cast<uint64_t>(t.g_completed[g]));
      out64(r + 5, static_cast<uint64_t>(t.g_nsteps[g]));
      if (c.op == OP_SAGA_READ) {
        for (uint64_t k = 0; k < n; ++k) {
          const int32_t st = idx[k];
          out64(b + 4 * k + 0, uint64_t(t.t_state[st]) | (uint64_t(static_cast<uint32_t>(t.t_retry[st])) << 8));
          out64(b + 4 * k + 1, static_cast<uint64_t>(t.t_started[st]));
          out64(b + 4 * k + 2, static_cast<uint64_t>(t.t_completed[st]));
          out64(b + 4 * k + 3, static_cast<uint64_t>(t.t_saga[st] == g));
        }
      } else {
        // K14: committed steps in reverse order
        uint64_t m = 0;
        for (uint64_t k = n; k-- > 0;) {
          const int32_t st = idx[k];
          if (t.t_state[st] == ST_COMMITTED) out64(b + m++, k);
        }
        out64(r + 6, m);
      }
      out64(r + 1, ST_OK);
      return;
    }
    default:
      out64(r + 1, ST_BAD_OP);
      break;
  }
}

// ------------------------------------------------------------- audit ops

// K08, command-wave half: validate, record the delta row and the chain links,
// and describe the hashing work.  Returns false (result written) on a bad request.
AHV_HD bool capture_begin(const Lanes& L, const Tables& t, const Cmd& c, uint64_t seq, uint64_t* r, HashJob& j) {
  if (!L.leader()) return true;
  // a0 session, a1 delta index, a2 turn, a3 ts, a4 payload offset, a5 payload length,
  // a6 parent-hole offset in the payload (-1: turn 1, "null" already written)
  const int64_t s = static_cast<int64_t>(c.a[0]);
  const int64_t d = static_cast<int64_t>(c.a[1]);
  const int32_t turn = static_cast<int32_t>(c.a[2]);
  const int64_t hole = static_cast<int64_t>(c.a[6]);
  bool ok = !(s < 0 || s >= t.cap.S || d < 0 || d >= t.cap.D || turn != t.s_dcount[s] + 1 ||
              c.a[4] + c.a[5] > static_cast<uint64_t>(t.cap.B));
  if (ok && (t.d_sess[d] != -1 || t.s_state[s] == kFree8)) ok = false;  // delta row in use / no session
  const int32_t prev = ok ? t.s_dlast[s] : -1;
  if (ok && hole >= 0 && prev < 0) ok = false;
  if (ok && hole >= 0 && (hole + 66 > static_cast<int64_t>(c.a[5]))) ok = false;
  if (!ok) {
    out64(r + 1, ST_BAD_ARG);
    return false;
  }
  t.d_sess[d] = static_cast<int32_t>(s);
  t.d_turn[d] = turn;
  t.d_prev[d] = prev;
  t.d_ts[d] = static_cast<int64_t>(c.a[3]);
  t.d_off[d] = static_cast<int64_t>(c.a[4]);
  t.d_len[d] = static_cast<int32_t>(c.a[5]);
  t.d_hole[d] = static_cast<int32_t>(hole);  // offset of the quoted parent digest (-1: null parent)
  t.s_dlast[s] = static_cast<int32_t>(d);
  t.s_dcount[s] = turn;
  j.seq = seq;
  j.s = s;
  j.d = d;
  j.off = static_cast<int64_t>(c.a[4]);
  j.len = static_cast<int64_t>(c.a[5]);
  j.hole = hole;
  j.prev = prev;
  j.spec = hole >= 0 && (c.a[7] & 1u) ? 1 : 0;
  j.full = 0;
  return true;
}

// Speculated link (worker helper waves): SHA-256 of a record stored with its
// predicted parent digest already in the hole (HashJob::spec), and that parent
// parsed back from its hex — the whole record hashed before the parent is final.
// ≤ `max_blocks` blocks (false otherwise: the engine hashes it).  `w`: LDS staging
// of max_blocks·16 words; the lanes expand the schedules, the leader runs the rounds.
// Valid on the leader.
AHV_HD bool capture_spec_full(const Lanes& L, const Tables& t, const HashJob& j, uint32_t* w, int32_t max_blocks,
                              uint32_t dig[8], uint32_t par[8]) {
  if (!j.spec || j.hole < 0) return false;
  const int64_t nblk = (j.len + 9 + 63) / 64;
  if (nblk > max_blocks) return false;
  if (stage_words(L, t.payload + j.off, static_cast<uint64_t>(j.len), w, 16 * max_blocks) < 0) return false;
  // the quoted parent hex at the hole, back to 8 digest words: lane k decodes char k
  // (the nibbles are gathered by shuffles)
  const uint8_t* lb = reinterpret_cast<const uint8_t*>(w);
  int bad = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t b = static_cast<uint64_t>(j.hole) + 1 + static_cast<uint64_t>(L.lane);
  const uint32_t ch = lb[(b & ~uint64_t(3)) | (3 - (b & 3))];
  const uint32_t dg = ch - 0x30u, lc = ch - 0x61u;
  const uint32_t nib = dg < 10u ? dg : lc + 10u;
  bad = __any(dg >= 10u && lc >= 6u) ? 1 : 0;
  uint32_t v = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) v = (v << 4) | __shfl(nib, 8 * (L.lane & 7) + e);
#pragma unroll
  for (int k = 0; k < 8; ++k) par[k] = __shfl(v, k);
#else
  (void)lb;
  bad = 1;  // host twin (one lane): spec jobs are a worker feature
#endif
  if (bad) return false;
  sha256_lds_blocks_par(L, w, nblk, dig);
  L.sync();
  return true;
}

// K08, hashing half (one wave): stage the record into LDS as message words with
// the parent's quoted digest spliced in, then the serial SHA-256 on lane 0;
// writes the digest row, the chain head and the result words r[1..9] (not the
// sequence word).
AHV_HD uint64_t engine_clock() {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_s_memrealtime();  // 100 MHz
#else
  return 0;
#endif
}

AHV_HD void capture_finish(const Lanes& L, const Tables& t, const HashJob& j, uint64_t* r, uint64_t* tele = nullptr,
                           uint32_t* hout = nullptr) {
  const uint64_t c0 = engine_clock();
  uint8_t* p = t.payload + j.off;
  const uint32_t* parent = j.prev >= 0 ? t.d_hash + 8 * j.prev : t.s_head + 8 * j.s;
  const int64_t nblk = stage_message(L, p, static_cast<uint64_t>(j.len), j.hole, parent);
  const uint64_t c1 = engine_clock();
  uint32_t h[8];
  // blocks before the parent hole may already be compressed (by the command wave)
  const int64_t skip = nblk >= 0 && j.mid_blocks > 0 && j.mid_blocks < nblk ? j.mid_blocks : 0;
  if (nblk >= 0) sha256_lds_blocks_par(L, L.lds + 16 * skip, nblk - skip, h, skip ? j.mid : nullptr);
  if (!L.leader()) return;
  // engine telemetry in the result slot: stage / hash ticks (10 ns) and blocks
  out64(r + 10, c1 - c0);
  out64(r + 11, engine_clock() - c1);
  out64(r + 12, static_cast<uint64_t>(nblk));
  if (tele) {  // worker timeline: blocks | skipped << 8 | stage ticks << 24 | hash ticks << 44
    const uint64_t c2 = engine_clock();
    tele[0] = (static_cast<uint64_t>(nblk) & 0xff) | (static_cast<uint64_t>(skip & 0xff) << 8) |
              ((c1 - c0) & 0xfffff) << 24 | ((c2 - c1) & 0xfffff) << 44;
  }
  if (nblk < 0) sha256_fine(p, static_cast<uint64_t>(j.len), h);  // record larger than the LDS window
  store8(t.d_hash + 8 * j.d, h);
  store8(t.s_head + 8 * j.s, h);
  for (int k = 0; k < 8; ++k) out64(r + 2 + k, h[k]);
  out64(r + 1, ST_OK);
  if (hout)
    for (int k = 0; k < 8; ++k) hout[k] = h[k];
}

AHV_HD void exec_delta(const Lanes& L, const Tables& t, const Cmd& c, uint64_t* r, uint8_t* bulk) {
  switch (c.op) {
    case OP_DELTA_MERKLE:
    case OP_SESS_CLOSE: {
      // MERKLE: a0 session, a1 n, a2 staging offset of indices.
      // CLOSE:  a0 session, a1 n, a2 staging offset, a3 now, a4 vsess (-1 none),
      //         a5 retention cutoff µs, a6 audit flag
      const int64_t s = static_cast<int64_t>(c.a[0]);
      const int64_t n = static_cast<int64_t>(c.a[1]);
      if (s < 0 || s >= t.cap.S || 8 * 4 * n > t.cap.X) {
        if (L.leader()) out64(r + 1, s < 0 || s >= t.cap.S ? ST_BAD_ARG : ST_SCRATCH);
        return;
      }
      const bool close = c.op == OP_SESS_CLOSE;
      // The hash engine may still be computing this chain's provisional root: every
      // step that does not read it (row checks, leaf gather, the close's row writes)
      // runs first, the wait for the tree (L.wait_tree) comes right before the root.
      // The row words this command reads, requested together (one memory round
      // trip for the lone command wave instead of one per check).
      uint8_t st_raw = 0;
      int64_t dcount_raw = 0;
      if (L.leader()) {
        st_raw = t.s_state[s];
        dcount_raw = static_cast<int64_t>(t.s_dcount[s]);
      }
      const uint8_t st0 = bcast(L, st_raw);
      if (close && !((session_op_allowed_from(OP_TERMINATE) >> st0) & 1u)) {
        if (L.leader()) {
          out64(r + 2, st0);
          out64(r + 1, ST_BAD_STATE);
        }
        return;
      }
      if (n != bcast(L, dcount_raw)) {
        if (L.leader()) out64(r + 1, ST_BAD_ARG);
        return;
      }
      uint32_t* lv = reinterpret_cast<uint32_t*>(t.scratch);
      int64_t expired = 0;
      const int64_t cutoff = close ? static_cast<int64_t>(c.a[5]) : INT64_MIN;
      const int64_t got = gather_leaves(L, t, s, index_list(t, c, static_cast<uint64_t>(n), c.a[2]), n, lv, cutoff,
                                        &expired);
      if (got < 0) {
        if (L.leader()) out64(r + 1, ST_BAD_ARG);
        return;
      }
      const bool want_root = n > 0 && (!close || c.a[6]);
      const int64_t now = static_cast<int64_t>(c.a[3]);
      int32_t rel = 0;
      if (close && L.leader()) {  // everything of the close that does not need the root
        t.s_state[s] = SS_TERMINATING;
        t.s_terminated[s] = now;
        if (want_root) mark_committed_participants(t, s);
        rel = release_vsess(t, static_cast<int32_t>(static_cast<int64_t>(c.a[4])), now);  // K07
        t.s_released[s] = rel;
        t.s_retained[s] = static_cast<int32_t>(n - expired);  // EphemeralGC retention
      }
      L.wait_tree(s);
      // the hash engine's provisional root, when it covers exactly these leaves
      // (its tag and digest requested together)
      const IndexList il = index_list(t, c, static_cast<uint64_t>(n), c.a[2]);
      uint32_t root[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int have_raw = 0;
      if (want_root && L.leader()) {
        const int64_t pn = static_cast<int64_t>(t.s_proot_n[s]);
        const int64_t pl = static_cast<int64_t>(t.s_proot_last[s]);
        load8(t.s_proot + 8 * s, root);
        have_raw = pn == n && pl == il[n - 1];
      }
      const bool have = want_root && bcast(L, have_raw) != 0;
      if (want_root && !have) merkle_inplace(L, lv, n);  // K09
      if (!L.leader()) return;
      if (want_root && !have) load8(lv, root);
      for (int k = 0; k < 8; ++k) out64(r + 3 + k, root[k]);
      out64(r + 2, want_root ? 1u : 0u);
      if (close) {
        if (want_root) {  // CommitmentEngine.commit
          store8(t.s_root + 8 * s, root);
          t.s_committed[s] = now;
          t.s_commit_n[s] = static_cast<int32_t>(n);
        }
        t.s_state[s] = SS_ARCHIVED;
        out64(r + 11, static_cast<uint64_t>(rel));
        out64(r + 12, static_cast<uint64_t>(expired));
      }
      out64(r + 1, ST_OK);
      return;
    }
    case OP_DELTA_VERIFY: {
      // K10 over host-presented records (the views the API handed out, possibly
      // tampered): a0 session, a1 n, a2 staging offset of the record table, a3
      // parity (reference verify: re-hash then compare links only, Q02), a4 bulk
      // offset for the re-hashed digests.  Record (11 u64): payload offset in
      // staging, length, arena index, presented digest (4 u64 = 8 u32 BE words),
      // presented parent (4 u64; all-ones = null).
      const int64_t s = static_cast<int64_t>(c.a[0]);
      const int64_t n = static_cast<int64_t>(c.a[1]);
      const uint64_t* rec = reinterpret_cast<const uint64_t*>(t.staging + c.a[2]);
      const bool parity = c.a[3] != 0;
      // scratch: re-hashed [n][8], presented digests [n][8], presented parents [n][8], ok flags
      uint32_t* rh = reinterpret_cast<uint32_t*>(t.scratch);
      uint8_t* okv = t.scratch + 96 * n;
      if (97 * n > t.cap.X || s < 0 || s >= t.cap.S) {
        if (L.leader()) out64(r + 1, ST_SCRATCH);
        return;
      }
      uint64_t* b = bulk ? reinterpret_cast<uint64_t*>(bulk + c.a[4]) : nullptr;
      for (int64_t i = L.lane; i < n; i += L.n) {  // SIMT: one record per lane
        uint64_t q[11];
        for (int k = 0; k < 11; ++k) q[k] = ld64f(rec + 11 * i + k);
        uint32_t h[8];
        sha256_fine(t.staging + q[0], q[1], h);
        store8(rh + 8 * i, h);
        const uint32_t* ph = reinterpret_cast<const uint32_t*>(q + 3);
        const int64_t d = static_cast<int64_t>(q[2]);
        bool ok = d >= 0 && d < t.cap.D && t.d_sess[d] == s;
        for (int k = 0; k < 8; ++k) {
          ok = ok && h[k] == ph[k];
          if (d >= 0 && d < t.cap.D) ok = ok && t.d_hash[8 * d + k] == ph[k];  // device-held chain
        }
        okv[i] = ok ? 1 : 0;
        if (b)
          for (int k = 0; k < 8; ++k) out64(b + 8 * i + k, h[k]);
        // presented digest/parent of record i kept for the link pass
        store8(rh + 8 * (n + i), ph);
        store8(rh + 8 * (2 * n + i), reinterpret_cast<const uint32_t*>(q + 7));
      }
      L.sync();
      if (!L.leader()) return;
      int64_t bad = -1;
      for (int64_t i = 0; i < n && bad < 0; ++i) {
        const uint32_t* pp = rh + 8 * (2 * n + i);
        if (!parity && !okv[i]) bad = i;
        if (i == 0) {
          for (int k = 0; k < 8; ++k)
            if (pp[k] != 0xffffffffu) bad = 0;
        } else {
          const uint32_t* prevh = parity ? rh + 8 * (i - 1) : rh + 8 * (n + i - 1);
          for (int k = 0; k < 8; ++k)
            if (pp[k] != prevh[k]) bad = i;
        }
      }
      out64(r + 2, bad < 0 ? 1u : 0u);
      out64(r + 3, static_cast<uint64_t>(bad));
      out64(r + 1, ST_OK);
      return;
    }
    case OP_DELTA_READ: {
      // a0 n, a1 staging offset of indices, a2 bulk offset: rows [turn, prev, ts, 8 hash words]
      if (!L.leader()) return;
      const uint64_t n = c.a[0];
      const IndexList idx = index_list(t, c, n, c.a[1]);
      uint64_t* b = reinterpret_cast<uint64_t*>(bulk + c.a[2]);
      for (uint64_t k = 0; k < n; ++k) {
        if (idx[k] < 0 || idx[k] >= t.cap.D) {
          out64(r + 1, ST_BAD_ARG);
          return;
        }
      }
      for (uint64_t k = 0; k < n; ++k) {
        const int32_t d = idx[k];
        out64(b + 12 * k + 0, static_cast<uint64_t>(static_cast<int64_t>(t.d_turn[d])));
        out64(b + 12 * k + 1, static_cast<uint64_t>(static_cast<int64_t>(t.d_prev[d])));
        out64(b + 12 * k + 2, static_cast<uint64_t>(t.d_ts[d]));
        out64(b + 12 * k + 3, static_cast<uint64_t>(static_cast<int64_t>(t.d_sess[d])));
        for (int w = 0; w < 8; ++w) out64(b + 12 * k + 4 + w, t.d_hash[8 * static_cast<int64_t>(d) + w]);
      }
      out64(r + 1, ST_OK);
      return;
    }
    default:
      if (L.leader()) out64(r + 1, ST_BAD_OP);
      break;
  }
}

// ------------------------------------------------------------- dispatch

AHV_HD bool session_drain(uint32_t op) {
  switch (op) {
    case OP_SESS_CLOSE:
    case OP_DELTA_MERKLE:
    case OP_DELTA_VERIFY:
    case OP_SESS_READ:
      return true;
    default:
      return false;
  }
}

AHV_HD bool needs_drain(uint32_t op) {
  if (op == OP_DELTA_CAPTURE) return false;
  if (op >= 40 && op < 80) return false;  // liability and saga rows: no audit state
  if (session_drain(op)) return false;
  switch (op) {
    case OP_SESS_CREATE:  // claims a FREE row: no queued capture refers to it (FREE_ROWS drained)
    case OP_SESS_JOIN:
    case OP_SESS_LEAVE:
    case OP_SESS_ACTIVATE:
    case OP_SESS_TERMINATE:
    case OP_SESS_ARCHIVE:
    case OP_SESS_UPDATE_RING:
    case OP_SESS_SET_MODE:
    case OP_SESS_SET_SIGMA:
    case OP_SESS_HANDSHAKE:
      return false;
    default:
      return true;
  }
}

// Execute one command.  All lanes of the wave call this with the same command;
// lane 0 owns the scalar logic, the SIMT sections (Merkle levels, leaf gathers,
// verify hashes) use every lane.  With `defer` set, a capture's hashing is
// handed back as a job (EXEC_DEFERRED) for the hash-engine wave; otherwise it
// is hashed in place.  Returns EXEC_STOP for OP_STOP.
AHV_HD int store_exec(const Lanes& L, const Tables& t, const Cmd& c, uint64_t seq, uint64_t* r, uint8_t* bulk,
                      HashJob* defer) {
  if (c.op == OP_DELTA_CAPTURE) {
    HashJob j;
    const bool ok = bcast(L, capture_begin(L, t, c, seq, r, j) ? 1 : 0) != 0;
    if (!ok) return EXEC_DONE;
    if (defer) {
      if (L.leader()) {
        j.mid_blocks = 0;
        *defer = j;
      }
      return EXEC_DEFERRED;
    }
    // host twin / single-wave: hash now (all lanes need the job)
    HashJob jb;
    jb.seq = bcast(L, j.seq);
    jb.s = bcast(L, j.s);
    jb.d = bcast(L, j.d);
    jb.off = bcast(L, j.off);
    jb.len = bcast(L, j.len);
    jb.hole = bcast(L, j.hole);
    jb.prev = bcast(L, j.prev);
    jb.mid_blocks = 0;
    capture_finish(L, t, jb, r);
    return EXEC_DONE;
  }
  if (c.op == OP_SESS_READ_MANY) {
    exec_read_many(L, t, c, r, bulk);
  } else if (c.op == OP_FREE_ROWS) {
    exec_free_rows(L, t, c, r);
  } else if (c.op >= 10 && c.op < 30 && c.op != OP_SESS_CLOSE) {
    exec_sess(L, t, c, r, bulk);
  } else if ((c.op >= 30 && c.op < 40) || c.op == OP_SESS_CLOSE) {
    exec_delta(L, t, c, r, bulk);
  } else if (c.op >= 40 && c.op < 60) {
    exec_vouch(L, t, c, r, bulk);
  } else if (c.op >= 60 && c.op < 80) {
    exec_saga(L, t, c, r, bulk);
  } else if (c.op == OP_STOP) {
    if (L.leader()) out64(r + 1, ST_OK);
    return EXEC_STOP;
  } else if (c.op == OP_NOP || c.op == OP_FLUSH || c.op == OP_ACQUIRE) {
    if (L.leader()) out64(r + 1, ST_OK);
  } else {
    if (L.leader()) out64(r + 1, ST_BAD_OP);
  }
  return EXEC_DONE;
}

}  // namespace store
}  // namespace ahv
