// Argument blocks of the batched governance kernels and their
// launcher / host-twin declarations.  Pointers are device pointers for the
// `launch_*` entry points and host pointers for the `*_host` twins.
#pragma once

#include <hip/hip_runtime.h>

#include "ahv/hd.h"

namespace ahv {

// K01 ring gate
struct RingGateArgs {
  int64_t n;
  const double* sigma;
  const uint8_t* consensus;  // may be null (no consensus)
  uint8_t* ring;
};
void launch_ring_gate(const RingGateArgs&, hipStream_t);
void ring_gate_host(const RingGateArgs&);

// K02 ring check
struct RingCheckArgs {
  int64_t n;
  const uint8_t* agent_ring;
  const uint8_t* action_flags;  // ActionFlag bits
  const double* sigma;
  const uint8_t* consensus;
  const uint8_t* witness;
  uint8_t* required;
  uint8_t* reason;
};
void launch_ring_check(const RingCheckArgs&, hipStream_t);
void ring_check_host(const RingCheckArgs&);

// K13 saga / step FSM
struct FsmArgs {
  int64_t n;
  int32_t kind;  // 0 step, 1 saga
  int64_t now_us;
  uint8_t* state;
  const uint8_t* target;
  uint8_t* ok;
  int64_t* started_us;    // may be null
  int64_t* completed_us;  // may be null
};
void launch_fsm(const FsmArgs&, hipStream_t);
void fsm_host(const FsmArgs&);

// K15 fan-out policy
struct FanoutArgs {
  int64_t groups;
  const int32_t* offsets;   // [groups+1] branch ranges
  const uint8_t* policy;    // [groups]
  const uint8_t* succeeded; // [branches]
  uint8_t* satisfied;       // [groups]
  int32_t* success_count;   // [groups]
  uint8_t* compensate;      // [branches]
};
void launch_fanout(const FanoutArgs&, hipStream_t);
void fanout_host(const FanoutArgs&);

// K16 breach window
// Calls are grouped by profile: group g applies calls [offsets[g], offsets[g+1])
// in order to profile rows[g] of the resident tables.  With rows/offsets null,
// group g is one call (index g) on profile g.  Per-call arrays are indexed by
// call, profile arrays by row.
struct BreachArgs {
  int64_t n;           // groups (profiles touched)
  int32_t window_cap;  // ring capacity (reference deque maxlen 1000)
  int64_t window_us;
  int64_t cooldown_us;
  const int32_t* rows;        // [n] profile row of each group, or null
  const int32_t* offsets;     // [n+1] call ranges, or null
  const int64_t* now_us;      // [calls] call timestamps
  const uint8_t* agent_ring;  // [calls] caller's current ring
  const uint8_t* new_called;  // [calls] ring being called
  int64_t* ts;                // [P, cap]
  uint8_t* called;            // [P, cap]
  int32_t* head;              // [P]
  int32_t* count;             // [P]
  int64_t* total;             // [P]
  uint8_t* tripped;           // [P]
  int64_t* tripped_at_us;     // [P]
  int64_t* ring_counts;       // [P, 4] calls per called ring, or null
  uint8_t* severity;          // [calls] out 0 none .. 4 critical
  double* rate;               // [calls] out
  int32_t* hits;              // [calls] out
  uint8_t* event;             // [calls] out 1 = BreachEvent produced
  int32_t* window;            // [calls] out windowed call count, or null
};
void launch_breach(const BreachArgs&, hipStream_t);
void breach_host(const BreachArgs&);

// K17 token bucket
// Requests grouped by bucket like BreachArgs (rows/offsets null = one request
// per bucket, index = row).
struct BucketArgs {
  int64_t n;                // groups
  int64_t now_us;
  const int32_t* rows;      // [n] or null
  const int32_t* offsets;   // [n+1] or null
  double* tokens;           // [B]
  int64_t* last_us;         // [B]
  const double* capacity;   // [B]
  const double* rate;       // [B]
  const double* cost;       // [requests]
  int64_t* total;           // [B] requests seen, or null
  int64_t* rejected;        // [B] requests refused, or null
  uint8_t* ok;              // [requests] out
};
void launch_bucket(const BucketArgs&, hipStream_t);
void bucket_host(const BucketArgs&);

// K18 expiry tick
struct ExpiryArgs {
  int64_t n;
  int64_t now_us;
  uint8_t* active;
  const int64_t* expires_us;  // < 0 = never
  int64_t* released_us;       // may be null
  uint8_t* expired;
};
void launch_expiry(const ExpiryArgs&, hipStream_t);
void expiry_host(const ExpiryArgs&);

// K22 ledger risk
struct LedgerArgs {
  int64_t agents;
  const int32_t* offsets;  // [agents+1]
  const uint8_t* type;     // LedgerType per entry
  const double* severity;
  double* raw_risk;
  double* risk;
  uint8_t* recommendation;
  int32_t* slash_count;
  int32_t* quarantine_count;
  int32_t* clean_count;
  double* fault_avg;
};
void launch_ledger(const LedgerArgs&, hipStream_t);
void ledger_host(const LedgerArgs&);

// K22 drift severity
struct DriftArgs {
  int64_t n;
  double low, medium, high, critical;
  const double* drift;
  uint8_t* severity;
};
void launch_drift(const DriftArgs&, hipStream_t);
void drift_host(const DriftArgs&);

// K21 attribution raw scores
struct AttributionArgs {
  int64_t cases;
  const int32_t* node_offsets;   // [cases+1]
  const int32_t* agent_offsets;  // [cases+1] into raw / node_count
  const int32_t* agent_of_node;  // local agent index of each node
  const uint8_t* success;
  const uint8_t* root_cause;
  const double* risk_weight;     // ω of each node's action (default 0.5)
  double* raw;
  int32_t* node_count;
};
void launch_attribution(const AttributionArgs&, hipStream_t);
void attribution_host(const AttributionArgs&);

// ---------------------------------------------------------------- liability
// Session-local vouch graphs: participants of a session have local indices
// 0..15; edges are stored per session in creation order (CSR).

constexpr int kTile = 16;

// K03 / K04 — σ_eff and exposure from dense per-session bond tiles (f64 MFMA)
struct BondTileArgs {
  int64_t sessions;
  const double* tiles;   // [S, 16, 16] live bonded amount, row = voucher, col = vouchee
  const double* sigma;   // [S, 16] vouchee σ
  const double* omega;   // [S] risk weight of the action being scored
  double* sigma_eff;     // [S, 16] out
  double* exposure;      // [S, 16] out: Σ bonded by voucher (row sums)
  double* bonded_in;     // [S, 16] out: Σ bonded for vouchee (column sums)
  // optional X01 input: add each participant's exposure into an agent-indexed
  // vector (fp64 atomics on the device; session order on the host), or null
  const int64_t* members;   // [S, 16] global agent id of each participant
  double* agent_exposure;   // [A] accumulated
};
void launch_bond_tiles(const BondTileArgs&, hipStream_t);
void bond_tiles_host(const BondTileArgs&);

// Edge-list (CSR) form: build the tiles, creation-order parity path, release.
struct VouchCsrArgs {
  int64_t sessions;
  int64_t now_us;
  const int32_t* offsets;  // [S+1]
  const uint8_t* voucher;  // [E] local index
  const uint8_t* vouchee;  // [E]
  const double* bonded;    // [E]
  uint8_t* active;         // [E]
  const int64_t* expiry_us;  // [E], < 0 = none
  int64_t* released_us;    // [E]
  double* tiles;           // [S,16,16] out (build)
  const double* sigma;     // [S,16] (sigma_eff_csr)
  const double* omega;     // [S]
  double* sigma_eff;       // [S,16] out (sigma_eff_csr)
  int32_t* released;       // [S] out (release)
};
void launch_build_tiles(const VouchCsrArgs&, hipStream_t);
void build_tiles_host(const VouchCsrArgs&);
void launch_sigma_eff_csr(const VouchCsrArgs&, hipStream_t);
void launch_sigma_eff_stream(const VouchCsrArgs&, hipStream_t);  // same results, streaming form
void sigma_eff_csr_host(const VouchCsrArgs&);
void launch_release(const VouchCsrArgs&, hipStream_t);
void release_host(const VouchCsrArgs&);

// K03/K04 fused: CSR edges → fp64 MFMA, no dense tile anywhere.  With 16
// sessions per wave, a chunk of 4 consecutive edges is one K=4 slice of
//   bonded_in[i][j] = Σ_k A[i][k]·Bin[k][j],  exposure[i][v] = Σ_k A[i][k]·Bout[k][v]
// where A[i][k] = live bond of edge k if it belongs to session i (else 0) and
// Bin/Bout are the one-hot vouchee/voucher of edge k.  σ_eff = min(σ + ω·bonded_in, 1).
struct BondFusedArgs {
  int64_t sessions;
  int64_t now_us;
  const int32_t* offsets;    // [S+1]
  const uint8_t* voucher;    // [E]
  const uint8_t* vouchee;    // [E]
  const double* bonded;      // [E]
  const uint8_t* active;     // [E]
  const int64_t* expiry_us;  // [E] or null (< 0 = none)
  const double* sigma;       // [S,16] (NaN = absent → 0)
  const double* omega;       // [S]
  double* sigma_eff;         // [S,16] out
  double* exposure;          // [S,16] out (per voucher)
  double* bonded_in;         // [S,16] out (per vouchee), or null
  const int64_t* members;    // [S,16] global agent ids, or null
  double* agent_exposure;    // [A] += exposure (fp64 atomics), with members
};
void launch_bond_fused(const BondFusedArgs&, hipStream_t);
void bond_fused_host(const BondFusedArgs&);

// K05 — admit new vouch requests (per session, in request order)
struct VouchAdmitArgs {
  int64_t sessions;
  int64_t now_us;
  double max_exposure;
  // existing edges (CSR, creation order); admitted requests are appended by
  // the caller from the `code` output (0 = admitted)
  const int32_t* e_offsets;
  const uint8_t* e_voucher;
  const uint8_t* e_vouchee;
  const double* e_bonded;
  const uint8_t* e_active;
  const int64_t* e_expiry;
  // requests (CSR per session)
  const int32_t* r_offsets;
  const uint8_t* r_voucher;
  const uint8_t* r_vouchee;
  const double* r_sigma;    // voucher σ
  const double* r_pct;      // bond pct (already defaulted)
  double* r_bonded;         // out
  uint8_t* code;            // out: 0 ok, 1 self, 2 low σ, 3 cycle, 4 exposure
};
void launch_vouch_admit(const VouchAdmitArgs&, hipStream_t);
void vouch_admit_host(const VouchAdmitArgs&);

// K06 — slash cascade (per session)
struct SlashArgs {
  int64_t sessions;
  int64_t now_us;
  const int32_t* offsets;   // edges CSR
  const uint8_t* voucher;
  const uint8_t* vouchee;
  uint8_t* active;
  const int64_t* expiry_us;
  int64_t* released_us;
  const uint8_t* target;    // [S] local index of the violator
  const double* omega;      // [S]
  double* scores;           // [S,16] in/out agent_scores (σ), NaN = absent
  int32_t* clip_offsets;    // [S] base offset of the session's clip records
  int32_t* clip_count;      // [S] out
  uint8_t* clip_voucher;    // [cap] out
  uint8_t* clip_depth;      // [cap] out
  double* clip_before;      // [cap] out
  double* clip_after;       // [cap] out
  int32_t clip_cap;         // records per session (records beyond it are dropped, not the cascade)
  uint8_t* clip_walk;       // [E] scratch: the cascade walk's (voucher | cascade<<7) per clip, uncapped —
                            // a session has at most (its edge count) clips, indexed from its first edge
  // Fused K03 (null = slash only): σ_eff of every session over its post-slash live
  // bonds, in the same pass — bit-identical to slash followed by sigma_eff_csr.
  const double* bonded;     // [E]
  double* sigma_eff;        // [S,16] out
  // Device form: 0 = split (cascade over the slashed sessions, then streaming
  // K03), 1 = one group pass per session (cascade + σ_eff), 2 = one lane per
  // session, 3 = split with one session per wave (slash_wave_kernel);
  // −1 = AHV_SLASH_FUSED / AHV_SLASH_PER_LANE / AHV_SLASH_MODE, else split.
  int32_t mode = -1;
  // Touched list (split mode; null = not wanted): the sessions with ≥ 1 clip, in
  // session order, written to `touched` [S] with their count in `touched_total`.
  int32_t* touched_tmp = nullptr;      // [S] window-local segments
  int32_t* touched_blocks = nullptr;   // [ceil(S/256)] per-window counts
  int32_t* touched_offsets = nullptr;  // [ceil(S/256)]
  int64_t* touched = nullptr;          // [S] out
  int64_t* touched_total = nullptr;    // [1] out
};
void launch_slash(const SlashArgs&, hipStream_t);
void slash_host(const SlashArgs&);

// ------------------------------------------------------------------ audit

// Payload rendering for re-hashed audit records: row r of `rows` is the template
// with decimal stamp fields (value = ids[r] mod m + add, zero-padded to the field
// width; m = 0: no modulus) and one lowercase-hex field (the `hex_bytes` bytes of
// source row ids[r]) written in place, at out + ids[r]·len.
constexpr int kRenderMaxStamps = 8;
struct RenderArgs {
  int64_t rows;
  int32_t len;
  int64_t pitch;            // bytes between rows of `out` (≥ len)
  const uint8_t* tmpl;      // [len]
  uint8_t* out;             // row ids[r] at out + ids[r]·pitch
  const int64_t* ids;       // [rows]
  int32_t nstamp;
  int32_t stamp_pos[kRenderMaxStamps];
  int32_t stamp_width[kRenderMaxStamps];
  int64_t stamp_mod[kRenderMaxStamps];
  int64_t stamp_add[kRenderMaxStamps];
  int32_t hex_pos;          // -1: none
  int32_t hex_bytes;
  const uint8_t* hex_src;   // source row ids[r] at hex_src + ids[r]·hex_stride
  int64_t hex_stride;
};
void launch_render_rows(const RenderArgs&, hipStream_t);
void render_rows_host(const RenderArgs&);

// K11 / K12 — SHA-256 of variable-length messages (offsets into a byte arena)
struct HashManyArgs {
  int64_t n;
  const uint8_t* bytes;
  const int64_t* offsets;  // [n+1]
  uint32_t* digest;        // [n, 8]
};
void launch_hash_many(const HashManyArgs&, hipStream_t);
void hash_many_host(const HashManyArgs&);

// K09 — Merkle roots of many chains of leaf digests (segmented)
struct MerkleArgs {
  int64_t chains;
  const int32_t* offsets;  // [chains+1] leaf ranges
  const uint32_t* leaves;  // [L, 8]
  uint32_t* scratch;       // [L, 8] level buffer
  uint32_t* root;          // [chains, 8] (zeros for empty chains)
  // optional fusions (null = off)
  const int64_t* leaf_idx;  // [L] leaf i of the concatenated list is leaves row leaf_idx[i] (gather fused)
  const int64_t* root_row;  // [chains] root c is written to root row root_row[c] (scatter fused)
  const int64_t* gate;      // with root_row: a zero gate[root_row[c]] writes a zero root (uncommitted)
};
void launch_merkle(const MerkleArgs&, hipStream_t);
void merkle_host(const MerkleArgs&);

// K10 — verify chains: recompute each stored delta's digest from its canonical
// payload (byte arena) and check parent links, without mutating anything.
struct VerifyArgs {
  int64_t deltas;
  int64_t chains;
  const uint8_t* bytes;
  const int64_t* offsets;       // [deltas+1] canonical payloads
  const uint32_t* stored;       // [deltas, 8] stored digests
  const uint32_t* parent;       // [deltas, 8] stored parent digests
  const uint8_t* has_parent;    // [deltas]
  const int32_t* chain_offsets; // [chains+1]
  uint8_t* delta_ok;            // [deltas] out
  uint8_t* chain_ok;            // [chains] out
};
void launch_verify(const VerifyArgs&, hipStream_t);
void verify_host(const VerifyArgs&);

// K08 — delta hash chains: digest_i = sha256(prefix_i ‖ parent_i ‖ suffix_i)
// where parent_i is the JSON text `null` for a chain's first delta (or the
// quoted hex of seed_parent when has_seed) and `"<hex of digest_{i-1}>"`
// otherwise.  Serial within a chain, one lane per chain.
struct ChainHashArgs {
  int64_t chains;
  const int32_t* chain_offsets;  // [chains+1] delta ranges
  const uint8_t* bytes;          // arena
  const int64_t* pre_off;        // [D]
  const int32_t* pre_len;        // [D]
  const int64_t* suf_off;        // [D]
  const int32_t* suf_len;        // [D]
  const uint32_t* seed_parent;   // [chains, 8] or null
  const uint8_t* has_seed;       // [chains] or null
  uint32_t* digest;              // [D, 8] out
  // K08 midstate split (null = single phase): [D, 8] scratch for the state after
  // each delta's whole prefix blocks, computed in parallel over all `deltas`.
  uint32_t* mid;
  int64_t deltas;
  // > 0: every chain has exactly this many deltas.  Phase 1 then gives a wave
  // the same turn of 64 chains (lane i → delta (i mod C)·len + i div C), so the
  // lanes of a wave hash prefixes of the same shape instead of idling behind the
  // longest turn of their chain.
  int32_t uniform_len;
  // With uniform_len > 0: chain c's span rows are sel[c]·len … sel[c]·len + len − 1
  // of the span tables (resident per-session tables, no gather), or null (rows
  // in packed order).  Digests and midstates stay in packed order.
  const int64_t* sel;
};
void launch_chain_hash(const ChainHashArgs&, hipStream_t);
void chain_hash_host(const ChainHashArgs&);

// ---------------------------------------------------------------- sessions

// K19 — vector clocks: dense clocks [paths, A] and [agents, A] (A ≤ 64, one
// component per lane of a wave).  Independent groups (sessions) run in parallel,
// one wave each; a group's operations apply in order.
struct VClockArgs {
  int64_t groups;
  int32_t A;               // clock width (agents of the session), ≤ 64
  int32_t strict;
  const int32_t* offsets;  // [groups+1] operation ranges
  const uint8_t* op;       // [n] 0 read, 1 write
  const int32_t* path;     // [n] row in path_clock
  const int32_t* agent;    // [n] row in agent_clock
  const int32_t* agent_col;  // [n] the agent's own component index
  uint32_t* path_clock;    // [P, A]
  uint32_t* agent_clock;   // [G, A]
  uint8_t* ok;             // [n] out (0 = causal violation rejected the write)
};
void vclock_host(const VClockArgs&);
void launch_vclock(const VClockArgs&, hipStream_t);

// K20 — intent-lock contention mask for requests against active locks
struct LockArgs {
  int64_t n;                  // requests
  const int32_t* res_offsets; // [R+1] active locks per resource (CSR)
  const int32_t* lock_agent;  // [L]
  const uint8_t* lock_intent; // [L] 0 read 1 write 2 exclusive
  const int32_t* req_res;     // [n]
  const int32_t* req_agent;   // [n]
  const uint8_t* req_intent;  // [n]
  int32_t* conflicts;         // [n] out: number of conflicting locks
};
void launch_locks(const LockArgs&, hipStream_t);
void locks_host(const LockArgs&);

// K20 grant pass: decide a batch of lock requests against resident
// per-resource holder tables, in request order within each resource (one lane
// per resource segment), and record the outcome in the tables.  Resource r's
// row (kLockRow int32): [0] active READ locks, [1] active WRITE/EXCLUSIVE
// locks, then kLockHolders slots of (agent, reads | writes << 16) (agent −1 =
// free).  An acquire by agent a conflicts iff another agent holds a lock it is
// incompatible with (only READ+READ coexist; an agent never conflicts with
// itself) — granted 1, refused 0, or 2 when all holder slots are taken by
// other agents (an overflow, reported instead of guessed).  A request with
// intent bit 0x80 releases one lock of that intent held by the agent instead.
constexpr int kLockHolders = 16;
constexpr int kLockRow = 2 + 2 * kLockHolders;
struct LockGrantArgs {
  int64_t segments;            // resources touched by the batch
  const int32_t* seg_offsets;  // [segments+1] into `order`
  const int32_t* order;        // [n] request indices, resource-major, request order within a resource
  const int32_t* req_res;      // [n] resource row
  const int32_t* req_agent;    // [n]
  const uint8_t* req_intent;   // [n] 0 read 1 write 2 exclusive (| 0x80: release)
  int32_t* table;              // [R, kLockRow] in/out
  uint8_t* granted;            // [n] out
};
void launch_lock_grant(const LockGrantArgs&, hipStream_t);
void lock_grant_host(const LockGrantArgs&);

// ------------------------------------------------------------------- sagas
// K13/K14 batched saga chains (args and semantics in ahv/saga_batch.h)
struct SagaBatchArgs;
void launch_saga_fused(const SagaBatchArgs&, hipStream_t);
void saga_fused_host(const SagaBatchArgs&);
void launch_saga_phase(const SagaBatchArgs&, int phase, int k, hipStream_t);
void saga_phase_host(const SagaBatchArgs&, int phase, int k);

}  // namespace ahv
