// Governance predicates and formulas, written once for host and gfx950.
//
// Each function is the element body of a batched kernel (K-ids from SURVEY
// §2.14) and is also instantiated on the host: the `*_host` entry points in
// csrc/host/py_kernels.cpp run these exact bodies on CPU so the CPU test suite
// checks device semantics against the Python reference behaviour, and the GPU
// suite checks device == host.
#pragma once

#include "ahv/hd.h"

namespace ahv {

// ------------------------------------------------------------------ rings

enum Ring : uint8_t { RING0 = 0, RING1 = 1, RING2 = 2, RING3 = 3 };

constexpr double kRing1Sigma = 0.95;
constexpr double kRing2Sigma = 0.60;

// K01 — ExecutionRing.from_sigma_eff (reference models.py:34-42): strict '>'.
AHV_HD uint8_t ring_from_sigma(double sigma, bool consensus) {
  if (consensus && sigma > kRing1Sigma) return RING1;
  if (sigma > kRing2Sigma) return RING2;
  return RING3;
}

// ActionDescriptor.required_ring (reference models.py:122-132).
// flags bit0 = is_admin, bit1 = is_read_only, bit2 = reversibility NONE.
enum ActionFlag : uint8_t { ACT_ADMIN = 1, ACT_READ_ONLY = 2, ACT_IRREVERSIBLE = 4 };

AHV_HD uint8_t required_ring(uint8_t flags) {
  if (flags & ACT_ADMIN) return RING0;
  if (flags & ACT_READ_ONLY) return RING3;
  if (flags & ACT_IRREVERSIBLE) return RING1;
  return RING2;
}

// K02 — RingEnforcer.check (reference rings/enforcer.py:44-128): non-strict '<'
// thresholds, rule order significant.  Reason codes match
// hypervisor/rings/enforcer.py REASON_*.
enum RingReason : uint8_t {
  REASON_GRANTED = 0,
  REASON_NEEDS_WITNESS = 1,
  REASON_RING1_SIGMA = 2,
  REASON_NEEDS_CONSENSUS = 3,
  REASON_RING2_SIGMA = 4,
  REASON_INSUFFICIENT = 5,
};

AHV_HD uint8_t ring_check(uint8_t agent_ring, uint8_t required, double sigma, bool consensus,
                          bool witness) {
  if (required == RING0 && !witness) return REASON_NEEDS_WITNESS;
  if (required == RING1) {
    if (sigma < kRing1Sigma) return REASON_RING1_SIGMA;
    if (!consensus) return REASON_NEEDS_CONSENSUS;
  }
  if (required == RING2 && sigma < kRing2Sigma) return REASON_RING2_SIGMA;
  if (agent_ring > required) return REASON_INSUFFICIENT;
  return REASON_GRANTED;
}

// ------------------------------------------------------- session lifecycle

enum SessState : uint8_t {
  SS_CREATED = 0,
  SS_HANDSHAKING = 1,
  SS_ACTIVE = 2,
  SS_TERMINATING = 3,
  SS_ARCHIVED = 4,
  SS_FREE = 255,  // unused table row
};

enum SessOp : uint8_t { OP_HANDSHAKE = 0, OP_ACTIVATE = 1, OP_JOIN = 2, OP_TERMINATE = 3, OP_ARCHIVE = 4 };

// Bit mask of states from which an op is allowed (reference session/__init__.py).
AHV_HD uint32_t session_op_allowed_from(uint8_t op) {
  switch (op) {
    case OP_HANDSHAKE: return 1u << SS_CREATED;
    case OP_ACTIVATE: return 1u << SS_HANDSHAKING;
    case OP_JOIN: return (1u << SS_HANDSHAKING) | (1u << SS_ACTIVE);
    case OP_TERMINATE: return (1u << SS_ACTIVE) | (1u << SS_HANDSHAKING);
    case OP_ARCHIVE: return 1u << SS_TERMINATING;
    default: return 0u;
  }
}

// Join admission codes (reference session/__init__.py:93-104).
enum JoinCode : uint8_t { JOIN_OK = 0, JOIN_BAD_STATE = 1, JOIN_DUPLICATE = 2, JOIN_FULL = 3, JOIN_LOW_SIGMA = 4 };

AHV_HD uint8_t join_check(uint8_t state, bool duplicate, int32_t active, int32_t max_participants,
                          double sigma_eff, double min_sigma, uint8_t ring) {
  if (!((session_op_allowed_from(OP_JOIN) >> state) & 1u)) return JOIN_BAD_STATE;
  if (duplicate) return JOIN_DUPLICATE;
  if (active >= max_participants) return JOIN_FULL;
  if (sigma_eff < min_sigma && ring != RING3) return JOIN_LOW_SIGMA;
  return JOIN_OK;
}

// ------------------------------------------------------------- saga FSMs

enum StepState : uint8_t {
  ST_PENDING = 0,
  ST_EXECUTING = 1,
  ST_COMMITTED = 2,
  ST_COMPENSATING = 3,
  ST_COMPENSATED = 4,
  ST_COMPENSATION_FAILED = 5,
  ST_FAILED = 6,
};

enum SagaStateCode : uint8_t { SG_RUNNING = 0, SG_COMPENSATING = 1, SG_COMPLETED = 2, SG_FAILED = 3, SG_ESCALATED = 4 };

// K13 — row = from-state, bit = allowed to-state (reference saga/state_machine.py:40-56).
AHV_HD uint32_t step_transitions(uint8_t from) {
  switch (from) {
    case ST_PENDING: return 1u << ST_EXECUTING;
    case ST_EXECUTING: return (1u << ST_COMMITTED) | (1u << ST_FAILED);
    case ST_COMMITTED: return 1u << ST_COMPENSATING;
    case ST_COMPENSATING: return (1u << ST_COMPENSATED) | (1u << ST_COMPENSATION_FAILED);
    default: return 0u;
  }
}

AHV_HD uint32_t saga_transitions(uint8_t from) {
  switch (from) {
    case SG_RUNNING: return (1u << SG_COMPENSATING) | (1u << SG_COMPLETED) | (1u << SG_FAILED);
    case SG_COMPENSATING: return (1u << SG_COMPLETED) | (1u << SG_FAILED) | (1u << SG_ESCALATED);
    default: return 0u;
  }
}

AHV_HD bool step_stamps_completed(uint8_t s) {
  return s == ST_COMMITTED || s == ST_COMPENSATED || s == ST_COMPENSATION_FAILED || s == ST_FAILED;
}

AHV_HD bool saga_terminal(uint8_t s) { return s == SG_COMPLETED || s == SG_FAILED || s == SG_ESCALATED; }

// K15 — FanOutGroup.check_policy (reference saga/fan_out.py:62-70).
enum FanOutPolicyCode : uint8_t { POL_ALL = 0, POL_MAJORITY = 1, POL_ANY = 2 };

AHV_HD bool fanout_policy_ok(uint8_t policy, int32_t success, int32_t total) {
  switch (policy) {
    case POL_ALL: return success == total;
    case POL_MAJORITY: return static_cast<double>(success) > static_cast<double>(total) / 2.0;
    case POL_ANY: return success >= 1;
    default: return false;
  }
}

// ------------------------------------------------------------- liability

constexpr double kSigmaFloor = 0.05;
constexpr double kCascadeBelow = kSigmaFloor + 0.01;
constexpr int kMaxCascadeDepth = 2;
constexpr double kMinVoucherSigma = 0.50;

// K06 element — one collateral clip (reference liability/slashing.py:96-98).
AHV_HD double clip_sigma(double sigma, double omega) {
  const double s = sigma * (1.0 - omega);
  return s > kSigmaFloor ? s : kSigmaFloor;
}

// K03 element — min(σ + ω·Σbonded, 1) (reference liability/vouching.py:128-151).
AHV_HD double sigma_eff_combine(double sigma, double omega, double bonded_sum) {
  const double s = sigma + omega * bonded_sum;
  return s < 1.0 ? s : 1.0;
}

// K22 — ledger risk increment (reference liability/ledger.py:124-136).
enum LedgerType : uint8_t {
  LG_VOUCH_GIVEN = 0,
  LG_VOUCH_RECEIVED = 1,
  LG_VOUCH_RELEASED = 2,
  LG_SLASH_RECEIVED = 3,
  LG_SLASH_CASCADED = 4,
  LG_QUARANTINE_ENTERED = 5,
  LG_QUARANTINE_RELEASED = 6,
  LG_FAULT_ATTRIBUTED = 7,
  LG_CLEAN_SESSION = 8,
};

AHV_HD double ledger_increment(uint8_t type, double sev) {
  switch (type) {
    case LG_SLASH_RECEIVED:
    case LG_SLASH_CASCADED: return 0.15 * (sev > 0.5 ? sev : 0.5);
    case LG_QUARANTINE_ENTERED: return 0.10 * (sev > 0.3 ? sev : 0.3);
    case LG_FAULT_ATTRIBUTED: return 0.05 * sev;
    case LG_CLEAN_SESSION: return -0.05;
    default: return 0.0;
  }
}

// recommendation: 0 admit, 1 probation, 2 deny
AHV_HD uint8_t ledger_recommendation(double risk) {
  if (risk >= 0.6) return 2;
  if (risk >= 0.3) return 1;
  return 0;
}

// K22 — CMVK drift severity (reference integrations/cmvk_adapter.py:240-250).
// 0 none, 1 low, 2 medium, 3 high, 4 critical.
AHV_HD uint8_t drift_severity(double d, double low, double medium, double high, double critical) {
  if (d >= critical) return 4;
  if (d >= high) return 3;
  if (d >= medium) return 2;
  if (d >= low) return 1;
  return 0;
}

// K16 — breach severity of an anomaly rate (reference rings/breach_detector.py:137-147).
AHV_HD uint8_t breach_severity(double rate) { return drift_severity(rate, 0.3, 0.5, 0.7, 0.9); }

// K17 — token bucket refill+consume (reference security/rate_limiter.py:30-43).
// Returns 1 if consumed.  `tokens`/`last_us` are updated in place.
AHV_HD uint8_t token_bucket_consume(double& tokens, int64_t& last_us, double capacity, double rate,
                                    int64_t now_us, double cost) {
  const double dt = static_cast<double>(now_us - last_us) / 1e6;
  double t = tokens + dt * rate;
  tokens = t < capacity ? t : capacity;
  last_us = now_us;
  if (tokens >= cost) {
    tokens -= cost;
    return 1;
  }
  return 0;
}

// ------------------------------------------------------------------- ids

// splitmix64: counter-based generator for device-minted ids (session/saga/step
// uuid4).  Host twin produces identical ids for the same (seed, counter).
AHV_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// 16 uuid4 bytes as 4 big-endian words (version 4, RFC-4122 variant).
AHV_HD void uuid4_words(uint64_t seed, uint64_t counter, uint32_t out[4]) {
  uint64_t hi = splitmix64(seed ^ splitmix64(2 * counter));
  uint64_t lo = splitmix64(seed ^ splitmix64(2 * counter + 1));
  hi = (hi & 0xffffffffffff0fffull) | 0x0000000000004000ull;
  lo = (lo & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  out[0] = static_cast<uint32_t>(hi >> 32);
  out[1] = static_cast<uint32_t>(hi);
  out[2] = static_cast<uint32_t>(lo >> 32);
  out[3] = static_cast<uint32_t>(lo);
}

}  // namespace ahv
