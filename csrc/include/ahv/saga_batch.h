// Batched saga execution with compensation (BASELINE
// config 4): one lane per saga, K ≤ 64 steps per saga, the reference
// orchestrator's semantics (saga/orchestrator.py:61-198):
//
//   execute step k:   attempts = 1 + max_retries; each attempt PENDING→EXECUTING,
//                     then COMMITTED, or FAILED (and back to PENDING while
//                     attempts remain); retry_count = index of the last attempt
//   first step that exhausts its attempts stops the forward pass
//   all committed    → saga COMPLETED
//   otherwise        → saga COMPENSATING; committed steps in reverse order:
//                     no Undo_API → COMPENSATION_FAILED ("No Undo_API available")
//                     else COMPENSATING → COMPENSATED | COMPENSATION_FAILED
//                     → saga ESCALATED if any compensation failed, else COMPLETED
//                     (or saga FAILED without compensation when disabled)
//
// Executor / compensator outcomes are inputs (device tables written by the
// caller or a synthetic generator): fail_attempts[k] = failing attempts before
// success (255 = never succeeds), fail_kind = 1 exception / 2 timeout, and
// comp_fail = 0 ok / 1 exception / 2 timeout.  Every transition stamps
// now_us + tick (tick = per-saga transition counter), so timestamps are
// strictly ordered within a saga and reproducible.
//
// The same element functions serve the fused kernel (whole chain per lane) and
// the per-step kernels that a hipGraph replays as the orchestrator's step loop.
#pragma once

#include "ahv/hd.h"
#include "ahv/semantics.h"

namespace ahv {

constexpr int kMaxSagaSteps = 64;

enum SagaErr : uint8_t {
  SE_NONE = 0,
  SE_EXEC_FAILED = 1,
  SE_EXEC_TIMEOUT = 2,
  SE_NO_UNDO = 3,
  SE_COMP_FAILED = 4,
  SE_COMP_TIMEOUT = 5,
};

struct SagaBatchArgs {
  int64_t sagas;
  int32_t steps;         // K
  int32_t compensate;    // compensate on failure (else saga → FAILED)
  int64_t now_us;
  // inputs [K, S] (step-major, see saga_elem)
  const uint8_t* fail_attempts;
  const uint8_t* fail_kind;
  const uint8_t* comp_fail;
  const uint8_t* has_undo;
  const uint8_t* max_retries;
  // state [K, S]
  uint8_t* step_state;
  uint8_t* retry_count;
  uint8_t* step_error;
  int64_t* started_us;
  int64_t* completed_us;
  // state [S]
  uint8_t* saga_state;
  int64_t* saga_completed_us;
  int32_t* failed_step;   // -1 = none yet
  int32_t* comp_failed;   // compensation failures
  int32_t* tick;          // transition counter (per-step mode keeps it across launches)
  unsigned long long* stats;  // [4] completed, escalated, failed, compensated steps (or null)
  // Device-resident time base (int64[1]) or null: when set it overrides now_us, so
  // a captured step-loop graph stamps each replay with the time written before it.
  const int64_t* now_dev;
};

AHV_HD SagaBatchArgs saga_with_now(SagaBatchArgs a) {
  if (a.now_dev) a.now_us = *a.now_dev;
  return a;
}

// Per-step tables are step-major, [K][S]: lane s of a wave touches element
// k*S + s, so every per-step access of a wave is one contiguous (coalesced)
// segment instead of a stride-K gather.
AHV_HD int64_t saga_elem(const SagaBatchArgs& a, int64_t s, int k) {
  return static_cast<int64_t>(k) * a.sagas + s;
}

AHV_HD void saga_init(const SagaBatchArgs& a, int64_t s) {
  for (int k = 0; k < a.steps; ++k) {
    const int64_t e = saga_elem(a, s, k);
    a.step_state[e] = ST_PENDING;
    a.retry_count[e] = 0;
    a.step_error[e] = SE_NONE;
    a.started_us[e] = 0;
    a.completed_us[e] = 0;
  }
  a.saga_state[s] = SG_RUNNING;
  a.saga_completed_us[s] = 0;
  a.failed_step[s] = -1;
  a.comp_failed[s] = 0;
  a.tick[s] = 0;
}

// Forward pass for step k (no-op once the saga has stopped).
AHV_HD void saga_exec_step(const SagaBatchArgs& a, int64_t s, int k, int32_t& tick) {
  if (a.saga_state[s] != SG_RUNNING || a.failed_step[s] >= 0) return;
  const int64_t e = saga_elem(a, s, k);
  const int attempts = 1 + a.max_retries[e];
  const int fails = a.fail_attempts[e];
  uint8_t st = a.step_state[e];
  for (int at = 0; at < attempts; ++at) {
    a.retry_count[e] = static_cast<uint8_t>(at);
    st = ST_EXECUTING;
    a.started_us[e] = a.now_us + (tick++);
    if (fails == 255 || at < fails) {
      st = ST_FAILED;
      a.completed_us[e] = a.now_us + (tick++);
      a.step_error[e] = a.fail_kind[e] == 2 ? SE_EXEC_TIMEOUT : SE_EXEC_FAILED;
      if (at < attempts - 1) {
        st = ST_PENDING;
        a.step_error[e] = SE_NONE;
      }
    } else {
      st = ST_COMMITTED;
      a.completed_us[e] = a.now_us + (tick++);
      break;
    }
  }
  a.step_state[e] = st;
  if (st == ST_FAILED) a.failed_step[s] = k;
}

// After the forward pass: COMPLETED, or enter compensation / FAILED.
AHV_HD void saga_decide(const SagaBatchArgs& a, int64_t s, int32_t& tick) {
  if (a.saga_state[s] != SG_RUNNING) return;
  if (a.failed_step[s] < 0) {
    a.saga_state[s] = SG_COMPLETED;
    a.saga_completed_us[s] = a.now_us + (tick++);
  } else if (a.compensate) {
    a.saga_state[s] = SG_COMPENSATING;
  } else {
    a.saga_state[s] = SG_FAILED;
    a.saga_completed_us[s] = a.now_us + (tick++);
  }
}

// Compensation of step k (called for k = K-1 … 0).
AHV_HD void saga_comp_step(const SagaBatchArgs& a, int64_t s, int k, int32_t& tick) {
  if (a.saga_state[s] != SG_COMPENSATING) return;
  const int64_t e = saga_elem(a, s, k);
  if (a.step_state[e] != ST_COMMITTED) return;
  if (!a.has_undo[e]) {
    a.step_state[e] = ST_COMPENSATION_FAILED;  // direct assignment, no completion stamp (reference)
    a.step_error[e] = SE_NO_UNDO;
    a.comp_failed[s] += 1;
    return;
  }
  const uint8_t cf = a.comp_fail[e];
  if (cf == 0) {
    a.step_state[e] = ST_COMPENSATED;
  } else {
    a.step_state[e] = ST_COMPENSATION_FAILED;
    a.step_error[e] = cf == 2 ? SE_COMP_TIMEOUT : SE_COMP_FAILED;
    a.comp_failed[s] += 1;
  }
  a.completed_us[e] = a.now_us + (tick++);
}

AHV_HD void saga_finish(const SagaBatchArgs& a, int64_t s, int32_t& tick) {
  if (a.saga_state[s] != SG_COMPENSATING) return;
  a.saga_state[s] = a.comp_failed[s] > 0 ? SG_ESCALATED : SG_COMPLETED;
  a.saga_completed_us[s] = a.now_us + (tick++);
}

struct SagaCounters {
  uint32_t completed, escalated, failed, compensated;
};

AHV_HD SagaCounters saga_counters(const SagaBatchArgs& a, int64_t s) {
  SagaCounters c{0, 0, 0, 0};
  const uint8_t g = a.saga_state[s];
  c.completed = g == SG_COMPLETED;
  c.escalated = g == SG_ESCALATED;
  c.failed = g == SG_FAILED;
  for (int k = 0; k < a.steps; ++k) c.compensated += a.step_state[saga_elem(a, s, k)] == ST_COMPENSATED;
  return c;
}

// Register-resident whole chain for a compile-time step count: the outcome
// tables are read once and every state column is written once (all coalesced,
// step-major), with the whole per-saga state machine in registers in between.
// Produces exactly what saga_run_chain produces.
template <int K>
AHV_HD SagaCounters saga_run_chain_regs(const SagaBatchArgs& a, int64_t s) {
  uint8_t st[K], rc[K], er[K];
  int64_t t0[K], t1[K];
  uint8_t fa[K], fk[K], cf[K], hu[K], mr[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t e = saga_elem(a, s, k);
    fa[k] = a.fail_attempts[e];
    fk[k] = a.fail_kind[e];
    cf[k] = a.comp_fail[e];
    hu[k] = a.has_undo[e];
    mr[k] = a.max_retries[e];
    st[k] = ST_PENDING;
    rc[k] = 0;
    er[k] = SE_NONE;
    t0[k] = 0;
    t1[k] = 0;
  }
  const int64_t now = a.now_us;
  int32_t tick = 0, failed = -1, compf = 0;
  uint8_t g = SG_RUNNING;
  int64_t gdone = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (failed < 0) {
      const int attempts = 1 + mr[k];
      const int fails = fa[k];
      for (int at = 0; at < attempts; ++at) {
        rc[k] = static_cast<uint8_t>(at);
        t0[k] = now + (tick++);
        t1[k] = now + (tick++);
        if (fails == 255 || at < fails) {
          st[k] = ST_FAILED;
          er[k] = fk[k] == 2 ? SE_EXEC_TIMEOUT : SE_EXEC_FAILED;
          if (at < attempts - 1) {
            st[k] = ST_PENDING;
            er[k] = SE_NONE;
          }
        } else {
          st[k] = ST_COMMITTED;
          break;
        }
      }
      if (st[k] == ST_FAILED) failed = k;
    }
  }
  if (failed < 0) {
    g = SG_COMPLETED;
    gdone = now + (tick++);
  } else if (a.compensate) {
    g = SG_COMPENSATING;
  } else {
    g = SG_FAILED;
    gdone = now + (tick++);
  }
  if (g == SG_COMPENSATING) {
#pragma unroll
    for (int k = K - 1; k >= 0; --k) {
      if (st[k] != ST_COMMITTED) continue;
      if (!hu[k]) {
        st[k] = ST_COMPENSATION_FAILED;
        er[k] = SE_NO_UNDO;
        ++compf;
        continue;
      }
      if (cf[k] == 0) {
        st[k] = ST_COMPENSATED;
      } else {
        st[k] = ST_COMPENSATION_FAILED;
        er[k] = cf[k] == 2 ? SE_COMP_TIMEOUT : SE_COMP_FAILED;
        ++compf;
      }
      t1[k] = now + (tick++);
    }
    g = compf > 0 ? SG_ESCALATED : SG_COMPLETED;
    gdone = now + (tick++);
  }
  SagaCounters c{g == SG_COMPLETED, g == SG_ESCALATED, g == SG_FAILED, 0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int64_t e = saga_elem(a, s, k);
    a.step_state[e] = st[k];
    a.retry_count[e] = rc[k];
    a.step_error[e] = er[k];
    a.started_us[e] = t0[k];
    a.completed_us[e] = t1[k];
    c.compensated += st[k] == ST_COMPENSATED;
  }
  a.saga_state[s] = g;
  a.saga_completed_us[s] = gdone;
  a.failed_step[s] = failed;
  a.comp_failed[s] = compf;
  a.tick[s] = tick;
  return c;
}

constexpr int kMaxRegSagaSteps = 16;

#define AHV_SAGA_REG_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

// Whole chain for one saga (fused path).
AHV_HD SagaCounters saga_run_chain(const SagaBatchArgs& a, int64_t s) {
  saga_init(a, s);
  int32_t tick = 0;
  for (int k = 0; k < a.steps; ++k) saga_exec_step(a, s, k, tick);
  saga_decide(a, s, tick);
  for (int k = a.steps - 1; k >= 0; --k) saga_comp_step(a, s, k, tick);
  saga_finish(a, s, tick);
  a.tick[s] = tick;
  return saga_counters(a, s);
}

// Fused chain: register-resident for K ≤ 16, generic (global-memory state) beyond.
AHV_HD SagaCounters saga_run_chain_fused(const SagaBatchArgs& a, int64_t s) {
  switch (a.steps) {
#define AHV_SAGA_CASE(K) \
  case K:                \
    return saga_run_chain_regs<K>(a, s);
    AHV_SAGA_REG_CASES(AHV_SAGA_CASE)
#undef AHV_SAGA_CASE
    default:
      return saga_run_chain(a, s);
  }
}

}  // namespace ahv
