// Batched governance predicates: ring gate K01, ring check K02,
// saga FSM K13, fan-out policy K15, breach window K16, token bucket K17,
// expiry tick K18, ledger risk + drift classification K22, fault attribution K21.
//
// Every kernel is a thin grid-stride loop around an element body from
// ahv/semantics.h; the `*_host` twin runs the same body on the CPU.  These are
// memory-bound streaming kernels: 256-thread workgroups, one element per lane
// per iteration, grid sized to ≥ 4 waves per SIMD of the 256 CUs.
#include "ahv/kernels.h"
#include "ahv/launch.h"
#include "ahv/semantics.h"

namespace ahv {

namespace {
constexpr int kBlock = 256;

inline dim3 grid_for(int64_t n) {
  const int64_t want = (n + kBlock - 1) / kBlock;
  const int64_t cap = 256 * 16;  // 16 workgroups per CU is plenty for streaming
  return dim3(static_cast<uint32_t>(want < cap ? (want > 0 ? want : 1) : cap));
}

#define AHV_GRID_STRIDE(i, n) \
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < (n); \
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
}  // namespace

// ------------------------------------------------------------------ K01

AHV_HD void ring_gate_elem(const RingGateArgs& a, int64_t i) {
  a.ring[i] = ring_from_sigma(a.sigma[i], a.consensus ? a.consensus[i] != 0 : false);
}
__global__ void ring_gate_kernel(RingGateArgs a) { AHV_GRID_STRIDE(i, a.n) ring_gate_elem(a, i); }
void launch_ring_gate(const RingGateArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(ring_gate_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "ring_gate_kernel");
}
void ring_gate_host(const RingGateArgs& a) { for (int64_t i = 0; i < a.n; ++i) ring_gate_elem(a, i); }

// ------------------------------------------------------------------ K02

AHV_HD void ring_check_elem(const RingCheckArgs& a, int64_t i) {
  const uint8_t req = required_ring(a.action_flags[i]);
  a.required[i] = req;
  a.reason[i] = ring_check(a.agent_ring[i], req, a.sigma[i], a.consensus[i] != 0, a.witness[i] != 0);
}
__global__ void ring_check_kernel(RingCheckArgs a) { AHV_GRID_STRIDE(i, a.n) ring_check_elem(a, i); }
void launch_ring_check(const RingCheckArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(ring_check_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "ring_check_kernel");
}
void ring_check_host(const RingCheckArgs& a) { for (int64_t i = 0; i < a.n; ++i) ring_check_elem(a, i); }

// ------------------------------------------------------------------ K13
// Apply requested transitions where valid.  `kind` 0 = step FSM, 1 = saga FSM.
// ok[i] = 1 if applied; timestamps stamped per the reference rules.

AHV_HD void fsm_elem(const FsmArgs& a, int64_t i) {
  const uint8_t from = a.state[i];
  const uint8_t to = a.target[i];
  const uint32_t mask = a.kind == 0 ? step_transitions(from) : saga_transitions(from);
  const bool ok = to < 8 && ((mask >> to) & 1u);
  a.ok[i] = ok ? 1 : 0;
  if (!ok) return;
  a.state[i] = to;
  if (a.kind == 0) {
    if (to == ST_EXECUTING && a.started_us) a.started_us[i] = a.now_us;
    else if (step_stamps_completed(to) && a.completed_us) a.completed_us[i] = a.now_us;
  } else if (saga_terminal(to) && a.completed_us) {
    a.completed_us[i] = a.now_us;
  }
}
__global__ void fsm_kernel(FsmArgs a) { AHV_GRID_STRIDE(i, a.n) fsm_elem(a, i); }
void launch_fsm(const FsmArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(fsm_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "fsm_kernel");
}
void fsm_host(const FsmArgs& a) { for (int64_t i = 0; i < a.n; ++i) fsm_elem(a, i); }

// ------------------------------------------------------------------ K15
// One lane per fan-out group: count succeeded branches, evaluate the policy,
// mark succeeded branches for compensation when the policy failed.

AHV_HD void fanout_elem(const FanoutArgs& a, int64_t g) {
  const int32_t b0 = a.offsets[g], b1 = a.offsets[g + 1];
  int32_t ok = 0;
  for (int32_t b = b0; b < b1; ++b) ok += a.succeeded[b] ? 1 : 0;
  const bool sat = fanout_policy_ok(a.policy[g], ok, b1 - b0);
  a.satisfied[g] = sat ? 1 : 0;
  a.success_count[g] = ok;
  for (int32_t b = b0; b < b1; ++b) a.compensate[b] = (!sat && a.succeeded[b]) ? 1 : 0;
}
__global__ void fanout_kernel(FanoutArgs a) { AHV_GRID_STRIDE(g, a.groups) fanout_elem(a, g); }
void launch_fanout(const FanoutArgs& a, hipStream_t s) {
  if (a.groups <= 0) return;
  hipLaunchKernelGGL(fanout_kernel, grid_for(a.groups), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "fanout_kernel");
}
void fanout_host(const FanoutArgs& a) { for (int64_t g = 0; g < a.groups; ++g) fanout_elem(a, g); }

// ------------------------------------------------------------------ K16
// One lane per (agent, session) call profile: append the new call to the
// ring-buffer window, prune entries older than the window, honour the breaker
// cooldown, then score the windowed calls against the *current* agent ring.

AHV_HD void breach_call(const BreachArgs& a, int64_t p, int64_t c) {
  const int64_t now = a.now_us[c];
  const int32_t W = a.window_cap;
  int64_t* ts = a.ts + p * W;
  uint8_t* called = a.called + p * W;
  int32_t head = a.head[p];   // index of the oldest live entry
  int32_t count = a.count[p];
  // append (deque maxlen semantics: drop the oldest when full)
  if (count == W) { head = (head + 1) % W; --count; }
  const int32_t slot = (head + count) % W;
  const uint8_t nc = a.new_called[c];
  ts[slot] = now;
  called[slot] = nc;
  ++count;
  a.total[p] += 1;
  if (a.ring_counts != nullptr && nc < 4) a.ring_counts[p * 4 + nc] += 1;
  // prune calls older than the window
  const int64_t cutoff = now - a.window_us;
  while (count > 0 && ts[head] < cutoff) { head = (head + 1) % W; --count; }
  a.head[p] = head;
  a.count[p] = count;
  a.severity[c] = 0;
  a.rate[c] = 0.0;
  a.event[c] = 0;
  if (a.window != nullptr) a.window[c] = count;
  // breaker cooldown suppresses analysis
  if (a.tripped[p] && a.tripped_at_us[p] != 0 && now < a.tripped_at_us[p] + a.cooldown_us) return;
  if (count < 5) return;
  const uint8_t ring = a.agent_ring[c];
  int32_t hits = 0;
  for (int32_t k = 0; k < count; ++k) hits += called[(head + k) % W] < ring ? 1 : 0;
  const double rate = static_cast<double>(hits) / static_cast<double>(count);
  const uint8_t sev = breach_severity(rate);
  a.rate[c] = rate;
  a.severity[c] = sev;
  a.hits[c] = hits;
  if (sev == 0) return;
  a.event[c] = 1;
  if (sev >= 3) {
    a.tripped[p] = 1;
    a.tripped_at_us[p] = now;
  }
}
AHV_HD void breach_elem(const BreachArgs& a, int64_t g) {
  const int64_t p = a.rows != nullptr ? a.rows[g] : g;
  const int64_t c0 = a.offsets != nullptr ? a.offsets[g] : g;
  const int64_t c1 = a.offsets != nullptr ? a.offsets[g + 1] : g + 1;
  for (int64_t c = c0; c < c1; ++c) breach_call(a, p, c);
}
__global__ void breach_kernel(BreachArgs a) { AHV_GRID_STRIDE(p, a.n) breach_elem(a, p); }
void launch_breach(const BreachArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(breach_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "breach_kernel");
}
void breach_host(const BreachArgs& a) { for (int64_t p = 0; p < a.n; ++p) breach_elem(a, p); }

// ------------------------------------------------------------------ K17

AHV_HD void bucket_elem(const BucketArgs& a, int64_t g) {
  const int64_t b = a.rows != nullptr ? a.rows[g] : g;
  const int64_t c0 = a.offsets != nullptr ? a.offsets[g] : g;
  const int64_t c1 = a.offsets != nullptr ? a.offsets[g + 1] : g + 1;
  for (int64_t c = c0; c < c1; ++c) {
    const uint8_t ok = token_bucket_consume(a.tokens[b], a.last_us[b], a.capacity[b], a.rate[b], a.now_us, a.cost[c]);
    a.ok[c] = ok;
    if (a.total != nullptr) a.total[b] += 1;
    if (a.rejected != nullptr && !ok) a.rejected[b] += 1;
  }
}
__global__ void bucket_kernel(BucketArgs a) { AHV_GRID_STRIDE(i, a.n) bucket_elem(a, i); }
void launch_bucket(const BucketArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(bucket_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "bucket_kernel");
}
void bucket_host(const BucketArgs& a) { for (int64_t i = 0; i < a.n; ++i) bucket_elem(a, i); }

// ------------------------------------------------------------------ K18
// Elevation / quarantine / vouch expiry: deactivate live records whose expiry
// (strictly) precedes now; expired[i] = 1 for records deactivated by this tick.

AHV_HD void expiry_elem(const ExpiryArgs& a, int64_t i) {
  const bool hit = a.active[i] && a.expires_us[i] >= 0 && a.now_us > a.expires_us[i];
  a.expired[i] = hit ? 1 : 0;
  if (hit) {
    a.active[i] = 0;
    if (a.released_us) a.released_us[i] = a.now_us;
  }
}
__global__ void expiry_kernel(ExpiryArgs a) { AHV_GRID_STRIDE(i, a.n) expiry_elem(a, i); }
void launch_expiry(const ExpiryArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(expiry_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "expiry_kernel");
}
void expiry_host(const ExpiryArgs& a) { for (int64_t i = 0; i < a.n; ++i) expiry_elem(a, i); }

// ------------------------------------------------------------------ K22
// Ledger: one lane per agent over its entries (agent-segmented, entry order).
// Drift: elementwise severity buckets.

AHV_HD void ledger_elem(const LedgerArgs& a, int64_t g) {
  double risk = 0.0, fault_sum = 0.0;
  int32_t slashes = 0, quars = 0, cleans = 0, faults = 0;
  for (int32_t e = a.offsets[g]; e < a.offsets[g + 1]; ++e) {
    const uint8_t t = a.type[e];
    const double sev = a.severity[e];
    if (t == LG_SLASH_RECEIVED || t == LG_SLASH_CASCADED) ++slashes;
    else if (t == LG_QUARANTINE_ENTERED) ++quars;
    else if (t == LG_FAULT_ATTRIBUTED) { ++faults; fault_sum += sev; }
    else if (t == LG_CLEAN_SESSION) ++cleans;
    risk += ledger_increment(t, sev);
  }
  a.raw_risk[g] = risk;
  const double clamped = risk < 0.0 ? 0.0 : (risk > 1.0 ? 1.0 : risk);
  a.risk[g] = clamped;
  a.recommendation[g] = ledger_recommendation(clamped);
  a.slash_count[g] = slashes;
  a.quarantine_count[g] = quars;
  a.clean_count[g] = cleans;
  a.fault_avg[g] = faults ? fault_sum / faults : 0.0;
}
__global__ void ledger_kernel(LedgerArgs a) { AHV_GRID_STRIDE(g, a.agents) ledger_elem(a, g); }
void launch_ledger(const LedgerArgs& a, hipStream_t s) {
  if (a.agents <= 0) return;
  hipLaunchKernelGGL(ledger_kernel, grid_for(a.agents), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "ledger_kernel");
}
void ledger_host(const LedgerArgs& a) { for (int64_t g = 0; g < a.agents; ++g) ledger_elem(a, g); }

AHV_HD void drift_elem(const DriftArgs& a, int64_t i) {
  a.severity[i] = drift_severity(a.drift[i], a.low, a.medium, a.high, a.critical);
}
__global__ void drift_kernel(DriftArgs a) { AHV_GRID_STRIDE(i, a.n) drift_elem(a, i); }
void launch_drift(const DriftArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(drift_kernel, grid_for(a.n), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "drift_kernel");
}
void drift_host(const DriftArgs& a) { for (int64_t i = 0; i < a.n; ++i) drift_elem(a, i); }

// ------------------------------------------------------------------ K21
// Fault attribution: one lane per failure case; nodes segmented per case and
// grouped by agent (agent_of_node = local agent index < 64).  Produces the raw
// per-agent scores in node order; normalisation and round(x, 4) stay on the host
// (CPython's correctly-rounded decimal rounding).

AHV_HD void attribution_elem(const AttributionArgs& a, int64_t c) {
  const int32_t n0 = a.node_offsets[c], n1 = a.node_offsets[c + 1];
  const int32_t g0 = a.agent_offsets[c], g1 = a.agent_offsets[c + 1];
  int32_t enabling = 0;
  for (int32_t n = n0; n < n1; ++n) enabling += (!a.success[n] && !a.root_cause[n]) ? 1 : 0;
  if (enabling < 1) enabling = 1;
  for (int32_t g = g0; g < g1; ++g) a.raw[g] = 0.0;
  // node count per agent
  for (int32_t g = g0; g < g1; ++g) a.node_count[g] = 0;
  for (int32_t n = n0; n < n1; ++n) a.node_count[g0 + a.agent_of_node[n]] += 1;
  for (int32_t n = n0; n < n1; ++n) {
    const int32_t g = g0 + a.agent_of_node[n];
    double s = a.raw[g];
    if (a.root_cause[n]) s += 0.5;
    if (!a.success[n] && !a.root_cause[n]) s += 0.3 / enabling;
    const int32_t cnt = a.node_count[g] > 1 ? a.node_count[g] : 1;
    s += 0.2 * a.risk_weight[n] / cnt;
    a.raw[g] = s;
  }
}
__global__ void attribution_kernel(AttributionArgs a) { AHV_GRID_STRIDE(c, a.cases) attribution_elem(a, c); }
void launch_attribution(const AttributionArgs& a, hipStream_t s) {
  if (a.cases <= 0) return;
  hipLaunchKernelGGL(attribution_kernel, grid_for(a.cases), dim3(kBlock), 0, s, a);
  check_hip(hipGetLastError(), "attribution_kernel");
}
void attribution_host(const AttributionArgs& a) { for (int64_t c = 0; c < a.cases; ++c) attribution_elem(a, c); }

}  // namespace ahv
