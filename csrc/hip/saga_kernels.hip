// Batched saga chains (BASELINE config 4): fused whole-chain kernel and the
// per-step kernels a hipGraph replays as the orchestrator's step loop.
// Semantics: ahv/saga_batch.h.
#include "ahv/launch.h"
#include "ahv/saga_batch.h"

namespace ahv {

void launch_saga_fused(const SagaBatchArgs& a, hipStream_t s);
void saga_fused_host(const SagaBatchArgs& a);
void launch_saga_phase(const SagaBatchArgs& a, int phase, int k, hipStream_t s);
void saga_phase_host(const SagaBatchArgs& a, int phase, int k);

namespace {
constexpr int kBlock = 256;
inline dim3 grid_for(int64_t n) {
  const int64_t b = (n + kBlock - 1) / kBlock;
  return dim3(static_cast<uint32_t>(b > 0 ? b : 1));
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ void add_counters(const SagaBatchArgs& a, SagaCounters c, bool active) {
  if (!a.stats) return;
  const uint32_t v[4] = {active ? c.completed : 0u, active ? c.escalated : 0u, active ? c.failed : 0u,
                         active ? c.compensated : 0u};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t s = wave_sum(v[k]);
    if ((threadIdx.x & 63) == 0 && s)
      atomicAdd(a.stats + ((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) % kStatSpread) * 4 + k,
                static_cast<unsigned long long>(s));
  }
}
}  // namespace

__global__ __launch_bounds__(kBlock) void saga_fused_kernel(SagaBatchArgs a0) {
  const SagaBatchArgs a = saga_with_now(a0);
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool active = s < a.sagas;
  SagaCounters c{0, 0, 0, 0};
  if (active) c = saga_run_chain(a, s);
  add_counters(a, c, active);
}

// One instantiation per step count: the chain's state lives in registers.
template <int K>
__global__ __launch_bounds__(kBlock) void saga_fused_regs_kernel(SagaBatchArgs a0) {
  const SagaBatchArgs a = saga_with_now(a0);
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool active = s < a.sagas;
  SagaCounters c{0, 0, 0, 0};
  if (active) c = saga_run_chain_regs<K>(a, s);
  add_counters(a, c, active);
}

// phase 0 init, 1 execute step k, 2 decide, 3 compensate step k, 4 finish (+counters)
__global__ __launch_bounds__(kBlock) void saga_phase_kernel(SagaBatchArgs a0, int phase, int k) {
  const SagaBatchArgs a = saga_with_now(a0);
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool active = s < a.sagas;
  SagaCounters c{0, 0, 0, 0};
  if (active) {
    if (phase == 0) {
      saga_init(a, s);
    } else {
      int32_t tick = a.tick[s];
      if (phase == 1) saga_exec_step(a, s, k, tick);
      else if (phase == 2) saga_decide(a, s, tick);
      else if (phase == 3) saga_comp_step(a, s, k, tick);
      else saga_finish(a, s, tick);
      a.tick[s] = tick;
      if (phase == 4) c = saga_counters(a, s);
    }
  }
  if (phase == 4) add_counters(a, c, active);
}

static void check_args(const SagaBatchArgs& a) {
  if (a.steps < 1 || a.steps > kMaxSagaSteps) throw std::invalid_argument("saga steps must be in [1, 64]");
}

void launch_saga_fused(const SagaBatchArgs& a, hipStream_t st) {
  check_args(a);
  if (a.sagas <= 0) return;
  switch (a.steps) {
#define AHV_SAGA_LAUNCH(K)                                                                       \
  case K:                                                                                        \
    hipLaunchKernelGGL(saga_fused_regs_kernel<K>, grid_for(a.sagas), dim3(kBlock), 0, st, a); \
    break;
    AHV_SAGA_REG_CASES(AHV_SAGA_LAUNCH)
#undef AHV_SAGA_LAUNCH
    default:
      hipLaunchKernelGGL(saga_fused_kernel, grid_for(a.sagas), dim3(kBlock), 0, st, a);
  }
  check_hip(hipGetLastError(), "saga_fused_kernel");
}

void saga_fused_host(const SagaBatchArgs& a0) {
  const SagaBatchArgs a = saga_with_now(a0);
  check_args(a);
  for (int64_t s = 0; s < a.sagas; ++s) {
    const SagaCounters c = saga_run_chain_fused(a, s);
    if (a.stats) {
      a.stats[0] += c.completed;
      a.stats[1] += c.escalated;
      a.stats[2] += c.failed;
      a.stats[3] += c.compensated;
    }
  }
}

void launch_saga_phase(const SagaBatchArgs& a, int phase, int k, hipStream_t st) {
  check_args(a);
  if (phase < 0 || phase > 4 || k < 0 || k >= a.steps) throw std::invalid_argument("bad saga phase/step");
  if (a.sagas <= 0) return;
  hipLaunchKernelGGL(saga_phase_kernel, grid_for(a.sagas), dim3(kBlock), 0, st, a, phase, k);
  check_hip(hipGetLastError(), "saga_phase_kernel");
}

void saga_phase_host(const SagaBatchArgs& a0, int phase, int k) {
  const SagaBatchArgs a = saga_with_now(a0);
  check_args(a);
  if (phase < 0 || phase > 4 || k < 0 || k >= a.steps) throw std::invalid_argument("bad saga phase/step");
  for (int64_t s = 0; s < a.sagas; ++s) {
    if (phase == 0) {
      saga_init(a, s);
      continue;
    }
    int32_t tick = a.tick[s];
    if (phase == 1) saga_exec_step(a, s, k, tick);
    else if (phase == 2) saga_decide(a, s, tick);
    else if (phase == 3) saga_comp_step(a, s, k, tick);
    else saga_finish(a, s, tick);
    a.tick[s] = tick;
    if (phase == 4 && a.stats) {
      const SagaCounters c = saga_counters(a, s);
      a.stats[0] += c.completed;
      a.stats[1] += c.escalated;
      a.stats[2] += c.failed;
      a.stats[3] += c.compensated;
    }
  }
}


void kernels_saga(std::vector<KernelEntry>& out) {
  out.push_back({"saga_fused_regs_kernel<10>", reinterpret_cast<const void*>(&saga_fused_regs_kernel<10>)});
  out.push_back({"saga_phase_kernel", reinterpret_cast<const void*>(&saga_phase_kernel)});
}

}  // namespace ahv
