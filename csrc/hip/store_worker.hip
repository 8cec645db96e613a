// Resident command worker of the device state store (csrc/include/ahv/store.h).
//
// One wave (64 lanes) on one CU polls the command ring — 512-byte slots in
// fine-grained device memory that the host writes through the PCIe BAR — and
// executes each command against the HBM tables.  Measured on MI355X
// (scripts/exp/doorbell2.hip, profiles/store_transport_r2.md): one host→device→
// host round trip of a 512-byte command is ≈3.1 µs p50, against ≈12 µs for a
// kernel launch + stream sync.
//
// Lifetime: a resident wave shares its hardware queue with whatever streams HIP
// maps there, so it must not linger — kernels queued behind it (and any device
// synchronize) wait until it exits.  The worker therefore exits after
// `idle_ticks` of the 100 MHz real-time counter without a command, after
// `max_ticks` in total, or on OP_STOP; the host relaunches it on the next
// command (≈12 µs).  Every exit path is reached by the whole wave.
//
// Memory: results and bulk outputs go to pinned host memory with system-scope
// stores; the result's sequence word is written last, after a system release
// fence.  `tail` (device memory) carries the next expected sequence number
// across relaunches.
#include <hip/hip_runtime.h>

#include "ahv/store.h"

namespace ahv {
namespace store {

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void store_worker_kernel(Tables t, const uint64_t* ring, int64_t nslots,
                                                          uint64_t* res, uint8_t* bulk, uint64_t* alive,
                                                          int64_t* tail, uint64_t idle_ticks, uint64_t max_ticks) {
  __shared__ uint64_t inl[kInlineWords];
  __shared__ uint32_t lds[kLdsWords];
  const int lane = threadIdx.x;
  const Lanes L{lane, 64, lds};
  uint64_t next = static_cast<uint64_t>(__hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t last = t0;
  for (;;) {
    const uint64_t* slot = ring + (next % static_cast<uint64_t>(nslots)) * kSlotWords;
    const uint64_t w = ld_sys(slot + lane);
    const uint64_t seq = __shfl(w, 0);
    if (seq != next + 1) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - last > idle_ticks || now - t0 > max_ticks) break;
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    uint64_t x = (lane == 0 || lane == 2) ? 0ull : w;
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o);
    if (x != __shfl(w, 2)) continue;  // torn read of a slot still being written: poll again
    Cmd c;
    c.op = static_cast<uint32_t>(__shfl(w, 1));
#pragma unroll
    for (int k = 0; k < kArgs; ++k) c.a[k] = __shfl(w, 3 + k);
    if (lane >= 16) inl[lane - 16] = w;
    __syncthreads();
    c.inl = inl;
    if (c.op == OP_ACQUIRE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    uint64_t* r = res + (next % static_cast<uint64_t>(nslots)) * kResWords;
    const bool go_on = store_exec(L, t, c, r, bulk);
    if (c.op == OP_FLUSH) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (lane == 0) {
      __hip_atomic_store(tail, static_cast<int64_t>(next + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      out64(r, next + 1);
    }
    ++next;
    last = __builtin_amdgcn_s_memrealtime();
    if (!go_on) break;
  }
  __syncthreads();
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace store
}  // namespace ahv

// Host-callable launcher (one wave, one workgroup).
extern "C" int ahv_store_launch_worker(const ahv::store::Tables* t, const uint64_t* ring, int64_t nslots,
                                       uint64_t* res, uint8_t* bulk, uint64_t* alive, int64_t* tail,
                                       uint64_t idle_ticks, uint64_t max_ticks, hipStream_t stream) {
  hipLaunchKernelGGL(ahv::store::store_worker_kernel, dim3(1), dim3(64), 0, stream, *t, ring, nslots, res, bulk,
                     alive, tail, idle_ticks, max_ticks);
  return static_cast<int>(hipGetLastError());
}
