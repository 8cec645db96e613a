// Resident command worker of the device state store (csrc/include/ahv/store.h).
//
// One workgroup of two waves on one CU:
//
//   wave 0 — command wave: polls the command ring (512-byte slots in fine-grained
//            device memory the host writes through the PCIe BAR), executes each
//            command against the HBM tables and writes its result slot.  An
//            audit capture is only *recorded* here (delta row, chain links) and
//            queued for wave 1, so lifecycle / saga / liability commands that
//            follow are answered while the digest is still being computed.
//   wave 1 — hash engine: pops capture jobs from an LDS ring in order, stages the
//            record into LDS as SHA-256 message words with the parent digest
//            spliced in (all 64 lanes), runs the serial compression on lane 0
//            (the chain is inherently serial: ≈2.4 µs per 64-byte block on one
//            lane, scripts/exp/doorbell2.hip) and completes the capture's result.
//
// Commands that read audit state (Merkle root, verify, terminate, reads, FLUSH,
// NOP = host drain) wait until wave 1 has drained (`needs_drain`).
//
// Measured transport (scripts/exp/doorbell2.hip): one host→device→host round
// trip of a 512-byte command ≈3.1 µs p50, vs ≈12 µs for a kernel launch + sync.
//
// Lifetime: a resident workgroup shares its hardware queue with whatever streams
// HIP maps there, so it must not linger — kernels queued behind it (and a device
// synchronize) wait until it exits.  It exits after `idle_ticks` of the 100 MHz
// real-time counter without a command, after `max_ticks` in total, or on
// OP_STOP; the host relaunches it on the next command.  Both waves reach the
// exit: wave 0 drains wave 1, raises `stop`, and waits for wave 1's goodbye
// before clearing the host-visible `alive` word.
//
// Memory: results and bulk outputs go to pinned host memory with system-scope
// stores, the sequence word last after a system release fence; `tail` (pinned
// host memory) carries the next expected sequence number across relaunches.
// Waves hand off through LDS with workgroup-scope release/acquire.
#include <hip/hip_runtime.h>

#include "ahv/store.h"

namespace ahv {
namespace store {

constexpr int kJobs = 64;  // LDS capture-job ring

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t lds_acquire(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ __launch_bounds__(128) void store_worker_kernel(Tables t, const uint64_t* ring, int64_t nslots,
                                                           uint64_t* res, uint8_t* bulk, uint64_t* alive,
                                                           int64_t* tail, uint64_t idle_ticks, uint64_t max_ticks,
                                                           int speculate) {
  __shared__ uint64_t inl[kInlineWords];
  __shared__ uint32_t lds1[kLdsWords];      // wave 1: capture message staging
  __shared__ uint32_t kw1[64 * kKwStride];  // wave 1: per-lane K+W schedule rows
  __shared__ uint32_t lds0[kLdsWords / 4];  // wave 0: staging for its own hashing (capture prefixes)
  __shared__ uint32_t kw0[64 * kKwStride];  // wave 0: K+W schedule rows
  __shared__ HashJob jobs[kJobs];
  __shared__ uint32_t q_head, q_done, stop, bye, spec_s;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  if (threadIdx.x == 0) {
    q_head = 0;
    q_done = 0;
    stop = 0;
    bye = 0;
    spec_s = 0;  // session + 1 whose provisional Merkle root wave 1 is computing (0: none)
  }
  __syncthreads();  // the only workgroup barrier: both waves pass it once

  if (wave == 1) {
    // ------------------------------------------------------------ hash engine
    const Lanes L{lane, 64, lds1, kw1};
    uint32_t done = 0;
    for (;;) {
      const uint32_t head = lds_acquire(&q_head);
      if (head == done) {
        if (lds_acquire(&stop)) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      const HashJob j = jobs[done % kJobs];
      uint64_t* r = res + (j.seq % static_cast<uint64_t>(nslots)) * kResWords;
      capture_finish(L, t, j, r);
      if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // digest row + result words before the sequence word
        out64(r, j.seq + 1);
      }
      ++done;
      // Idle next?  Then compute the chain's provisional Merkle root now, so a
      // terminate / compute_merkle_root that follows finds it ready.  `spec_s`
      // is raised before q_done: a drained command wave sees it and, for the
      // same session, waits for the (abortable, few-µs) tree instead of
      // recomputing it; every other command runs alongside.
      const bool idle = (speculate & 1) && __shfl(static_cast<int>(lds_acquire(&q_head) == done), 0) != 0;  // wave-uniform
      if (lane == 0) {
        if (idle) lds_release(&spec_s, static_cast<uint32_t>(j.s) + 1u);
        lds_release(&q_done, done);
      }
      if (idle) {
        const int64_t n = static_cast<int64_t>(t.d_turn[j.d]);
        merkle_provisional(L, t, j.s, j.d, n, lds1, [&] { return lds_acquire(&q_head) != done; });
        if (lane == 0) lds_release(&spec_s, 0u);  // the s_proot rows precede this release
      }
    }
    if (lane == 0) lds_release(&bye, 1u);
    return;
  }

  // ------------------------------------------------------------ command wave
  const Lanes L{lane, 64, lds0, kw0};
  uint64_t next = static_cast<uint64_t>(__hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  uint32_t queued = 0;
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
    L.sync();
    c.inl = inl;
    if (needs_drain(c.op)) {
      while (lds_acquire(&q_done) != queued) __builtin_amdgcn_s_sleep(1);
    }
    if (c.op == OP_SESS_CLOSE || c.op == OP_DELTA_MERKLE) {  // wait for the tree in flight
      const uint32_t want = static_cast<uint32_t>(c.a[0]) + 1u;
      while (lds_acquire(&spec_s) == want) __builtin_amdgcn_s_sleep(1);
    }
    if (c.op == OP_DELTA_CAPTURE) {
      while (queued - lds_acquire(&q_done) >= static_cast<uint32_t>(kJobs)) __builtin_amdgcn_s_sleep(1);
    }
    if (c.op == OP_ACQUIRE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    uint64_t* r = res + (next % static_cast<uint64_t>(nslots)) * kResWords;
    HashJob job;
    const int rc = store_exec(L, t, c, next, r, bulk, &job);
    if (c.op == OP_FLUSH) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    L.sync();
    if (rc == EXEC_DEFERRED) {
      // A capture with a parent: while the hash engine works through the queue,
      // compress the record's blocks that precede the parent hole here — unless
      // the next command is already waiting (then wave 1 does all of it).
      const int64_t jhole = bcast(L, job.hole);
      if ((speculate & 2) && jhole >= 64 && lds_acquire(&q_done) != queued) {
        const uint64_t* nslot = ring + ((next + 1) % static_cast<uint64_t>(nslots)) * kSlotWords;
        if (__shfl(ld_sys(nslot + lane), 0) != next + 2) {
          HashJob jb;
          jb.off = bcast(L, job.off);
          jb.hole = jhole;
          uint32_t mid[8];
          const int32_t pb = capture_prefix(L, t, jb, lds0, kLdsWords / 4, 4, mid);
          if (lane == 0 && pb > 0) {
            job.mid_blocks = pb;
            for (int k = 0; k < 8; ++k) job.mid[k] = mid[k];
          }
        }
      }
      if (lane == 0) {
        jobs[queued % kJobs] = job;
        lds_release(&q_head, queued + 1);  // the capture's global row writes precede this release
      }
      ++queued;
    } else if (lane == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      out64(r, next + 1);
    }
    if (lane == 0) __hip_atomic_store(tail, static_cast<int64_t>(next + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ++next;
    last = __builtin_amdgcn_s_memrealtime();
    if (rc == EXEC_STOP) break;
  }
  // drain the hash engine, stop it, wait for its goodbye, then release the queue
  while (lds_acquire(&q_done) != queued) __builtin_amdgcn_s_sleep(1);
  if (lane == 0) lds_release(&stop, 1u);
  while (!lds_acquire(&bye)) __builtin_amdgcn_s_sleep(1);
  if (lane == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace store
}  // namespace ahv

// Host-callable launcher (one workgroup: command wave + hash-engine wave).
extern "C" int ahv_store_launch_worker(const ahv::store::Tables* t, const uint64_t* ring, int64_t nslots,
                                       uint64_t* res, uint8_t* bulk, uint64_t* alive, int64_t* tail,
                                       uint64_t idle_ticks, uint64_t max_ticks, int speculate,
                                       hipStream_t stream) {
  hipLaunchKernelGGL(ahv::store::store_worker_kernel, dim3(1), dim3(128), 0, stream, *t, ring, nslots, res, bulk,
                     alive, tail, idle_ticks, max_ticks, speculate);
  return static_cast<int>(hipGetLastError());
}
