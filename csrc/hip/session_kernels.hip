// Session concurrency kernels: vector clocks (K19) and intent-lock contention
// (K20), SURVEY §2.14.
#include "ahv/kernels.h"
#include "ahv/launch.h"

namespace ahv {

// ------------------------------------------------------------------ K19
// One wave per group; lane j owns component j of every clock it touches.
// read : agent ← max(agent, path)
// write: reject (strict) iff path ≠ 0 and agent happens-before path
//        (all agent ≤ path, some agent < path); else tick agent[col] and
//        path ← max(path, agent).  (reference session/vector_clock.py:88-149)

__global__ __launch_bounds__(64) void vclock_kernel(VClockArgs a) {
  const int64_t g = blockIdx.x;
  if (g >= a.groups) return;
  const int j = threadIdx.x;
  const bool lane_on = j < a.A;
  for (int32_t q = a.offsets[g]; q < a.offsets[g + 1]; ++q) {
    uint32_t* pc = a.path_clock + static_cast<int64_t>(a.path[q]) * a.A;
    uint32_t* ac = a.agent_clock + static_cast<int64_t>(a.agent[q]) * a.A;
    const uint32_t p = lane_on ? pc[j] : 0u;
    uint32_t ag = lane_on ? ac[j] : 0u;
    if (a.op[q] == 0) {
      if (lane_on) ac[j] = ag > p ? ag : p;
      if (j == 0) a.ok[q] = 1;
    } else {
      const bool path_set = __any(p != 0u);
      const bool le = __all(ag <= p);
      const bool lt = __any(ag < p);
      const bool violation = a.strict && path_set && le && lt;
      if (j == 0) a.ok[q] = violation ? 0 : 1;
      if (!violation) {
        if (j == a.agent_col[q]) ag += 1;
        if (lane_on) {
          ac[j] = ag;
          pc[j] = p > ag ? p : ag;
        }
      }
    }
    __syncthreads();  // the next op of this group may touch the same rows
  }
}

void launch_vclock(const VClockArgs& a, hipStream_t st) {
  if (a.groups <= 0) return;
  if (a.A > 64) throw std::runtime_error("vector clock width > 64");
  hipLaunchKernelGGL(vclock_kernel, dim3(static_cast<uint32_t>(a.groups)), dim3(64), 0, st, a);
  check_hip(hipGetLastError(), "vclock_kernel");
}

void vclock_host(const VClockArgs& a) {
  for (int64_t g = 0; g < a.groups; ++g) {
    for (int32_t q = a.offsets[g]; q < a.offsets[g + 1]; ++q) {
      uint32_t* pc = a.path_clock + static_cast<int64_t>(a.path[q]) * a.A;
      uint32_t* ac = a.agent_clock + static_cast<int64_t>(a.agent[q]) * a.A;
      if (a.op[q] == 0) {
        for (int j = 0; j < a.A; ++j) ac[j] = ac[j] > pc[j] ? ac[j] : pc[j];
        a.ok[q] = 1;
        continue;
      }
      bool path_set = false, le = true, lt = false;
      for (int j = 0; j < a.A; ++j) {
        path_set = path_set || pc[j] != 0;
        le = le && ac[j] <= pc[j];
        lt = lt || ac[j] < pc[j];
      }
      const bool violation = a.strict && path_set && le && lt;
      a.ok[q] = violation ? 0 : 1;
      if (violation) continue;
      ac[a.agent_col[q]] += 1;
      for (int j = 0; j < a.A; ++j) pc[j] = pc[j] > ac[j] ? pc[j] : ac[j];
    }
  }
}

// ------------------------------------------------------------------ K20
// Only READ + READ is compatible; an agent never conflicts with its own locks
// (reference session/intent_locks.py:158-178).

AHV_HD void locks_elem(const LockArgs& a, int64_t i) {
  const int32_t r = a.req_res[i];
  int32_t n = 0;
  for (int32_t l = a.res_offsets[r]; l < a.res_offsets[r + 1]; ++l) {
    if (a.lock_agent[l] == a.req_agent[i]) continue;
    if (!(a.lock_intent[l] == 0 && a.req_intent[i] == 0)) ++n;
  }
  a.conflicts[i] = n;
}
__global__ void locks_kernel(LockArgs a) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    locks_elem(a, i);
}
void launch_locks(const LockArgs& a, hipStream_t st) {
  if (a.n <= 0) return;
  const int64_t b = (a.n + 255) / 256;
  hipLaunchKernelGGL(locks_kernel, dim3(static_cast<uint32_t>(b)), dim3(256), 0, st, a);
  check_hip(hipGetLastError(), "locks_kernel");
}
void locks_host(const LockArgs& a) { for (int64_t i = 0; i < a.n; ++i) locks_elem(a, i); }

AHV_HD void lock_grant_segment(const LockGrantArgs& a, int64_t g) {
  const int32_t k0 = a.seg_offsets[g], k1 = a.seg_offsets[g + 1];
  int32_t* row = a.table + static_cast<int64_t>(a.req_res[a.order[k0]]) * kLockRow;
  int32_t rc = row[0], wc = row[1];
  for (int32_t k = k0; k < k1; ++k) {
    const int32_t i = a.order[k];
    const int32_t ag = a.req_agent[i];
    const uint8_t in = a.req_intent[i];
    const bool write = (in & 0x7f) != 0;
    int own = -1, free_slot = -1;
    for (int h = 0; h < kLockHolders; ++h) {
      const int32_t who = row[2 + 2 * h];
      if (who == ag) own = h;
      if (who == -1 && free_slot < 0) free_slot = h;
    }
    const int32_t rw = own >= 0 ? row[3 + 2 * own] : 0;
    const int32_t own_r = rw & 0xffff, own_w = rw >> 16;
    if (in & 0x80) {  // release one lock of this intent
      if (own >= 0 && (write ? own_w : own_r) > 0) {
        const int32_t nrw = write ? rw - 0x10000 : rw - 1;
        row[3 + 2 * own] = nrw;
        if (nrw == 0) row[2 + 2 * own] = -1;
        if (write) --wc;
        else --rc;
        a.granted[i] = 1;
      } else {
        a.granted[i] = 0;
      }
      continue;
    }
    const bool ok = write ? (rc - own_r) + (wc - own_w) == 0 : wc - own_w == 0;
    if (!ok) {
      a.granted[i] = 0;
      continue;
    }
    const int slot = own >= 0 ? own : free_slot;
    if (slot < 0) {  // every holder slot belongs to another agent
      a.granted[i] = 2;
      continue;
    }
    row[2 + 2 * slot] = ag;
    row[3 + 2 * slot] = write ? rw + 0x10000 : rw + 1;
    if (write) ++wc;
    else ++rc;
    a.granted[i] = 1;
  }
  row[0] = rc;
  row[1] = wc;
}
__global__ void lock_grant_kernel(LockGrantArgs a) {
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < a.segments;
       g += static_cast<int64_t>(gridDim.x) * blockDim.x)
    lock_grant_segment(a, g);
}
void launch_lock_grant(const LockGrantArgs& a, hipStream_t st) {
  if (a.segments <= 0) return;
  const int64_t b = (a.segments + 255) / 256;
  hipLaunchKernelGGL(lock_grant_kernel, dim3(static_cast<uint32_t>(b)), dim3(256), 0, st, a);
  check_hip(hipGetLastError(), "lock_grant_kernel");
}
void lock_grant_host(const LockGrantArgs& a) { for (int64_t g = 0; g < a.segments; ++g) lock_grant_segment(a, g); }

}  // namespace ahv
