// Doorbell microbenchmark v2: one wave-wide read per poll (header + payload in
// one PCIe round trip, torn reads caught by a checksum), look-ahead ingestion
// of queued commands, command ring in host memory vs fine-grained device memory.
//   ./doorbell2 host|dev
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ahv/sha256.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// 512-byte slot = 64 words: w[0] = seq, w[1] = op, w[2] = nwords, w[3] = arg,
// w[4] = checksum (xor of every other word), w[5..63] payload.
constexpr int kSlots = 256;
constexpr int kW = 64;

struct alignas(64) Done {
  uint64_t seq;
  uint64_t result[7];
};

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t wave_xor(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(64) void worker(const uint64_t* ring, Done* done, uint64_t start_seq,
                                             uint64_t idle_ticks, uint64_t* exit_code, uint64_t* torn) {
  const int lane = threadIdx.x;
  uint64_t next = start_seq;
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  uint64_t ntorn = 0;
  for (;;) {
    const uint64_t* s = ring + (next % kSlots) * kW;
    const uint64_t w = ld_sys(s + lane);
    const uint64_t seq = __shfl(w, 0);
    if (seq != next + 1) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - last > idle_ticks) {
        if (lane == 0) { st_sys(exit_code, 2); st_sys(torn, ntorn); }
        return;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    const uint64_t x = wave_xor(lane == 0 || lane == 4 ? 0 : w);
    if (x != __shfl(w, 4)) { ++ntorn; continue; }  // torn read: poll again
    const uint64_t op = __shfl(w, 1);
    const uint64_t arg = __shfl(w, 3);
    uint64_t r = 0;
    if (op == 0) {
      if (lane == 0) { st_sys(exit_code, 1); st_sys(torn, ntorn); st_sys(&done[next % kSlots].seq, next + 1); }
      return;
    } else if (op == 1) {
      r = arg + 1;
    } else if (op == 2) {
      uint64_t v = lane >= 5 ? w : 0;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      r = v;
    } else if (op == 3) {
      uint32_t st[8];
      ahv::sha256_init(st);
      uint32_t blk[16];
      for (int i = 0; i < 16; ++i) blk[i] = (uint32_t)(i * 0x9e3779b9u) ^ (uint32_t)w;
      for (uint64_t k = 0; k < arg; ++k) {
        ahv::sha256_compress(st, blk);
        blk[k & 15] ^= st[0];
      }
      r = st[0];
    }
    if (lane == 0) {
      st_sys(&done[next % kSlots].result[0], r);
      __atomic_thread_fence(__ATOMIC_RELEASE);
      st_sys(&done[next % kSlots].seq, next + 1);
    }
    ++next;
    last = __builtin_amdgcn_s_memrealtime();
  }
}

static uint64_t g_seq = 0;

static void put(uint64_t* ring, uint64_t seq_index, uint64_t op, uint64_t arg, const uint64_t* payload, int pw) {
  uint64_t* s = ring + (seq_index % kSlots) * kW;
  s[1] = op;
  s[2] = (uint64_t)pw;
  s[3] = arg;
  uint64_t x = op ^ (uint64_t)pw ^ arg;
  for (int i = 0; i < 59; ++i) {
    const uint64_t v = i < pw ? payload[i] : 0;
    s[5 + i] = v;
    x ^= v;
  }
  s[4] = x;
  __atomic_store_n(&s[0], seq_index + 1, __ATOMIC_RELEASE);
}

static uint64_t wait_for(Done* done, uint64_t seq_index) {
  Done* d = done + (seq_index % kSlots);
  while (__atomic_load_n(&d->seq, __ATOMIC_ACQUIRE) != seq_index + 1) __builtin_ia32_pause();
  return d->result[0];
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
  const bool devmem = argc > 1 && std::strcmp(argv[1], "dev") == 0;
  uint64_t* ring = nullptr;
  Done* done = nullptr;
  uint64_t* ctl = nullptr;
  const size_t ring_bytes = sizeof(uint64_t) * kW * kSlots;
  if (devmem) {
    CK(hipExtMallocWithFlags((void**)&ring, ring_bytes, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, ring));
    std::printf("fine-grained device ring: type=%d hostPointer=%p devicePointer=%p\n", (int)at.type, at.hostPointer,
                at.devicePointer);
    CK(hipMemset(ring, 0, ring_bytes));
    CK(hipDeviceSynchronize());
    std::fflush(stdout);
    volatile uint64_t probe = ring[0];  // faults here if the host cannot map device memory
    (void)probe;
    std::printf("host can read the device ring\n");
  } else {
    CK(hipHostMalloc((void**)&ring, ring_bytes, hipHostMallocCoherent));
    std::memset(ring, 0, ring_bytes);
  }
  CK(hipHostMalloc((void**)&done, sizeof(Done) * kSlots, hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&ctl, 128, hipHostMallocCoherent));
  std::memset(done, 0, sizeof(Done) * kSlots);
  std::memset(ctl, 0, 128);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, st, ring, done, g_seq, (uint64_t)20000000, ctl, ctl + 8);
  CK(hipGetLastError());
  put(ring, g_seq, 1, 41, nullptr, 0);
  wait_for(done, g_seq++);

  uint64_t payload[59];
  for (int i = 0; i < 59; ++i) payload[i] = i * 3;
  for (int pw : {0, 40}) {
    std::vector<double> lat;
    for (int it = 0; it < 20000; ++it) {
      auto t0 = clk::now();
      put(ring, g_seq, pw ? 2 : 1, it, payload, pw);
      wait_for(done, g_seq++);
      auto t1 = clk::now();
      if (it >= 1000) lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("[%s] RT payload %2d words: p50 %.2f us p90 %.2f p99 %.2f min %.2f\n", devmem ? "dev" : "host", pw,
                pct(lat, 0.5), pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.0));
  }
  for (int q : {4, 8}) {
    std::vector<double> lat;
    for (int it = 0; it < 5000; ++it) {
      auto t0 = clk::now();
      for (int k = 0; k < q; ++k) put(ring, g_seq + k, 2, k, payload, 40);
      wait_for(done, g_seq + q - 1);
      g_seq += q;
      auto t1 = clk::now();
      if (it >= 500) lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("[%s] %d queued 40-word commands then wait: p50 %.2f us (%.2f us/cmd)\n", devmem ? "dev" : "host", q,
                pct(lat, 0.5), pct(lat, 0.5) / q);
  }
  for (uint64_t n : {1ull, 1025ull}) {
    std::vector<double> lat;
    for (int it = 0; it < 200; ++it) {
      auto t0 = clk::now();
      put(ring, g_seq, 3, n, nullptr, 0);
      wait_for(done, g_seq++);
      lat.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    std::printf("[%s] SHA %llu compressions: p50 RT %.2f us\n", devmem ? "dev" : "host", (unsigned long long)n,
                pct(lat, 0.5));
  }
  put(ring, g_seq, 0, 0, nullptr, 0);
  wait_for(done, g_seq++);
  CK(hipStreamSynchronize(st));
  std::printf("[%s] exit code %llu, torn reads %llu\n", devmem ? "dev" : "host", (unsigned long long)ctl[0],
              (unsigned long long)ctl[8]);
  return 0;
}
