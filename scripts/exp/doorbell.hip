// Microbenchmark: host <-> persistent-worker round trip over a pinned-memory
// doorbell, and single-wave SHA-256 compression time, on one MI355X.
//
// Decides the transport of the device-authoritative state store: if a command
// round trip through a polling worker costs a few µs, every public-API call can
// be served by the device (no host mirror of session state).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/doorbell scripts/exp/doorbell.hip
//   ./build/doorbell
//
// The worker exits on a STOP command or after 200 ms without a command (idle
// timeout on the 100 MHz real-time counter), so no wave outlives the process.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ahv/sha256.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

struct alignas(64) Slot {
  uint64_t seq;      // written last by the host
  uint64_t op;
  uint64_t arg[6];
  uint64_t payload[56];  // 448 bytes
};

struct alignas(64) Done {
  uint64_t seq;
  uint64_t result[7];
};

constexpr int kSlots = 64;

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void worker(Slot* ring, Done* done, uint64_t start_seq, uint64_t idle_ticks,
                                             uint64_t* exit_code) {
  const int lane = threadIdx.x;
  __shared__ uint64_t s_hdr[8];
  uint64_t next = start_seq;
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    Slot* s = ring + (next % kSlots);
    uint64_t seq = 0;
    if (lane == 0) seq = ld_sys(&s->seq);
    seq = __shfl(seq, 0);
    if (seq != next + 1) {
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (now - last > idle_ticks) {
        if (lane == 0) st_sys(exit_code, 2);
        return;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    // header words 1..7 and the payload, one 8-byte word per lane
    uint64_t w = 0;
    if (lane < 7) w = ld_sys(&s->op + lane);
    uint64_t pw = 0;
    const uint64_t op = __shfl(w, 0);
    const uint64_t plen = __shfl(w, 1);  // arg[0] = payload words
    if ((uint64_t)lane < plen) pw = ld_sys(&s->payload[lane]);
    if (op == 0) {  // STOP
      if (lane == 0) {
        st_sys(exit_code, 1);
        st_sys(&done[next % kSlots].seq, next + 1);
      }
      return;
    }
    uint64_t r = 0;
    if (op == 1) {  // PING: echo arg[1] + 1
      r = __shfl(w, 2) + 1;
    } else if (op == 2) {  // SUM of payload words (wave reduction)
      uint64_t v = pw;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      r = v;
    } else if (op == 3) {  // SHA-256: arg[1] serial compressions on lane 0
      const uint64_t n = __shfl(w, 2);
      uint32_t st[8];
      ahv::sha256_init(st);
      uint32_t blk[16];
      for (int i = 0; i < 16; ++i) blk[i] = (uint32_t)(i * 0x9e3779b9u) ^ (uint32_t)lane;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (uint64_t k = 0; k < n; ++k) {
        ahv::sha256_compress(st, blk);
        blk[0] ^= st[0];
      }
      const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
      r = (t1 - t0);  // 100 MHz ticks
      if (lane == 0) s_hdr[0] = st[0];
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

static void submit(Slot* ring, uint64_t op, uint64_t a1, const uint64_t* payload, int pw) {
  Slot* s = ring + (g_seq % kSlots);
  s->op = op;
  s->arg[0] = (uint64_t)pw;
  s->arg[1] = a1;
  for (int i = 0; i < pw; ++i) s->payload[i] = payload[i];
  __atomic_store_n(&s->seq, g_seq + 1, __ATOMIC_RELEASE);
}

static uint64_t wait(Done* done) {
  Done* d = done + (g_seq % kSlots);
  while (__atomic_load_n(&d->seq, __ATOMIC_ACQUIRE) != g_seq + 1) {
    __builtin_ia32_pause();
  }
  uint64_t r = d->result[0];
  ++g_seq;
  return r;
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main() {
  Slot* ring = nullptr;
  Done* done = nullptr;
  uint64_t* exit_code = nullptr;
  CK(hipHostMalloc((void**)&ring, sizeof(Slot) * kSlots, hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&done, sizeof(Done) * kSlots, hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&exit_code, 64, hipHostMallocCoherent));
  std::memset(ring, 0, sizeof(Slot) * kSlots);
  std::memset(done, 0, sizeof(Done) * kSlots);
  *exit_code = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;

  auto t_launch0 = clk::now();
  hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, st, ring, done, g_seq, (uint64_t)20000000 /*200 ms*/,
                     exit_code);
  CK(hipGetLastError());
  // first round trip includes the launch
  submit(ring, 1, 41, nullptr, 0);
  uint64_t r = wait(done);
  auto t_launch1 = clk::now();
  std::printf("first ping (launch + RT): %.2f us  (r=%llu)\n",
              std::chrono::duration<double, std::micro>(t_launch1 - t_launch0).count(), (unsigned long long)r);

  for (int pw : {0, 8, 40, 56}) {
    std::vector<double> lat;
    uint64_t payload[56];
    for (int i = 0; i < 56; ++i) payload[i] = i;
    for (int it = 0; it < 20000; ++it) {
      auto t0 = clk::now();
      submit(ring, pw ? 2 : 1, it, payload, pw);
      r = wait(done);
      auto t1 = clk::now();
      if (it >= 1000) lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("RT payload %3d words: p50 %.2f us  p90 %.2f  p99 %.2f  min %.2f  (r=%llu)\n", pw, pct(lat, 0.5),
                pct(lat, 0.9), pct(lat, 0.99), pct(lat, 0.0), (unsigned long long)r);
  }
  // pipelined: 8 async commands, then wait for all
  {
    std::vector<double> lat;
    for (int it = 0; it < 5000; ++it) {
      auto t0 = clk::now();
      uint64_t base = g_seq;
      for (int k = 0; k < 8; ++k) {
        Slot* s = ring + ((base + k) % kSlots);
        s->op = 1; s->arg[0] = 0; s->arg[1] = k;
        __atomic_store_n(&s->seq, base + k + 1, __ATOMIC_RELEASE);
      }
      Done* d = done + ((base + 7) % kSlots);
      while (__atomic_load_n(&d->seq, __ATOMIC_ACQUIRE) != base + 8) __builtin_ia32_pause();
      g_seq = base + 8;
      auto t1 = clk::now();
      if (it >= 500) lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::printf("8 queued pings then wait: p50 %.2f us (%.2f us/cmd)\n", pct(lat, 0.5), pct(lat, 0.5) / 8);
  }
  for (uint64_t n : {1ull, 16ull, 256ull}) {
    submit(ring, 3, n, nullptr, 0);
    uint64_t ticks = wait(done);
    std::printf("SHA-256 %4llu serial compressions on one lane: %.3f us/block\n", (unsigned long long)n,
                ticks * 0.01 / n);
  }
  submit(ring, 0, 0, nullptr, 0);
  wait(done);
  CK(hipStreamSynchronize(st));
  std::printf("worker exit code %llu\n", (unsigned long long)*exit_code);

  // relaunch cost after idle exit
  auto t2 = clk::now();
  hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, st, ring, done, g_seq, (uint64_t)2000000 /*20 ms*/, exit_code);
  submit(ring, 1, 1, nullptr, 0);
  wait(done);
  auto t3 = clk::now();
  std::printf("relaunch + first RT: %.2f us\n", std::chrono::duration<double, std::micro>(t3 - t2).count());
  auto t4 = clk::now();
  CK(hipStreamSynchronize(st));  // idle exit after 20 ms
  auto t5 = clk::now();
  std::printf("idle exit observed after %.2f ms, exit code %llu\n",
              std::chrono::duration<double, std::milli>(t5 - t4).count(), (unsigned long long)*exit_code);
  // tiny-kernel launch + sync for comparison
  return 0;
}
