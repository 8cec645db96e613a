// Does a resident polling worker block other streams' kernels?  Worker on
// (a) a plain non-blocking stream, (b) a CU-masked stream; while it runs, time
// a tiny kernel on the null stream, on a fresh non-blocking stream, and on 8
// more streams.  Worker exits on STOP or 50 ms idle.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1);} } while (0)

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

__global__ void worker(const uint64_t* cmd, uint64_t* ack, uint64_t idle_ticks) {
  uint64_t last = __builtin_amdgcn_s_memrealtime();
  uint64_t seen = 0;
  for (;;) {
    uint64_t c = 0;
    if (threadIdx.x == 0) c = ld_sys(cmd);
    c = __shfl(c, 0);
    if (c == ~0ull) { if (threadIdx.x == 0) st_sys(ack, ~0ull); return; }
    if (c != seen) { seen = c; if (threadIdx.x == 0) st_sys(ack, c); last = __builtin_amdgcn_s_memrealtime(); continue; }
    if (__builtin_amdgcn_s_memrealtime() - last > idle_ticks) { if (threadIdx.x == 0) st_sys(ack, 0xdeadull); return; }
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ void tiny(int* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main() {
  uint64_t *cmd, *ack;
  CK(hipExtMallocWithFlags((void**)&cmd, 4096, hipDeviceMallocFinegrained));
  CK(hipHostMalloc((void**)&ack, 4096, hipHostMallocCoherent));
  CK(hipMemset(cmd, 0, 4096));
  CK(hipDeviceSynchronize());
  int* buf;
  CK(hipMalloc((void**)&buf, 4096 * 4));
  CK(hipMemset(buf, 0, 4096 * 4));
  for (int mode = 0; mode < 2; ++mode) {
    hipStream_t ws;
    if (mode == 0) {
      CK(hipStreamCreateWithFlags(&ws, hipStreamNonBlocking));
    } else {
      uint32_t mask[8] = {1u, 0, 0, 0, 0, 0, 0, 0};  // CU 0 only
      CK(hipExtStreamCreateWithCUMask(&ws, 8, mask));
    }
    *ack = 0;
    cmd[0] = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(worker, dim3(1), dim3(64), 0, ws, cmd, ack, (uint64_t)5000000 /*50 ms*/);
    CK(hipGetLastError());
    cmd[0] = 1;
    auto t0 = clk::now();
    while (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != 1) {}
    std::printf("[%s] worker alive after %.1f us\n", mode ? "cumask" : "plain", us(t0, clk::now()));
    // null stream kernel
    auto a = clk::now();
    hipLaunchKernelGGL(tiny, dim3(256), dim3(64), 0, 0, buf);
    CK(hipStreamSynchronize(0));
    auto b = clk::now();
    std::printf("[%s] null-stream tiny kernel + sync: %.1f us\n", mode ? "cumask" : "plain", us(a, b));
    std::vector<hipStream_t> ss(9);
    for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int k = 0; k < 9; ++k) {
      a = clk::now();
      hipLaunchKernelGGL(tiny, dim3(256), dim3(64), 0, ss[k], buf);
      CK(hipStreamSynchronize(ss[k]));
      b = clk::now();
      std::printf("[%s] stream %d tiny kernel + sync: %.1f us\n", mode ? "cumask" : "plain", k, us(a, b));
    }
    // still alive?
    cmd[0] = 2;
    t0 = clk::now();
    while (__atomic_load_n(ack, __ATOMIC_ACQUIRE) != 2 && us(t0, clk::now()) < 200000) {}
    std::printf("[%s] worker ack 2: %llx after %.1f us\n", mode ? "cumask" : "plain", (unsigned long long)*ack, us(t0, clk::now()));
    a = clk::now();
    cmd[0] = ~0ull;
    CK(hipDeviceSynchronize());
    std::printf("[%s] stop + device sync: %.1f us\n", mode ? "cumask" : "plain", us(a, clk::now()));
    for (auto& s : ss) CK(hipStreamDestroy(s));
    CK(hipStreamDestroy(ws));
  }
  return 0;
}
