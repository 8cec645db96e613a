// Which SIMD does each wave of a multi-wave workgroup run on, and how much does a
// busy sibling wave slow a lone wave's serial SHA-256 rounds (with / without
// s_setprio)?  One workgroup, `nw` waves: wave 0 runs `nblk` dependent
// compressions on lane 0 (the store worker's hash engine), waves 1.. run 64-lane
// compressions (the prefix wave's load) when `busy` is set.
//   hipcc --offload-arch=gfx950 -O3 -I csrc/include scripts/exp/simd_probe.hip -o /tmp/simd_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "ahv/sha256.h"

using namespace ahv;

__global__ void probe(int nblk, int busy, int prio, uint32_t* hwid, uint64_t* ticks, uint32_t* sink) {
  __shared__ uint32_t msg[16 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x) msg[i] = 0x9e3779b9u * (i + 1);
  __syncthreads();
  if (lane == 0) hwid[wave] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  uint32_t st[8];
  sha256_init(st);
  st[0] ^= threadIdx.x;
  if (wave == 0) {
    if (prio) __builtin_amdgcn_s_setprio(3);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (lane == 0)
      for (int b = 0; b < nblk; ++b) sha256_compress(st, msg + 16 * (b & 63));
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) ticks[0] = t1 - t0;
  } else if (busy) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nblk; ++b) sha256_compress(st, msg + 16 * ((b + lane) & 63));
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) ticks[wave] = t1 - t0;
  }
  if (st[0] == 0x12345678u) sink[threadIdx.x] = st[1];
}

int main() {
  uint32_t *hw, *sink;
  uint64_t* tk;
  hipMalloc(&hw, 64);
  hipMalloc(&tk, 64);
  hipMalloc(&sink, 4096);
  const int nblk = 256;
  for (int nw : {1, 2, 3, 4})
    for (int busy : {0, 1})
      for (int prio : {0, 1}) {
        if (nw == 1 && (busy || prio)) continue;
        double best = 1e30;
        uint32_t h[4] = {0, 0, 0, 0};
        uint64_t t[4] = {0, 0, 0, 0};
        for (int rep = 0; rep < 5; ++rep) {
          hipMemset(tk, 0, 64);
          hipLaunchKernelGGL(probe, dim3(1), dim3(64 * nw), 0, 0, nblk, busy, prio, hw, tk, sink);
          if (hipDeviceSynchronize() != hipSuccess) return 2;
          hipMemcpy(h, hw, 4 * nw, hipMemcpyDeviceToHost);
          hipMemcpy(t, tk, 8 * nw, hipMemcpyDeviceToHost);
          if (t[0] < best) best = static_cast<double>(t[0]);
        }
        std::printf("{\"waves\": %d, \"busy\": %d, \"prio\": %d, \"wave0_cycles_per_block\": %.0f, \"simd\": [", nw, busy,
                    prio, best / nblk);
        for (int w = 0; w < nw; ++w) std::printf("%s%u", w ? ", " : "", (h[w] >> 4) & 3);
        std::printf("], \"hw_id\": [");
        for (int w = 0; w < nw; ++w) std::printf("%s\"0x%08x\"", w ? ", " : "", h[w]);
        std::printf("], \"sibling_cycles_per_block\": %.0f}\n", nw > 1 ? static_cast<double>(t[1]) / nblk : 0.0);
      }
  return 0;
}
