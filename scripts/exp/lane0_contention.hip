// Do lone-lane SHA-256 round loops on sibling waves (one per SIMD) slow each other
// down, as the store worker's engine and helper waves appear to?  `nw` waves; the
// first `active` run `nblk` K+W round loops on lane 0 over a row in LDS (the
// worker's split form: ahv/store.h sha256_rounds_kw); the rest idle.  Per-wave
// s_memtime ticks per block.
//   hipcc --offload-arch=gfx950 -O3 -I csrc/include scripts/exp/lane0_contention.hip -o scripts/exp/lane0_contention
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "ahv/store.h"

using namespace ahv;
using namespace ahv::store;

__global__ void probe(int nblk, int active, int expand, uint64_t* ticks, uint32_t* sink) {
  __shared__ uint32_t msg[4][16];
  __shared__ uint32_t kw[4][64 * kKwStride];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = lane; i < 16; i += 64) msg[wave][i] = 0x9e3779b9u * (i + 1 + wave);
  __syncthreads();
  if (lane < 1) sha256_expand_kw(msg[wave], kw[wave]);
  __syncthreads();
  uint32_t st[8];
  sha256_init(st);
  st[0] ^= threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (wave < active) {
    for (int b = 0; b < nblk; ++b) {
      if (expand && lane < 4) sha256_expand_kw(msg[wave], kw[wave] + kKwStride * lane);
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) sha256_rounds_kw(st, kw[wave]);
      __builtin_amdgcn_wave_barrier();
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) ticks[wave] = t1 - t0;
  if (st[0] == 0x12345678u) sink[threadIdx.x] = st[1];
}

int main() {
  uint64_t* tk;
  uint32_t* sink;
  hipMalloc(&tk, 64);
  hipMalloc(&sink, 4096);
  const int nblk = 256;
  for (int expand : {0, 1})
    for (int active = 1; active <= 4; ++active) {
      uint64_t best[4] = {~0ull, ~0ull, ~0ull, ~0ull};
      for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, nblk, active, expand, tk, sink);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        uint64_t t[4];
        hipMemcpy(t, tk, 32, hipMemcpyDeviceToHost);
        for (int w = 0; w < 4; ++w)
          if (t[w] < best[w]) best[w] = t[w];
      }
      std::printf("{\"expand_each_block\": %d, \"active_waves\": %d, \"ticks_per_block\": [", expand, active);
      for (int w = 0; w < active; ++w) std::printf("%s%.0f", w ? ", " : "", static_cast<double>(best[w]) / nblk);
      std::printf("]}\n");
    }
  return 0;
}
