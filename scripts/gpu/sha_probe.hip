// Single-wave SHA-256 latency probe (gfx950).  Measures what one serial
// compression costs on the lone hash-engine wave of the store worker: the wall
// time (s_memrealtime, 100 MHz) and the shader-clock cycles (s_memtime) of N
// dependent compressions run by lane 0, so both the per-block cost and the clock
// the CU actually ran at come out of one launch.
//
//   hipcc --offload-arch=gfx950 -O3 -I csrc/include scripts/gpu/sha_probe.hip -o /tmp/sha_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#include "ahv/sha256.h"

using namespace ahv;

__device__ __forceinline__ uint32_t add3d(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// rounds over a K+W row held in LDS (the worker's split form)
__device__ void rounds_kw(uint32_t st[8], const uint32_t* kw) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
  uint32_t q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = kw[i];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint32_t kwi = q[i & 7];
    if (i + 8 < 64) q[i & 7] = kw[i + 8];
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t t1 = add3d(h + kwi, S1, sha_ch(e, f, g));
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t na = add3d(t1, S0, sha_maj(a, b, c));
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = na;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// mode 0: full compression on lane 0; 1: K+W rounds on lane 0; 2: full
// compression on all 64 lanes (independent messages: throughput reference);
// 3: full compression on lane 0 with the message in SGPR-uniform registers
// (readfirstlane'd state: the compiler may pick SALU)
__global__ __launch_bounds__(64) void probe(int mode, int nblk, uint64_t* out) {
  __shared__ uint32_t msg[16 * 64];
  __shared__ uint32_t kw[64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * 64; i += 64) msg[i] = 0x9e3779b9u * (i + 1);
  for (int i = lane; i < 64; i += 64) kw[i] = sha256_k(i) + msg[i & 15];
  __syncthreads();
  uint32_t st[8];
  sha256_init(st);
  st[0] ^= lane;
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {
    if (lane == 0)
      for (int b = 0; b < nblk; ++b) sha256_compress(st, msg + 16 * (b & 63));
  } else if (mode == 1) {
    if (lane == 0)
      for (int b = 0; b < nblk; ++b) rounds_kw(st, kw);
  } else if (mode == 2) {
    for (int b = 0; b < nblk; ++b) sha256_compress(st, msg + 16 * ((b + lane) & 63));
  } else {
    uint32_t u[8];
    for (int k = 0; k < 8; ++k) u[k] = __builtin_amdgcn_readfirstlane(st[k]);
    for (int b = 0; b < nblk; ++b) {
      uint32_t w[16];
      for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_readfirstlane(msg[16 * (b & 63) + k]);
      sha256_compress(u, w);
    }
    for (int k = 0; k < 8; ++k) st[k] = u[k];
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    out[0] = r1 - r0;
    out[1] = c1 - c0;
    out[2] = st[0] ^ st[7];
  }
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 64) != hipSuccess) return 1;
  const char* names[] = {"lane0_full", "lane0_kw_rounds", "64lanes_full", "uniform_full"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int nblk : {64, 1024}) {
      double best_ns = 1e30, cyc = 0;
      for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, nblk, d);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        uint64_t h[3];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        const double ns = h[0] * 10.0;
        if (ns < best_ns) {
          best_ns = ns;
          cyc = static_cast<double>(h[1]);
        }
      }
      std::printf("{\"mode\": \"%s\", \"blocks\": %d, \"ns_per_block\": %.1f, \"memtime_ticks_per_block\": %.1f, "
                  "\"memtime_MHz\": %.0f}\n",
                  names[mode], nblk, best_ns / nblk, cyc / nblk, cyc / best_ns * 1e3);
    }
  }
  hipFree(d);
  return 0;
}
