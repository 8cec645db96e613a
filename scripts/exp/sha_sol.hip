// Experiment: SHA-256 compression speed-of-light on gfx950.
//
// Each lane runs `iters` dependent compressions on register-resident state
// (the message block is derived from the state so nothing folds away).
// Variants: fully unrolled 64 rounds vs a 16-round body looped 4x (small
// code), and 1..8 waves per SIMD via __launch_bounds__.
//
//   hipcc --offload-arch=gfx950 -O3 -I csrc/include scripts/exp/sha_sol.hip -o /tmp/sha_sol
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ahv/sha256.h"

using namespace ahv;

__constant__ uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

// 16 rounds with the schedule step folded in when `expand` (rounds 16..63).
template <bool Expand>
__device__ __forceinline__ void rounds16(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                         uint32_t& f, uint32_t& g, uint32_t& h, uint32_t w[16],
                                         const uint32_t* K) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (Expand) {
      const uint32_t x = w[(i + 1) & 15];
      const uint32_t y = w[(i + 14) & 15];
      const uint32_t s0 = xor3(rotr32(x, 7), rotr32(x, 18), x >> 3);
      const uint32_t s1 = xor3(rotr32(y, 17), rotr32(y, 19), y >> 10);
      w[i] = w[i] + s0 + w[(i + 9) & 15] + s1;
    }
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t t1 = h + S1 + sha_ch(e, f, g) + K[i] + w[i];
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t t2 = S0 + sha_maj(a, b, c);
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
  }
}

__device__ __forceinline__ void compress_looped(uint32_t st[8], const uint32_t blk[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  rounds16<false>(a, b, c, d, e, f, g, h, w, kK);
#pragma nounroll
  for (int r = 1; r < 4; ++r) rounds16<true>(a, b, c, d, e, f, g, h, w, kK + 16 * r);
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

template <int Waves, bool Looped>
__global__ __launch_bounds__(64, Waves) void sol_kernel(uint32_t* out, int iters) {
  uint32_t st[8];
  sha256_init(st);
  st[0] ^= blockIdx.x * 64 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    uint32_t blk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) blk[k] = st[k & 7] ^ (k * 0x9e3779b9u);
    if (Looped) compress_looped(st, blk);
    else sha256_compress(st, blk);
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= st[k];
  out[blockIdx.x * 64 + threadIdx.x] = x;
}

template <int Waves, bool Looped>
void run(uint32_t* d, int blocks, int iters, int per_simd = 0) {
  // cap residency with dynamic LDS: 160 KiB per CU / (4 SIMDs x per_simd waves)
  const size_t lds = per_simd ? (160u * 1024u) / (4u * per_simd) + 64 : 0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((sol_kernel<Waves, Looped>), dim3(blocks), dim3(64), lds, 0, d, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((sol_kernel<Waves, Looped>), dim3(blocks), dim3(64), lds, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double comps = double(blocks) * 64 * iters;
  printf("cap=%d/SIMD waves/SIMD>=%d %-8s blocks=%d iters=%d  %.3f ms  %.2f G compressions/s\n", per_simd, Waves,
         Looped ? "looped" : "unrolled", blocks, iters, ms, comps / ms / 1e6);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 16384;
  const int iters = argc > 2 ? atoi(argv[2]) : 24;
  uint32_t* d;
  hipMalloc(&d, size_t(blocks) * 64 * 4);
  for (int cap : {1, 2, 3, 4, 0}) {
    run<4, false>(d, blocks, iters, cap);
    run<8, false>(d, blocks, iters, cap);
    run<4, true>(d, blocks, iters, cap);
  }
  hipFree(d);
  return 0;
}
