// Host-CPU SHA-256 using the x86 SHA extensions (SHA-NI), for the scalar API
// path (one delta hash per DeltaEngine.capture, Merkle nodes at terminate).
// Compiled as plain C++ (no offload); selected at runtime when the CPU reports
// the `sha` feature, otherwise the portable ahv/sha256.h code is used.
#include <immintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

extern "C" {

__attribute__((visibility("hidden"))) int ahv_cpu_has_sha_ni() {
  __builtin_cpu_init();
  return __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
}

// Process `nblocks` 64-byte blocks of `data` into state `st` (standard order).
__attribute__((visibility("hidden"), target("sha,sse4.1,ssse3"))) void ahv_sha256_ni_blocks(
    uint32_t st[8], const uint8_t* data, size_t nblocks) {
  const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i tmp = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[0]));
  __m128i state1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&st[4]));
  tmp = _mm_shuffle_epi32(tmp, 0xB1);          // CDAB
  state1 = _mm_shuffle_epi32(state1, 0x1B);    // EFGH
  __m128i state0 = _mm_alignr_epi8(tmp, state1, 8);  // ABEF
  state1 = _mm_blend_epi16(state1, tmp, 0xF0);       // CDGH

  alignas(16) static const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
      0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
      0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
      0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
      0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
      0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
      0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
      0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
      0xc67178f2u};

  while (nblocks--) {
    const __m128i abef_save = state0;
    const __m128i cdgh_save = state1;
    __m128i msg0 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 0)), MASK);
    __m128i msg1 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 16)), MASK);
    __m128i msg2 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 32)), MASK);
    __m128i msg3 = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(data + 48)), MASK);
    __m128i msgs[4] = {msg0, msg1, msg2, msg3};

#pragma GCC unroll 16
    for (int r = 0; r < 16; ++r) {
      __m128i& cur = msgs[r & 3];
      __m128i msg = _mm_add_epi32(cur, _mm_load_si128(reinterpret_cast<const __m128i*>(&K[4 * r])));
      state1 = _mm_sha256rnds2_epu32(state1, state0, msg);
      msg = _mm_shuffle_epi32(msg, 0x0E);
      state0 = _mm_sha256rnds2_epu32(state0, state1, msg);
      if (r >= 3 && r < 15) {
        // schedule the block 4 ahead: w[r+1] uses msgs[(r+1)&3] (= r-3) updated from r-2, r-1, r
        __m128i& nxt = msgs[(r + 1) & 3];
        const __m128i t = _mm_alignr_epi8(cur, msgs[(r + 3) & 3], 4);
        nxt = _mm_add_epi32(nxt, t);
        nxt = _mm_sha256msg2_epu32(nxt, cur);
      }
      if (r >= 1 && r < 13) {
        __m128i& prev = msgs[(r + 3) & 3];
        prev = _mm_sha256msg1_epu32(prev, cur);
      }
    }
    state0 = _mm_add_epi32(state0, abef_save);
    state1 = _mm_add_epi32(state1, cdgh_save);
    data += 64;
  }

  tmp = _mm_shuffle_epi32(state0, 0x1B);       // FEBA
  state1 = _mm_shuffle_epi32(state1, 0xB1);    // DCHG
  state0 = _mm_blend_epi16(tmp, state1, 0xF0); // DCBA
  state1 = _mm_alignr_epi8(state1, tmp, 8);    // ABEF -> HGFE
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[0]), state0);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(&st[4]), state1);
}

}  // extern "C"
