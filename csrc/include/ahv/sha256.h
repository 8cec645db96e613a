// SHA-256 (FIPS 180-4), written once for host and gfx950.
//
// Used by every hashing path of the audit subsystem:
//   * SemanticDelta.compute_hash   (reference audit/delta.py:41-64)
//   * DeltaEngine.compute_merkle_root (reference audit/delta.py:117-134)
//   * SessionVFS content hashes    (reference session/sso.py:214-216)
//   * SemanticCheckpoint goal hash (reference saga/checkpoint.py:32-36)
//
// Device notes (CDNA4): the 64 rounds are fully unrolled with a 16-word rolling
// message schedule so that the whole state lives in VGPRs; rotations lower to
// v_alignbit_b32, Ch/Maj to v_bfi_b32, the round adds to v_add3_u32.  A block
// whose words are compile-time constants (SHA padding blocks of fixed-length
// messages, e.g. the 3rd block of every 128-byte Merkle node) has its message
// expansion constant-folded by the compiler.
#pragma once

#include "ahv/hd.h"

namespace ahv {

AHV_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// 3-input XOR: one v_bitop3_b32 (truth table 0x96) on gfx950; LLVM otherwise
// emits two v_xor_b32 for every Σ/σ function (~13 % of a compression).
AHV_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// Ch(e, f, g) = e ? f : g  (bitop3 truth table 0xCA, index = e·4 + f·2 + g)
AHV_HD uint32_t sha_ch(uint32_t e, uint32_t f, uint32_t g) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
#else
  return (e & f) ^ (~e & g);
#endif
}

// Maj(a, b, c) = majority  (truth table 0xE8)
AHV_HD uint32_t sha_maj(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
#else
  return (a & b) ^ (a & c) ^ (b & c);
#endif
}

AHV_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0x0000ff00u) | ((x << 8) & 0x00ff0000u) | (x << 24);
}

AHV_HD void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

AHV_HD uint32_t sha256_k(int i) {
  constexpr uint32_t K[64] = {
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
  return K[i];
}

// One compression.  `blk` holds the 16 big-endian message words.
AHV_HD void sha256_compress(uint32_t st[8], const uint32_t blk[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      const uint32_t x = w[(i + 1) & 15];
      const uint32_t y = w[(i + 14) & 15];
      const uint32_t s0 = xor3(rotr32(x, 7), rotr32(x, 18), x >> 3);
      const uint32_t s1 = xor3(rotr32(y, 17), rotr32(y, 19), y >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t ch = sha_ch(e, f, g);
    const uint32_t t1 = h + S1 + ch + sha256_k(i) + wi;
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t maj = sha_maj(a, b, c);
    const uint32_t t2 = S0 + maj;
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Final padding block for a message whose length is an exact multiple of 64
// bytes: 0x80 then zeros then the 64-bit bit length.  All words are constants
// for a constant `total_bytes`, so the schedule folds away.
AHV_HD void sha256_compress_pad_only(uint32_t st[8], uint64_t total_bytes) {
  uint32_t w[16];
  w[0] = 0x80000000u;
#pragma unroll
  for (int i = 1; i < 14; ++i) w[i] = 0u;
  const uint64_t bits = total_bytes * 8u;
  w[14] = static_cast<uint32_t>(bits >> 32);
  w[15] = static_cast<uint32_t>(bits);
  sha256_compress(st, w);
}

// Lowercase hex of a nibble, as an ASCII byte.
AHV_HD uint32_t hex_nibble(uint32_t n) { return n + (n < 10u ? 0x30u : 0x57u); }

// Four hex chars from two bytes laid out as x = [Bh Bh Bl Bl] (SWAR): spread
// the nibbles to one per byte, then add '0' and, where the nibble is ≥ 10, the
// extra 0x27 that lands on 'a' — per byte, with no carry between bytes.
AHV_HD uint32_t hex4_spread(uint32_t x) {
  const uint32_t n = ((x >> 4) & 0x0F000F00u) | (x & 0x000F000Fu);
  const uint32_t m = ((n + 0x06060606u) >> 4) & 0x01010101u;
  // m·0x27 as shift-adds (full-rate v_lshl_add_u32, not a quarter-rate v_mul_lo_u32)
  const uint32_t m3 = (m << 1) + m, m7 = (m << 2) + m3;
  return n + 0x30303030u + (m << 5) + m7;
}

// Expand one digest word into 8 lowercase-hex ASCII chars packed as two
// big-endian message words (first char in the most significant byte).  On the
// device the byte duplication is one v_perm_b32 per half (~9 VALU per 4 chars
// instead of ~5 per char for the nibble-at-a-time form).
AHV_HD void word_to_hex_words(uint32_t v, uint32_t& hi, uint32_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  hi = hex4_spread(__builtin_amdgcn_perm(0u, v, 0x03030202u));
  lo = hex4_spread(__builtin_amdgcn_perm(0u, v, 0x01010000u));
#else
  const uint32_t b3 = v >> 24, b2 = (v >> 16) & 0xffu, b1 = (v >> 8) & 0xffu, b0 = v & 0xffu;
  hi = hex4_spread(b3 * 0x01010000u | b2 * 0x0101u);
  lo = hex4_spread(b1 * 0x01010000u | b0 * 0x0101u);
#endif
}

// Digest (8 words) -> 64 ASCII hex chars as 16 big-endian message words.
AHV_HD void digest_to_hex_words(const uint32_t d[8], uint32_t out[16]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) word_to_hex_words(d[i], out[2 * i], out[2 * i + 1]);
}

// Merkle interior node (reference audit/delta.py:128): sha256 over the ASCII of
// hex(left) || hex(right) = exactly 128 bytes = 2 data blocks + 1 pad block.
AHV_HD void merkle_node(const uint32_t left[8], const uint32_t right[8], uint32_t out[8]) {
  uint32_t blk[16];
  sha256_init(out);
  digest_to_hex_words(left, blk);
  sha256_compress(out, blk);
  digest_to_hex_words(right, blk);
  sha256_compress(out, blk);
  sha256_compress_pad_only(out, 128u);
}

// Byte-oriented streaming hasher (host and device).  Used where messages are
// assembled byte-by-byte; the batched device kernels assemble whole words in
// LDS instead (see csrc/hip/audit_kernels.hip).
struct Sha256Stream {
  uint32_t st[8];
  uint32_t blk[16];
  uint32_t fill;   // bytes in the current block
  uint64_t total;  // bytes consumed

  AHV_HD void init() {
    sha256_init(st);
    fill = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) blk[i] = 0;
  }

  AHV_HD void put(uint8_t byte) {
    const uint32_t wi = fill >> 2;
    const uint32_t sh = 24u - 8u * (fill & 3u);
    blk[wi] = (fill & 3u) ? (blk[wi] | (uint32_t(byte) << sh)) : (uint32_t(byte) << sh);
    ++fill;
    ++total;
    if (fill == 64) {
      sha256_compress(st, blk);
      fill = 0;
    }
  }

  AHV_HD void update(const uint8_t* p, size_t n) {
    // Fast path: whole blocks straight from the input once aligned to a block.
    while (n && fill) { put(*p++); --n; }
    while (n >= 64) {
      uint32_t w[16];
      for (int i = 0; i < 16; ++i)
        w[i] = (uint32_t(p[4 * i]) << 24) | (uint32_t(p[4 * i + 1]) << 16) |
               (uint32_t(p[4 * i + 2]) << 8) | uint32_t(p[4 * i + 3]);
      sha256_compress(st, w);
      p += 64;
      n -= 64;
      total += 64;
    }
    while (n) { put(*p++); --n; }
  }

  AHV_HD void final(uint32_t out[8]) {
    const uint64_t bits = total * 8u;
    put(0x80);
    while (fill != 56) put(0x00);
    for (int i = 7; i >= 0; --i) put(static_cast<uint8_t>(bits >> (8 * i)));
    for (int i = 0; i < 8; ++i) out[i] = st[i];
  }
};

}  // namespace ahv
