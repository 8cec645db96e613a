// Host SHA-256 (SHA-NI when the CPU has it, else the shared ahv/sha256.h core)
// and the reference Merkle node, for the host runtime: the scalar audit API
// (py_audit.cpp) and the store's host-side digest predictions (py_store.cpp).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "ahv/sha256.h"

extern "C" int ahv_cpu_has_sha_ni();
extern "C" void ahv_sha256_ni_blocks(uint32_t st[8], const uint8_t* data, size_t nblocks);

namespace ahv {
namespace host {

inline bool sha_ni() {
  static const bool v = ahv_cpu_has_sha_ni() != 0;
  return v;
}

// Compress whole 64-byte blocks with SHA-NI when present, else the shared core.
inline void compress_blocks(uint32_t st[8], const uint8_t* p, size_t nblocks) {
  if (sha_ni()) {
    ahv_sha256_ni_blocks(st, p, nblocks);
    return;
  }
  for (size_t b = 0; b < nblocks; ++b, p += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t(p[4 * i]) << 24) | (uint32_t(p[4 * i + 1]) << 16) |
             (uint32_t(p[4 * i + 2]) << 8) | uint32_t(p[4 * i + 3]);
    sha256_compress(st, w);
  }
}

inline void sha256_bytes(const uint8_t* p, size_t n, uint32_t out[8]) {
  sha256_init(out);
  const size_t full = n / 64;
  compress_blocks(out, p, full);
  uint8_t tail[128];
  const size_t r = n - full * 64;
  std::memcpy(tail, p + full * 64, r);
  tail[r] = 0x80;
  const size_t padded = (r < 56) ? 64 : 128;
  std::memset(tail + r + 1, 0, padded - r - 1);
  const uint64_t bits = uint64_t(n) * 8u;
  for (int i = 0; i < 8; ++i) tail[padded - 1 - i] = static_cast<uint8_t>(bits >> (8 * i));
  compress_blocks(out, tail, padded / 64);
}

inline void hex_bytes(const uint32_t d[8], uint8_t out[64]) {
  static const char* digits = "0123456789abcdef";
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = static_cast<uint8_t>(digits[(d[i] >> (28 - 4 * j)) & 15u]);
}

// Merkle interior node over two digests: sha256(hex(l) || hex(r)), 3 blocks.
inline void merkle_node_host(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) {
  alignas(16) uint8_t buf[192];
  hex_bytes(l, buf);
  hex_bytes(r, buf + 64);
  std::memset(buf + 128, 0, 64);
  buf[128] = 0x80;
  buf[190] = 0x04;  // 1024 bits
  sha256_init(out);
  compress_blocks(out, buf, 3);
}

// Reference Merkle root over n digests (odd node paired with itself), in place.
inline void merkle_root_host(uint32_t* level, size_t n, uint32_t out[8]) {
  size_t m = n;
  while (m > 1) {
    const size_t half = (m + 1) / 2;
    for (size_t i = 0; i < half; ++i) {
      const uint32_t* l = level + 16 * i;
      const uint32_t* r = (2 * i + 1 < m) ? level + 16 * i + 8 : l;
      uint32_t o[8];
      merkle_node_host(l, r, o);
      std::memcpy(level + 8 * i, o, sizeof o);
    }
    m = half;
  }
  std::memcpy(out, level, 32);
}

}  // namespace host
}  // namespace ahv
