// WaveWindowSink: per-lane SHA-256 of an emitted message, assembled in LDS.
//
// The message is produced by an *emitter* (ahv/delta_emit.h) that knows each
// segment's length before writing it.  Hashing runs in passes over a 4-block
// (256-byte) window per lane:
//
//   pass k: run the emitter; bytes whose position falls in [256k, 256k+256) are
//           stored to LDS, whole segments outside the window are skipped by
//           length (no per-byte work); append the SHA padding bytes that fall
//           in the window; compress the window's complete blocks.
//
// Typical governance deltas (≈ 330 bytes → 6 blocks) take two passes.  The
// point of the design is code shape on CDNA: there is exactly one compression
// site in the loop (a kernel with many inlined 64-round compressions blew the
// VGPR budget; non-inlined calls spilled around every call site), every lane
// runs the same loop trip count (wave-uniform `__any`), and lanes whose messages
// differ in length only mask the tail blocks.
//
// LDS layout [word][lane] (word w of lane l at dword w*64 + l): a wave-wide
// ds_write_b8 touches 64 distinct dwords on bank l mod 32 — conflict-free — and
// block reads are conflict-free ds_read_b32.  16 KiB per wave → 10 waves/CU.
#pragma once

#include "ahv/delta_emit.h"
#include "ahv/sha256.h"

namespace ahv {

// 2 blocks (8 KiB of LDS per wave) keeps LDS from capping occupancy below what
// the VGPR budget allows (3 waves/SIMD at ≤ 168 VGPRs); each extra pass only
// re-walks the segment lengths, its bytes outside the window are skipped whole.
constexpr int kWinBlocks = 2;
constexpr uint32_t kWinBytes = kWinBlocks * 64;  // 128
constexpr int kWinWords = kWinBlocks * 16;       // 32
constexpr int kWaveLanes = 64;

static __shared__ uint32_t g_ring[kWinWords * kWaveLanes];

struct WaveWindowSink {
  uint32_t lane;
  uint32_t pos;  // position of the next emitted byte
  uint32_t lo;   // window start of the current pass

  // Does the next `len` bytes overlap the window?  If not, skip them.
  __device__ __forceinline__ bool want(uint32_t len) {
    if (pos + len > lo && pos < lo + kWinBytes) return true;
    pos += len;
    return false;
  }

  __device__ __forceinline__ void byte(uint8_t b) {
    const uint32_t rel = pos - lo;
    if (rel < kWinBytes)
      reinterpret_cast<uint8_t*>(g_ring)[(((rel >> 2) * kWaveLanes + lane) << 2) + (3u - (rel & 3u))] = b;
    ++pos;
  }

  __device__ __forceinline__ bool any(bool b) const { return __any(b); }

  // Make a value opaque to loop-invariant code motion (see emit_delta_payload).
  __device__ __forceinline__ void launder(uint32_t& x) const { asm volatile("" : "+v"(x)); }
  __device__ __forceinline__ void launder(int32_t& x) const { asm volatile("" : "+v"(x)); }
  __device__ __forceinline__ void launder(int64_t& x) const { asm volatile("" : "+v"(x)); }

  // Hash the message produced by `emit(*this)`.
  template <class Emit>
  __device__ __forceinline__ void hash(Emit&& emit, uint32_t out[8]) {
    Digest unused;
    hash_mid(emit, out, unused, MID_OFF);
  }

  // As hash(), with midstate capture (MID_CAPTURE: state after block 0 → mid)
  // or resumption (MID_RESUME: start from mid at byte 64, skipping block 0's
  // emission and compression).  The mode may differ per lane.
  template <class Emit>
  __device__ __forceinline__ void hash_mid(Emit&& emit, uint32_t out[8], Digest& mid, int mode) {
    uint32_t st[8];
    if (mode == MID_RESUME) {
#pragma unroll
      for (int k = 0; k < 8; ++k) st[k] = mid.v[k];
      lo = 64;
    } else {
      sha256_init(st);
      lo = 0;
    }
    uint32_t total = 0;  // padded length, known after the first pass
    bool first = true;
    while (first || __any(lo < total)) {
      if (first || lo < total) {
        pos = 0;
        emit(*this);
        const uint32_t L = pos;
        total = ((L + 8u) / 64u + 1u) * 64u;
        // padding bytes [L, total) that fall in this window
        const uint32_t a = L > lo ? L : lo;
        const uint32_t e = total < lo + kWinBytes ? total : lo + kWinBytes;
        const uint64_t bits = static_cast<uint64_t>(L) * 8u;
        for (uint32_t p = a; p < e; ++p) {
          uint8_t b = 0;
          if (p == L) b = 0x80;
          else if (p >= total - 8) b = static_cast<uint8_t>(bits >> (8 * (total - 1 - p)));
          pos = p;
          byte(b);
        }
        // complete blocks of this window
        const uint32_t nb = ((e > lo ? e : lo) - lo) >> 6;
        for (uint32_t blk = 0; blk < nb; ++blk) {
          uint32_t w[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) w[k] = g_ring[(blk * 16 + k) * kWaveLanes + lane];
          sha256_compress(st, w);
          if (mode == MID_CAPTURE && lo == 0 && blk == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mid.v[k] = st[k];
          }
        }
      }
      first = false;
      lo += kWinBytes;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
  }

  // Merkle digest scratch: slot j (< 8) lives in window words 8j..8j+7.
  __device__ __forceinline__ void stash(int j, const uint32_t d[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g_ring[(8 * j + k) * kWaveLanes + lane] = d[k];
  }
  __device__ __forceinline__ void load(int j, uint32_t d[8]) const {
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = g_ring[(8 * j + k) * kWaveLanes + lane];
  }
  // Merkle interior node: two data blocks (hex of l, hex of r) share one loop
  // body; the third is the constant padding block of a 128-byte message, whose
  // message schedule (and K+W sums) the compiler folds to immediates.
  __device__ __forceinline__ void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) const {
    uint32_t st[8];
    sha256_init(st);
#pragma nounroll
    for (int blk = 0; blk < 2; ++blk) {
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 8; ++k) word_to_hex_words(blk == 0 ? l[k] : r[k], w[2 * k], w[2 * k + 1]);
      sha256_compress(st, w);
    }
    sha256_compress_pad_only(st, 128);
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
  }
};

}  // namespace ahv
