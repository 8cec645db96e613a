// WordWindowSink: per-lane SHA-256 of an emitted message, assembled in LDS one
// 32-bit word at a time.
//
// The message is produced by an *emitter* (ahv/delta_emit.h) that hands over
// big-endian chunks of 1–4 bytes and announces each segment's byte length
// first.  Each lane keeps a funnel: the `sh/8` pending bytes of the word being
// filled sit left-aligned in `carry`; a 4-byte chunk v always completes exactly
// one word, `carry | v >> sh`, and leaves `v << (32 - sh)` pending (one
// v_alignbit).  So a 4-byte chunk costs ~3 VALU + one ds_write_b32 whatever the
// lane's byte phase — lanes whose messages are shifted by a different DID
// length run the same instructions.
//
// Hashing runs in passes over a window of kWinBlocks SHA blocks:
//
//   pass k: zero the window; run the emitter — words whose index falls in the
//           window land in LDS, all others in a trash row (an unsigned min, no
//           branch), segments wholly before or after the window are skipped by
//           length for every lane at once (`__all`); flush the pending word
//           with the 0x80 pad byte, write the bit length; compress the
//           window's blocks that belong to the lane's padded message.
//
// A ~330-byte governance delta (6 blocks) takes 2 passes with a 3-block window.
// There is one compression site in the loop (a kernel with several inlined
// 64-round compressions overflows the VGPR budget and the instruction cache).
//
// LDS layout [word][lane] (word w of lane l at dword w*64 + l, row kWinWords is
// the trash row): every ds_write_b32 / ds_read_b32 of a wave touches 64
// consecutive dwords — conflict-free.
#pragma once

#include "ahv/delta_emit.h"
#include "ahv/sha256.h"

namespace ahv {

#ifndef AHV_WIN_BLOCKS
#define AHV_WIN_BLOCKS 3
#endif
constexpr int kWinBlocks = AHV_WIN_BLOCKS;
constexpr int kWinWords = kWinBlocks * 16;
constexpr int kWaveLanes = 64;

static __shared__ uint32_t g_win[(kWinWords + 1) * kWaveLanes];

struct WordWindowSink {
  uint32_t lane;
  int32_t rel;     // index of the word being filled, relative to the window start
  uint32_t sh;     // 8 × bytes pending in `carry` (0, 8, 16, 24)
  uint32_t carry;  // pending bytes, left-aligned
  int32_t lo;      // window start (word index), wave-uniform

  __device__ __forceinline__ void store(int32_t r, uint32_t v) const {
    const uint32_t u = static_cast<uint32_t>(r);  // negative → huge → trash row
    const uint32_t slot = u < static_cast<uint32_t>(kWinWords) ? u : static_cast<uint32_t>(kWinWords);
    g_win[slot * kWaveLanes + lane] = v;
  }

  // Segment of `len` bytes: false (and the position advanced) when it lies
  // wholly outside the window for every lane of the wave.
  __device__ __forceinline__ bool seg(uint32_t len) {
    const uint32_t tot = (sh >> 3) + len;
    const int32_t last = rel + static_cast<int32_t>((tot - 1) >> 2);  // word holding the last byte
    if (__all(last < 0 || rel >= kWinWords)) {
      rel += static_cast<int32_t>(tot >> 2);
      sh = (tot & 3u) << 3;
      carry = 0;  // its word is outside the window
      return false;
    }
    return true;
  }

  __device__ __forceinline__ void put4(uint32_t v) {
    store(rel, carry | (v >> sh));
    carry = __builtin_amdgcn_alignbit(v, 0u, sh);
    ++rel;
  }

  // n ∈ [0, 4] bytes (top of v, rest zero); n may differ per lane.
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    const uint32_t w = carry | (v >> sh);
    const uint32_t tot = sh + 8u * n;
    const bool full = tot >= 32u;
    store(full ? rel : kWinWords, w);
    carry = full ? __builtin_amdgcn_alignbit(v, 0u, sh) : w;
    rel += full ? 1 : 0;
    sh = tot & 31u;
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
  // or resumption (MID_RESUME: start from mid at word 16, skipping block 0's
  // emission and compression).  The mode is wave-uniform.
  template <class Emit>
  __device__ __forceinline__ void hash_mid(Emit&& emit, uint32_t out[8], Digest& mid, int mode) {
    uint32_t st[8];
    if (mode == MID_RESUME) {
#pragma unroll
      for (int k = 0; k < 8; ++k) st[k] = mid.v[k];
      lo = 16;
    } else {
      sha256_init(st);
      lo = 0;
    }
    int32_t total = 0;  // padded length in words, known after the first pass
    bool first = true;
    while (first || __any(lo < total)) {
#pragma unroll
      for (int k = 0; k < kWinWords; ++k) g_win[k * kWaveLanes + lane] = 0u;
      rel = -lo;
      sh = 0;
      carry = 0;
      emit(*this);
      const uint32_t L = static_cast<uint32_t>(rel + lo) * 4u + (sh >> 3);  // message bytes
      total = static_cast<int32_t>(((L + 8u) / 64u + 1u) * 16u);
      // pad byte, flushed with the pending word (the zeroed window supplies the rest)
      put(0x80000000u, 1);
      store(sh ? rel : kWinWords, carry);
      const uint64_t bits = static_cast<uint64_t>(L) * 8u;
      store(total - 2 - lo, static_cast<uint32_t>(bits >> 32));
      store(total - 1 - lo, static_cast<uint32_t>(bits));
#pragma nounroll
      for (int blk = 0; blk < kWinBlocks; ++blk) {
        if (lo + 16 * blk < total) {
          uint32_t w[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) w[k] = g_win[(blk * 16 + k) * kWaveLanes + lane];
          sha256_compress(st, w);
          if (mode == MID_CAPTURE && lo == 0 && blk == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mid.v[k] = st[k];
          }
        }
      }
      first = false;
      lo += kWinWords;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
  }

  // Merkle digest scratch: slot j (< kWinWords / 8) lives in window words 8j..8j+7.
  __device__ __forceinline__ void stash(int j, const uint32_t d[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g_win[(8 * j + k) * kWaveLanes + lane] = d[k];
  }
  __device__ __forceinline__ void load(int j, uint32_t d[8]) const {
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = g_win[(8 * j + k) * kWaveLanes + lane];
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
