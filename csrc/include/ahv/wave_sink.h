// WordWindowSink: per-lane SHA-256 of an emitted message, assembled in LDS one
// 32-bit word at a time.
//
// The message is produced by an *emitter* (ahv/delta_emit.h) that hands over
// big-endian chunks of 1–4 bytes and announces each segment's byte length
// first.  Each lane keeps a funnel: the `sh/8` pending bytes of the word being
// filled sit right-aligned in `prev` (the tail of the previous chunk); a 4-byte
// chunk v always completes exactly one word, ({prev, v} >> sh)[31:0] — a single
// v_alignbit — and leaves its own tail pending (`prev = v`).  So a 4-byte chunk
// costs ~3 VALU (funnel, trash clamp, address step) + one ds_write_b32 whatever
// the lane's byte phase — lanes whose messages are shifted by a different DID
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

constexpr int kWaveLanes = 64;

// The window of one wave: (W·16 + 1) rows of 64 lanes (one LDS array per
// window size; a kernel instantiates exactly one).
template <int WinBlocks>
__device__ __forceinline__ uint32_t* win_lds() {
  __shared__ uint32_t buf[(WinBlocks * 16 + 1) * kWaveLanes];
  return buf;
}

template <int WinBlocks>
struct WordWindowSink {
  static constexpr int kWinBlocks = WinBlocks;
  static constexpr int kWinWords = WinBlocks * 16;
  uint32_t* g_win;  // win_lds<WinBlocks>()
  uint32_t lane;
  int32_t rel;     // index of the word being filled, relative to the window start
  uint32_t addr;   // its LDS byte offset, (rel·64 + lane)·4 mod 2^32 (negative rel wraps high)
  uint32_t trash;  // (kWinWords·64 + lane)·4, this lane's trash-row offset
  uint32_t sh;     // 8 × bytes pending (0, 8, 16, 24)
  uint32_t prev;   // the pending bytes, RIGHT-aligned (the tail of the last chunk)
  int32_t lo;      // window start (word index); per lane: a record resumed from a midstate starts at 16

  // Word at LDS byte offset `a` (already relative to the window); anything
  // outside [0, kWinWords) rows — including wrapped negatives — hits the trash row.
  __device__ __forceinline__ void store_at(uint32_t a, uint32_t v) const {
    const uint32_t c = a < trash ? a : trash;
    *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(g_win) + c) = v;
  }
  __device__ __forceinline__ void store(int32_t r, uint32_t v) const {
    store_at((static_cast<uint32_t>(r) * kWaveLanes + lane) * 4u, v);
  }
  __device__ __forceinline__ void seek(int32_t r) {
    rel = r;
    addr = (static_cast<uint32_t>(r) * kWaveLanes + lane) * 4u;
  }

  // Segment of `len` bytes: false (and the position advanced) when it lies
  // wholly outside the window for every lane of the wave.
  __device__ __forceinline__ bool seg(uint32_t len) {
    const uint32_t tot = (sh >> 3) + len;
    const int32_t last = rel + static_cast<int32_t>((tot - 1) >> 2);  // word holding the last byte
    if (__all(last < 0 || rel >= kWinWords)) {
      seek(rel + static_cast<int32_t>(tot >> 2));
      sh = (tot & 3u) << 3;  // `prev` is stale, but its word lies outside the window
      return false;
    }
    return true;
  }

  // Funnel: the completed word is the pending sh/8 bytes followed by the head of
  // v, i.e. ({prev, v} >> sh)[31:0] — one v_alignbit; the new pending bytes are
  // the tail of v, so `prev = v`.
  __device__ __forceinline__ void put4(uint32_t v) {
    store_at(addr, __builtin_amdgcn_alignbit(prev, v, sh));
    prev = v;
    ++rel;
    addr += kWaveLanes * 4u;
  }

  // n ∈ [0, 4] bytes at the top of v (the low bytes of v are ignored); n may
  // differ per lane.  The pending tail becomes ({prev, v} >> (32 − 8n))[31:0].
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    const uint32_t tot = sh + 8u * n;
    const bool full = tot >= 32u;
    store_at(full ? addr : trash, __builtin_amdgcn_alignbit(prev, v, sh));
    prev = n ? __builtin_amdgcn_alignbit(prev, v, 32u - 8u * n) : prev;
    rel += full ? 1 : 0;
    addr += full ? kWaveLanes * 4u : 0u;
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
    run(emit, st, 0u, out, mid, mode);
  }

  // Resume from an arbitrary midstate `st_in` taken after `base_bytes` (a
  // multiple of 64, per lane) of message that the emitter does NOT replay: the
  // emitter produces only the remaining bytes; the bit length counts both.
  template <class Emit>
  __device__ __forceinline__ void hash_from(Emit&& emit, const uint32_t st_in[8], uint32_t base_bytes,
                                            uint32_t out[8]) {
    uint32_t st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) st[k] = st_in[k];
    lo = 0;
    Digest unused;
    run(emit, st, base_bytes, out, unused, MID_OFF);
  }

  template <class Emit>
  __device__ __forceinline__ void run(Emit&& emit, uint32_t st[8], uint32_t base_bytes, uint32_t out[8],
                                      Digest& mid, int mode) {
    int32_t total = 0;  // padded length in words, known after the first pass
    bool first = true;
    while (first || __any(lo < total)) {
#pragma unroll
      for (int k = 0; k < kWinWords; ++k) g_win[k * kWaveLanes + lane] = 0u;
      trash = (static_cast<uint32_t>(kWinWords) * kWaveLanes + lane) * 4u;
      seek(-lo);
      sh = 0;
      prev = 0;
      emit(*this);
      const uint32_t L = static_cast<uint32_t>(rel + lo) * 4u + (sh >> 3);  // message bytes
      total = static_cast<int32_t>(((L + 8u) / 64u + 1u) * 16u);
      // pad byte, then the pending word flushed left-aligned (the zeroed window
      // supplies the zero bytes up to the length words)
      put(0x80000000u, 1);
      store_at(sh ? addr : trash, __builtin_amdgcn_alignbit(prev, 0u, sh));
      const uint64_t bits = (static_cast<uint64_t>(L) + base_bytes) * 8u;
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

  // Render the whole message `emit(*this)` into the window (one pass: it must fit
  // in kWinBlocks blocks) with its SHA padding and bit length, without hashing it.
  // Returns the padded length in words; `len` = message bytes.
  template <class Emit>
  __device__ __forceinline__ int32_t render(Emit&& emit, uint32_t& len) {
#pragma unroll
    for (int k = 0; k < kWinWords; ++k) g_win[k * kWaveLanes + lane] = 0u;
    trash = (static_cast<uint32_t>(kWinWords) * kWaveLanes + lane) * 4u;
    lo = 0;
    seek(0);
    sh = 0;
    prev = 0;
    emit(*this);
    const uint32_t L = static_cast<uint32_t>(rel) * 4u + (sh >> 3);
    const int32_t total = static_cast<int32_t>(((L + 8u) / 64u + 1u) * 16u);
    put(0x80000000u, 1);
    store_at(sh ? addr : trash, __builtin_amdgcn_alignbit(prev, 0u, sh));
    const uint64_t bits = static_cast<uint64_t>(L) * 8u;
    store(total - 2, static_cast<uint32_t>(bits >> 32));
    store(total - 1, static_cast<uint32_t>(bits));
    len = L;
    return total;
  }

  // Compress window blocks [b0, b1) (per lane) into `st`: one compression site.
  __device__ __forceinline__ void compress_blocks(uint32_t st[8], int32_t b0, int32_t b1) const {
#pragma nounroll
    for (int blk = 0; blk < kWinBlocks; ++blk) {
      if (blk >= b0 && blk < b1) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = g_win[(blk * 16 + k) * kWaveLanes + lane];
        sha256_compress(st, w);
      }
    }
  }

  // Overwrite the 64 hex chars at byte `at` of the rendered message (the quoted
  // parent digest's inside, rendered as a placeholder) with the hex of `d`.
  __device__ __forceinline__ void patch_hex(uint32_t at, const uint32_t d[8]) const {
    uint32_t hw[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) word_to_hex_words(d[k], hw[2 * k], hw[2 * k + 1]);
    const uint32_t sh8 = (at & 3u) * 8u;
    const uint32_t base = at >> 2;
    uint32_t* col = g_win + lane;
    const uint32_t keep = sh8 ? ~(0xffffffffu >> sh8) : 0u;  // bytes before `at` in the first word
    uint32_t w0 = col[base * kWaveLanes];
    col[base * kWaveLanes] = (w0 & keep) | (sh8 ? hw[0] >> sh8 : hw[0]);
#pragma unroll
    for (int j = 1; j < 16; ++j) col[(base + j) * kWaveLanes] = __builtin_amdgcn_alignbit(hw[j - 1], hw[j], sh8);
    if (sh8) {  // the last word keeps the bytes after the hex
      const uint32_t w16 = col[(base + 16) * kWaveLanes];
      col[(base + 16) * kWaveLanes] = (hw[15] << (32u - sh8)) | (w16 & (0xffffffffu >> sh8));
    }
  }

  // Store the rendered message's bytes (memory order) at `dst` (16-byte aligned):
  // `nw` words, per lane.
  __device__ __forceinline__ void tee(uint32_t* dst, int32_t nw) const {
#pragma nounroll
    for (int k = 0; k < kWinWords; k += 4) {
      if (k < nw) {
        const uint32_t* w = g_win + k * kWaveLanes + lane;
        *reinterpret_cast<uint4*>(dst + k) =
            make_uint4(bswap_word(w[0]), bswap_word(w[kWaveLanes]), bswap_word(w[2 * kWaveLanes]),
                       bswap_word(w[3 * kWaveLanes]));
      }
    }
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
