// Batched audit kernels: many-message SHA-256 (K11 content
// hashes, K12 goal hashes), segmented Merkle roots (K09) and non-mutating chain
// verification (K10) over canonical payloads stored in a byte arena.
//
// The standalone hash kernel reads each lane's message straight from global
// memory (aligned 16-byte loads with byte funnel-shifting for unaligned starts);
// the fused pipeline kernel (pipeline.hip) instead renders its payloads in LDS.
#include "ahv/delta_emit.h"
#include "ahv/kernels.h"
#include "ahv/launch.h"
#include "ahv/sha256.h"
#include "ahv/wave_sink.h"

namespace ahv {

namespace {
constexpr int kBlock = 256;
inline dim3 grid1(int64_t n, int per_block = kBlock) {
  const int64_t b = (n + per_block - 1) / per_block;
  return dim3(static_cast<uint32_t>(b > 0 ? b : 1));
}

// Byte i of the message as a big-endian-ready value (bounds-checked).
AHV_HD uint32_t msg_byte(const uint8_t* p, int64_t len, int64_t i) { return i < len ? p[i] : 0u; }

// SHA-256 of bytes [p, p+len) with standard padding; block words gathered from
// 4-byte loads where the message is aligned.
AHV_HD void sha256_span(const uint8_t* p, int64_t len, uint32_t out[8]) {
  sha256_init(out);
  const int64_t total = ((len + 8) / 64 + 1) * 64;
  const uint64_t bits = static_cast<uint64_t>(len) * 8u;
  for (int64_t b = 0; b < total; b += 64) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int64_t i = b + 4 * k;
      uint32_t v;
      if (i + 4 <= len && ((reinterpret_cast<uintptr_t>(p + i) & 3) == 0)) {
        v = bswap32(*reinterpret_cast<const uint32_t*>(p + i));
      } else {
        v = 0;
        for (int j = 0; j < 4; ++j) {
          const int64_t x = i + j;
          uint32_t byte;
          if (x < len) byte = p[x];
          else if (x == len) byte = 0x80;
          else if (x >= total - 8) byte = static_cast<uint32_t>((bits >> (8 * (total - 1 - x))) & 0xff);
          else byte = 0;
          v = (v << 8) | byte;
        }
      }
      w[k] = v;
    }
    sha256_compress(out, w);
  }
}
}  // namespace

// ------------------------------------------------------------ K11 / K12

AHV_HD void hash_many_elem(const HashManyArgs& a, int64_t i) {
  const int64_t o = a.offsets[i];
  sha256_span(a.bytes + o, a.offsets[i + 1] - o, a.digest + i * 8);
}
__global__ void hash_many_kernel(HashManyArgs a) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    hash_many_elem(a, i);
}
void launch_hash_many(const HashManyArgs& a, hipStream_t st) {
  if (a.n <= 0) return;
  hipLaunchKernelGGL(hash_many_kernel, grid1(a.n, 64), dim3(64), 0, st, a);
  check_hip(hipGetLastError(), "hash_many_kernel");
}
void hash_many_host(const HashManyArgs& a) { for (int64_t i = 0; i < a.n; ++i) hash_many_elem(a, i); }

// ------------------------------------------------------- payload rendering
// One workgroup per row, threads over its bytes: template byte, or a stamp digit
// (only the stamp's own bytes do the division), or a hex nibble.

// Stamp values of one row (uniform across the row's workgroup: computed once).
AHV_HD void render_stamp_values(const RenderArgs& a, int64_t id, uint64_t sv[kRenderMaxStamps]) {
  for (int k = 0; k < a.nstamp; ++k) {
    const int64_t m = a.stamp_mod[k];
    int64_t v = id;
    if (m > 0) {  // 32-bit remainder when both fit (64-bit division is a long software sequence)
      v = (id >= 0 && id <= 0x7fffffff && m <= 0x7fffffff)
              ? static_cast<int64_t>(static_cast<uint32_t>(id) % static_cast<uint32_t>(m))
              : id % m;
    }
    sv[k] = static_cast<uint64_t>(v + a.stamp_add[k]);
  }
}

AHV_HD uint32_t render_char(const RenderArgs& a, const uint8_t* tmpl, int64_t id, const uint64_t sv[kRenderMaxStamps],
                            int32_t j) {
  constexpr uint64_t kPow10[19] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                   100000000ull, 1000000000ull, 10000000000ull, 100000000000ull,
                                   1000000000000ull, 10000000000000ull, 100000000000000ull,
                                   1000000000000000ull, 10000000000000000ull, 100000000000000000ull,
                                   1000000000000000000ull};
  uint32_t c = tmpl[j];
  for (int k = 0; k < a.nstamp; ++k) {
    const int32_t p = j - a.stamp_pos[k];
    if (p >= 0 && p < a.stamp_width[k]) {
      const uint64_t v = sv[k], d = kPow10[a.stamp_width[k] - 1 - p];
      uint32_t digit;
      if ((v >> 32) == 0)  // 32-bit division whenever the value fits (stamps are short ids)
        digit = d > 0xffffffffull ? 0u : (static_cast<uint32_t>(v) / static_cast<uint32_t>(d)) % 10u;
      else
        digit = static_cast<uint32_t>((v / d) % 10u);
      c = '0' + digit;
    }
  }
  if (a.hex_pos >= 0) {
    const int32_t p = j - a.hex_pos;
    if (p >= 0 && p < 2 * a.hex_bytes) {
      const uint32_t b = a.hex_src[id * a.hex_stride + (p >> 1)];
      c = hex_nibble((p & 1) ? (b & 15u) : (b >> 4));
    }
  }
  return c;
}

// Rows are written a 32-bit word (4 chars) per thread when the rows are word
// aligned and the pitch leaves room for the last partial word.
// One wave per row (4 rows per 256-thread workgroup); the template is staged in
// LDS once per workgroup, so the only global reads per row are its id and hex
// source bytes (a wave's rows are latency-bound otherwise: dependent byte loads).
constexpr int kRenderRowsPerBlock = kBlock / 64;
constexpr int kRenderLdsTmpl = 4096;
__global__ __launch_bounds__(kBlock) void render_rows_kernel(RenderArgs a) {
  __shared__ uint8_t s_tmpl[kRenderLdsTmpl];
  const bool words = ((reinterpret_cast<uintptr_t>(a.out) | static_cast<uintptr_t>(a.pitch)) & 3u) == 0 &&
                     a.pitch >= ((a.len + 3) & ~3);
  const int lane = threadIdx.x & 63;
  const bool staged = a.len <= kRenderLdsTmpl;  // uniform
  if (staged) {
    for (int32_t j = threadIdx.x; j < a.len; j += kBlock) s_tmpl[j] = a.tmpl[j];
    __syncthreads();
  }
  const uint8_t* tmpl = staged ? s_tmpl : a.tmpl;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * kRenderRowsPerBlock + (threadIdx.x >> 6); r < a.rows;
       r += static_cast<int64_t>(gridDim.x) * kRenderRowsPerBlock) {
    const int64_t id = a.ids[r];
    uint64_t sv[kRenderMaxStamps];
    render_stamp_values(a, id, sv);
    uint8_t* row = a.out + id * a.pitch;
    if (words) {
      for (int32_t w = lane; 4 * w < a.len; w += 64) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int32_t j = 4 * w + b;
          if (j < a.len) v |= render_char(a, tmpl, id, sv, j) << (8 * b);
        }
        reinterpret_cast<uint32_t*>(row)[w] = v;
      }
    } else {
      for (int32_t j = lane; j < a.len; j += 64) row[j] = static_cast<uint8_t>(render_char(a, tmpl, id, sv, j));
    }
  }
}
// Fast path (word-aligned rows, len ≤ 2 KiB): each wave assembles its row in LDS
// — template words copied, then only the stamp digits (one lane per digit) and
// the hex field (one lane per source byte pair, 4 chars) overwritten — and
// streams the finished row out with word stores.  Per-byte ALU work only where
// the row differs from the template.  (A register form — lanes patching their own
// words, hex bytes handed over by shuffles — measured 95 µs vs 43 µs for config5's
// 40 k slash deltas: every lane pays the stamp/hex range tests for every byte.)
constexpr int kRenderFastLen = 2048;

// Wave-scope LDS hand-off: release/acquire fences plus the wave barrier.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ __launch_bounds__(kBlock) void render_rows_fast_kernel(RenderArgs a) {
  __shared__ uint32_t s_tmpl[kRenderFastLen / 4];
  __shared__ uint32_t s_row[kRenderRowsPerBlock][kRenderFastLen / 4];
  constexpr uint32_t kPow10[10] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u,
                                   1000000000u};
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int32_t nw = (a.len + 3) >> 2;
  uint8_t* tb = reinterpret_cast<uint8_t*>(s_tmpl);
  for (int32_t j = threadIdx.x; j < 4 * nw; j += kBlock) tb[j] = j < a.len ? a.tmpl[j] : uint8_t(0);
  __syncthreads();
  uint32_t* row = s_row[wave];
  uint8_t* rb = reinterpret_cast<uint8_t*>(row);
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kRenderRowsPerBlock; base < a.rows;
       base += static_cast<int64_t>(gridDim.x) * kRenderRowsPerBlock) {
    const int64_t r = base + wave;
    const bool act = r < a.rows;
    const int64_t id = act ? a.ids[r] : 0;
    if (act)
      for (int32_t w = lane; w < nw; w += 64) row[w] = s_tmpl[w];
    // each wave owns its row: a wave barrier orders the LDS phases (a wave's LDS
    // instructions execute in order; the barrier keeps the compiler from moving them)
    wave_lds_sync();
    if (act) {
      uint64_t sv[kRenderMaxStamps];
      render_stamp_values(a, id, sv);
      for (int k = 0; k < a.nstamp; ++k) {
        const int32_t wd = a.stamp_width[k];
        if (lane < wd) {
          const int32_t e = wd - 1 - lane;  // power of ten of this digit
          const uint64_t v = sv[k];
          uint32_t digit;
          if ((v >> 32) == 0) digit = e > 9 ? 0u : (static_cast<uint32_t>(v) / kPow10[e]) % 10u;
          else {
            uint64_t d = 1;
            for (int q = 0; q < e; ++q) d *= 10u;
            digit = static_cast<uint32_t>((v / d) % 10u);
          }
          rb[a.stamp_pos[k] + lane] = static_cast<uint8_t>('0' + digit);
        }
      }
      if (a.hex_pos >= 0) {
        const uint8_t* src = a.hex_src + id * a.hex_stride;
        for (int32_t q = lane; 2 * q < a.hex_bytes; q += 64) {
          const uint32_t b0 = src[2 * q];
          const bool two = 2 * q + 1 < a.hex_bytes;
          const uint32_t b1 = two ? src[2 * q + 1] : 0u;
          uint8_t* o = rb + a.hex_pos + 4 * q;
          o[0] = static_cast<uint8_t>(hex_nibble(b0 >> 4));
          o[1] = static_cast<uint8_t>(hex_nibble(b0 & 15u));
          if (two) {
            o[2] = static_cast<uint8_t>(hex_nibble(b1 >> 4));
            o[3] = static_cast<uint8_t>(hex_nibble(b1 & 15u));
          }
        }
      }
    }
    wave_lds_sync();
    if (act) {
      uint32_t* dst = reinterpret_cast<uint32_t*>(a.out + id * a.pitch);
      for (int32_t w = lane; w < nw; w += 64) dst[w] = row[w];
    }
    wave_lds_sync();
  }
}

void launch_render_rows(const RenderArgs& a, hipStream_t st) {
  if (a.rows <= 0 || a.len <= 0) return;
  const int64_t need = (a.rows + kRenderRowsPerBlock - 1) / kRenderRowsPerBlock;
  const int64_t blocks = need < 65536 ? need : 65536;
  const bool fast = ((reinterpret_cast<uintptr_t>(a.out) | static_cast<uintptr_t>(a.pitch)) & 3u) == 0 &&
                    a.pitch >= ((a.len + 3) & ~3) && a.len <= kRenderFastLen;
  if (fast)
    hipLaunchKernelGGL(render_rows_fast_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL(render_rows_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0, st, a);
  check_hip(hipGetLastError(), "render_rows_kernel");
}
void render_rows_host(const RenderArgs& a) {
  for (int64_t r = 0; r < a.rows; ++r) {
    uint64_t sv[kRenderMaxStamps];
    render_stamp_values(a, a.ids[r], sv);
    for (int32_t j = 0; j < a.len; ++j)
      a.out[a.ids[r] * a.pitch + j] = static_cast<uint8_t>(render_char(a, a.tmpl, a.ids[r], sv, j));
  }
}

// ------------------------------------------------------------------ K08
// The message is virtual: prefix bytes, then the parent field text, then the
// suffix bytes.  The device assembles each message a 32-bit word at a time in
// the wave's LDS window (ahv/wave_sink.h) — aligned word loads of the arena
// funnel-shifted to the span offset, SWAR hex for the parent — the host twin
// streams the same bytes.
//
// Midstate split: the prefix (agent_did, changes, delta_id —
// the keys that sort before "parent_hash") does not depend on the chain, so with
// `mid` set the whole 64-byte blocks of every delta's prefix are compressed first,
// one lane per delta over all deltas at once (phase 1, fills the part however few
// chains there are).  The serial pass (phase 2, one lane per chain) resumes each
// delta from its midstate and hashes only the prefix remainder, the parent hex
// and the suffix — about half the blocks of a governance delta.

namespace {
AHV_HD uint32_t funnel32(uint32_t lo, uint32_t hi, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
  return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
#endif
}

// Span-table row of packed delta i (see ChainHashArgs::sel).
// (i / d, i % d) with 32-bit division when both fit (64-bit integer division is a
// long software sequence on the device)
AHV_HD void divmod_idx(int64_t i, int64_t d, int64_t& q, int64_t& r) {
  if (i >= 0 && i <= 0x7fffffff && d > 0 && d <= 0x7fffffff) {
    const uint32_t qq = static_cast<uint32_t>(i) / static_cast<uint32_t>(d);
    q = qq;
    r = i - static_cast<int64_t>(qq) * d;
  } else {
    q = i / d;
    r = i - q * d;
  }
}

AHV_HD int64_t span_row(const ChainHashArgs& a, int64_t i) {
  if (!a.sel) return i;
  int64_t c, k;
  divmod_idx(i, a.uniform_len, c, k);
  return a.sel[c] * a.uniform_len + k;
}

AHV_HD void chain_prefix_elem(const ChainHashArgs& a, int64_t i) {
  uint32_t st[8];
  sha256_init(st);
  const int64_t sr = span_row(a, i);
  const uint8_t* p = a.bytes + a.pre_off[sr];
  const int32_t nb = a.pre_len[sr] >> 6;
  const uintptr_t ad = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(ad & ~static_cast<uintptr_t>(3));
  const uint32_t sh = static_cast<uint32_t>(ad & 3u) * 8u;
  for (int32_t b = 0; b < nb; ++b) {
    uint32_t raw[17];
#pragma unroll
    for (int k = 0; k < 16; ++k) raw[k] = w[b * 16 + k];
    // the 17th word holds the block's last bytes only when the span is unaligned
    // (and then lies inside the prefix: never past the arena)
    raw[16] = sh ? w[b * 16 + 16] : 0u;
    uint32_t blk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) blk[k] = bswap_word(funnel32(raw[k], raw[k + 1], sh));
    sha256_compress(st, blk);
  }
  for (int k = 0; k < 8; ++k) a.mid[i * 8 + k] = st[k];
}

template <class Sink>
AHV_HD void chain_emit(Sink& s, const ChainHashArgs& a, int64_t sr, uint32_t skip, bool have, const Digest& prev) {
  emit_span_prefetch<16>(s, a.bytes + a.pre_off[sr] + skip, static_cast<uint32_t>(a.pre_len[sr]) - skip);
  if (have) emit_hex_digest_quoted(s, prev.v);
  else emit_lit(s, canon::K_NULL);
  emit_span_prefetch<16>(s, a.bytes + a.suf_off[sr], static_cast<uint32_t>(a.suf_len[sr]));
}

template <class Sink>
AHV_HD void chain_hash_elem(const ChainHashArgs& a, int64_t c, Sink& sink) {
  Digest prev;
  bool have = a.has_seed && a.seed_parent && a.has_seed[c];
  if (have)
    for (int k = 0; k < 8; ++k) prev.v[k] = a.seed_parent[c * 8 + k];
  for (int32_t i = a.chain_offsets[c]; i < a.chain_offsets[c + 1]; ++i) {
    uint32_t h[8];
    const bool hv = have;
    const Digest pv = prev;
    // span-table row of delta i (chain c's rows start at sel[c]·len)
    const int64_t sr = a.sel ? a.sel[c] * a.uniform_len + (i - a.chain_offsets[c]) : i;
    if (a.mid) {
      const uint32_t skip = static_cast<uint32_t>(a.pre_len[sr]) & ~63u;
      uint32_t st[8];
      for (int k = 0; k < 8; ++k) st[k] = a.mid[static_cast<int64_t>(i) * 8 + k];
      sink.hash_from([&](Sink& k) { chain_emit(k, a, sr, skip, hv, pv); }, st, skip, h);
    } else {
      sink.hash([&](Sink& k) { chain_emit(k, a, sr, 0u, hv, pv); }, h);
    }
    for (int k = 0; k < 8; ++k) {
      a.digest[static_cast<int64_t>(i) * 8 + k] = h[k];
      prev.v[k] = h[k];
    }
    have = true;
  }
}
}  // namespace

// Phase 1 on the device: one lane per delta, 256-thread blocks.  (Staging every
// delta's prefix rows in LDS with coalesced 256-byte loads measured slower —
// 56 → 92 µs for 160 k deltas: the kernel is bound by the SHA rounds of its
// longest lanes, not by the scattered word loads, which mostly hit L2.)
AHV_HD int64_t prefix_lane_delta(const ChainHashArgs& a, int64_t i) {
  if (a.uniform_len <= 0) return i;
  const int64_t c = a.deltas / a.uniform_len;  // chains (wave-uniform)
  int64_t turn, chain;
  divmod_idx(i, c, turn, chain);
  return chain * a.uniform_len + turn;
}

__global__ __launch_bounds__(256) void chain_prefix_kernel(ChainHashArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.deltas) chain_prefix_elem(a, prefix_lane_delta(a, i));
}

// One wave per 64 chains; lanes whose chains are shorter idle (masked) while
// the wave finishes its longest chain.  (A 4-block window — one emission pass
// for a governance delta's ≈ 225-byte post-midstate remainder — measured no
// faster than 3 blocks: the walk is bound by its SHA rounds and load latency.)
constexpr int kChainWin = 3;
__global__ __launch_bounds__(kWaveLanes, 3) void chain_hash_kernel(ChainHashArgs a) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kWaveLanes + threadIdx.x;
  WordWindowSink<kChainWin> sink;
  sink.g_win = win_lds<kChainWin>();
  sink.lane = threadIdx.x;
  if (c < a.chains) chain_hash_elem(a, c, sink);
}
void launch_chain_hash(const ChainHashArgs& a, hipStream_t st) {
  if (a.chains <= 0) return;
  if (a.mid && a.deltas > 0) {
    hipLaunchKernelGGL(chain_prefix_kernel, grid1(a.deltas, 256), dim3(256), 0, st, a);
    check_hip(hipGetLastError(), "chain_prefix_kernel");
  }
  hipLaunchKernelGGL(chain_hash_kernel, grid1(a.chains, kWaveLanes), dim3(kWaveLanes), 0, st, a);
  check_hip(hipGetLastError(), "chain_hash_kernel");
}
void chain_hash_host(const ChainHashArgs& a) {
  if (a.mid)
    for (int64_t i = 0; i < a.deltas; ++i) chain_prefix_elem(a, prefix_lane_delta(a, i));
  HostSink sink;
  for (int64_t c = 0; c < a.chains; ++c) chain_hash_elem(a, c, sink);
}

// ------------------------------------------------------------------ K09
// One lane per chain: level-wise Merkle (delta_emit.h merkle_root_levels, one
// node-hash site) with its ⌈n/2⌉ interior digests parked in the chain's rows of
// `scratch` (a chain of n leaves owns n scratch rows).

struct GlobalStash {
  uint32_t* rows;  // this chain's scratch rows
  AHV_HD void stash(int j, const uint32_t d[8]) {
    for (int k = 0; k < 8; ++k) rows[j * 8 + k] = d[k];
  }
  AHV_HD void load(int j, uint32_t d[8]) const {
    for (int k = 0; k < 8; ++k) d[k] = rows[j * 8 + k];
  }
  AHV_HD void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) const {
    uint32_t t[8];
    merkle_node(l, r, t);
    for (int k = 0; k < 8; ++k) out[k] = t[k];
  }
};

AHV_HD void merkle_elem(const MerkleArgs& a, int64_t c) {
  const int32_t b = a.offsets[c], e = a.offsets[c + 1];
  const int64_t row = a.root_row ? a.root_row[c] : c;
  uint32_t* root = a.root + row * 8;
  if (e <= b || (a.root_row && a.gate && a.gate[row] == 0)) {
    for (int k = 0; k < 8; ++k) root[k] = 0;
    return;
  }
  GlobalStash gs{a.scratch + static_cast<int64_t>(b) * 8};
  uint32_t r[8];
  merkle_root_levels(
      gs, static_cast<uint32_t>(e - b),
      [&](uint32_t i, uint32_t h[8]) {
        const int64_t li = static_cast<int64_t>(b) + i;
        const int64_t src = a.leaf_idx ? a.leaf_idx[li] : li;  // the leaf gather, fused
        for (int k = 0; k < 8; ++k) h[k] = a.leaves[src * 8 + k];
      },
      r);
  for (int k = 0; k < 8; ++k) root[k] = r[k];
}
__global__ __launch_bounds__(kWaveLanes) void merkle_kernel(MerkleArgs a) {
  for (int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; c < a.chains;
       c += static_cast<int64_t>(gridDim.x) * blockDim.x)
    merkle_elem(a, c);
}
void launch_merkle(const MerkleArgs& a, hipStream_t st) {
  if (a.chains <= 0) return;
  hipLaunchKernelGGL(merkle_kernel, grid1(a.chains, 64), dim3(64), 0, st, a);
  check_hip(hipGetLastError(), "merkle_kernel");
}
void merkle_host(const MerkleArgs& a) { for (int64_t c = 0; c < a.chains; ++c) merkle_elem(a, c); }

// ------------------------------------------------------------------ K10
// Embarrassingly parallel over deltas (one lane recomputes one digest), then a
// per-chain AND that also checks every parent link against the predecessor's
// stored digest.  Nothing is written back to the stored digests (fix of the
// reference's self-"repairing" verify_chain).

AHV_HD void verify_delta_elem(const VerifyArgs& a, int64_t i) {
  uint32_t h[8];
  const int64_t o = a.offsets[i];
  sha256_span(a.bytes + o, a.offsets[i + 1] - o, h);
  bool ok = true;
  for (int k = 0; k < 8; ++k) ok = ok && h[k] == a.stored[i * 8 + k];
  a.delta_ok[i] = ok ? 1 : 0;
}
AHV_HD void verify_chain_elem(const VerifyArgs& a, int64_t c) {
  bool ok = true;
  for (int32_t i = a.chain_offsets[c]; i < a.chain_offsets[c + 1]; ++i) {
    ok = ok && a.delta_ok[i];
    if (i == a.chain_offsets[c]) {
      ok = ok && !a.has_parent[i];
    } else {
      ok = ok && a.has_parent[i];
      for (int k = 0; k < 8; ++k) ok = ok && a.parent[static_cast<int64_t>(i) * 8 + k] == a.stored[static_cast<int64_t>(i - 1) * 8 + k];
    }
  }
  a.chain_ok[c] = ok ? 1 : 0;
}
__global__ void verify_delta_kernel(VerifyArgs a) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.deltas;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    verify_delta_elem(a, i);
}
__global__ void verify_chain_kernel(VerifyArgs a) {
  for (int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; c < a.chains;
       c += static_cast<int64_t>(gridDim.x) * blockDim.x)
    verify_chain_elem(a, c);
}
void launch_verify(const VerifyArgs& a, hipStream_t st) {
  if (a.deltas > 0) {
    hipLaunchKernelGGL(verify_delta_kernel, grid1(a.deltas, 64), dim3(64), 0, st, a);
    check_hip(hipGetLastError(), "verify_delta_kernel");
  }
  if (a.chains > 0) {
    hipLaunchKernelGGL(verify_chain_kernel, grid1(a.chains), dim3(kBlock), 0, st, a);
    check_hip(hipGetLastError(), "verify_chain_kernel");
  }
}
void verify_host(const VerifyArgs& a) {
  for (int64_t i = 0; i < a.deltas; ++i) verify_delta_elem(a, i);
  for (int64_t c = 0; c < a.chains; ++c) verify_chain_elem(a, c);
}


void kernels_audit(std::vector<KernelEntry>& out) {
  out.push_back({"chain_hash_kernel", reinterpret_cast<const void*>(&chain_hash_kernel)});
  out.push_back({"chain_prefix_kernel", reinterpret_cast<const void*>(&chain_prefix_kernel)});
  out.push_back({"render_rows_kernel", reinterpret_cast<const void*>(&render_rows_kernel)});
  out.push_back({"render_rows_fast_kernel", reinterpret_cast<const void*>(&render_rows_fast_kernel)});
  out.push_back({"merkle_kernel", reinterpret_cast<const void*>(&merkle_kernel)});
  out.push_back({"hash_many_kernel", reinterpret_cast<const void*>(&hash_many_kernel)});
  out.push_back({"verify_delta_kernel", reinterpret_cast<const void*>(&verify_delta_kernel)});
}

}  // namespace ahv
