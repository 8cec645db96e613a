// Template pipeline over the store's rows (ahv/store_template.h): the headline
// kernel of bench.py and the engine behind `Hypervisor.pipeline_batch`.
//
// Geometry: one 64-lane wave per workgroup, one session per lane, and the same
// 3-block LDS message window as the governance pipeline kernel (ahv/wave_sink.h:
// 12.5 KiB → 3 waves per SIMD, [word][lane] layout, conflict-free).  The record
// sink tees the window: after each emission pass, the lane's words of the
// canonical-JSON record that fall in the window are byte-swapped back to memory
// order and stored to its arena reservation with 16-byte stores (the window
// start and the reservation are 64-byte aligned), so the record is written once,
// by the lane that hashes it, without a separate render or re-read pass.  The SHA
// rounds dominate (VALU-issue bound); the record stores (≈300 B per delta) and the
// row writes overlap them across the resident waves.
//
// Batch counters (X04 input) are reduced per wave with DPP shuffles into spread
// rows (one 64-bit atomic per counter per wave), as in pipeline.hip.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdlib>

#include "ahv/launch.h"
#include "ahv/store_template.h"
#include "ahv/wave_sink.h"

namespace py = pybind11;

namespace ahv {
namespace {

template <int W>
struct TeeWindowSink : WordWindowSink<W> {
  using B = WordWindowSink<W>;
  bool nohash = false;    // A/B: emission and tee only
  bool lane_tee = false;  // A/B: per-lane record stores instead of the transposed tee

  // Hash the record `emit(*this)` produces (midstate modes as WordWindowSink::
  // hash_mid) and store its bytes at `dst` (memory order); `len` = its length.
  template <class Emit>
  __device__ __forceinline__ void hash_record(Emit&& emit, uint32_t out[8], Digest& mid, int mode, uint32_t* dst,
                                              uint32_t& len) {
    uint32_t st[8];
    if (mode == MID_RESUME) {
#pragma unroll
      for (int k = 0; k < 8; ++k) st[k] = mid.v[k];
      this->lo = 16;
    } else {
      sha256_init(st);
      this->lo = 0;
    }
    int32_t total = 0;
    uint32_t L = 0;
    bool first = true;
    while (first || __any(this->lo < total)) {
#pragma unroll
      for (int k = 0; k < B::kWinWords; ++k) this->g_win[k * kWaveLanes + this->lane] = 0u;
      this->trash = (static_cast<uint32_t>(B::kWinWords) * kWaveLanes + this->lane) * 4u;
      this->seek(-this->lo);
      this->sh = 0;
      this->prev = 0;
      emit(*this);
      L = static_cast<uint32_t>(this->rel + this->lo) * 4u + (this->sh >> 3);
      total = static_cast<int32_t>(((L + 8u) / 64u + 1u) * 16u);
      this->put(0x80000000u, 1);
      this->store_at(this->sh ? this->addr : this->trash, __builtin_amdgcn_alignbit(this->prev, 0u, this->sh));
      const uint64_t bits = static_cast<uint64_t>(L) * 8u;
      this->store(total - 2 - this->lo, static_cast<uint32_t>(bits >> 32));
      this->store(total - 1 - this->lo, static_cast<uint32_t>(bits));
      // tee: the record's words in this window → the arena (whole 16-byte chunks up to
      // the record's last word; bytes past `L` are padding inside the reservation)
      const int32_t nw = dst ? static_cast<int32_t>((L + 3u) >> 2) - this->lo : 0;
      // (the transposed form needs every lane of the wave here: a partial wave — the
      // grid's tail, lanes whose row was refused — stores per lane)
      if (lane_tee || __builtin_amdgcn_read_exec() != ~0ull) {  // each lane stores its own record
#pragma unroll
        for (int k = 0; k < B::kWinWords; k += 4) {
          if (k < nw) {
            const uint32_t* w = this->g_win + k * kWaveLanes + this->lane;
            *reinterpret_cast<uint4*>(dst + this->lo + k) =
                make_uint4(bswap_word(w[0]), bswap_word(w[kWaveLanes]), bswap_word(w[2 * kWaveLanes]),
                           bswap_word(w[3 * kWaveLanes]));
          }
        }
      } else {
        // transposed: lane 4a + b stores 16-byte chunk 4·ln + b (line ln, quarter b) of
        // record 16·rg + a, so four consecutive lanes fill one 64-byte line of one record
        // — 16 whole lines per store instead of 64 partial ones
        constexpr int C = B::kWinWords / 4;  // chunks of a record in the window
        const uint64_t mine = reinterpret_cast<uint64_t>(dst);
        const int qa = static_cast<int>(this->lane) >> 2, qb = static_cast<int>(this->lane) & 3;
#pragma nounroll
        for (int rg = 0; rg < kWaveLanes / 16; ++rg) {
          const int r = 16 * rg + qa;
          const int32_t nwr = __shfl(nw, r);
          const int32_t lor = __shfl(this->lo, r);  // per lane: 16 for a record resumed from the midstate
          const uint64_t dr = __shfl(mine, r);
#pragma nounroll
          for (int ln = 0; ln < C / 4; ++ln) {
            const int q = 4 * ln + qb;
            if (4 * q < nwr) {
              const uint32_t* w = this->g_win + (4 * q) * kWaveLanes + r;
              *reinterpret_cast<uint4*>(reinterpret_cast<uint32_t*>(dr) + lor + 4 * q) =
                  make_uint4(bswap_word(w[0]), bswap_word(w[kWaveLanes]), bswap_word(w[2 * kWaveLanes]),
                             bswap_word(w[3 * kWaveLanes]));
            }
          }
        }
      }
#pragma nounroll
      for (int blk = 0; blk < W; ++blk) {
        if (!nohash && this->lo + 16 * blk < total) {
          uint32_t w[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) w[k] = this->g_win[(blk * 16 + k) * kWaveLanes + this->lane];
          sha256_compress(st, w);
          if (mode == MID_CAPTURE && this->lo == 0 && blk == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) mid.v[k] = st[k];
          }
        }
      }
      first = false;
      this->lo += B::kWinWords;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = st[k];
    len = L;
  }
};

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWaveLanes);
  return v;
}

// A/B switches (AHV_TEMPLATE_AB, measurement only): bit 0 — skip the record tee
// (digests and rows only); bit 1 — tee into a coarse-grained scratch buffer
// instead of the store's fine-grained payload arena; bit 2 — no Merkle root;
// bit 3 — no record compressions (emission + tee only); bit 6 — per-lane record
// stores instead of the transposed tee.
static int template_ab() {
  static const int v = [] {
    const char* e = std::getenv("AHV_TEMPLATE_AB");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// Small batches (n ≤ AHV_TEMPLATE_SMALL sessions, default 65,536: fewer waves than
// the chip has SIMDs, so each wave runs alone and latency is all that counts) use a
// 6-block window: a whole record in one emission pass instead of two.
static int64_t template_small() {
  static const int64_t v = [] {
    const char* e = std::getenv("AHV_TEMPLATE_SMALL");
    return e ? std::atoll(e) : int64_t(65536);
  }();
  return v;
}

// Cooperative small-batch kernel (store_template_coop_kernel): AHV_TEMPLATE_COOP=0 off;
// used up to AHV_TEMPLATE_COOP_MAX sessions (default 16,384: one workgroup per CU).
static int template_coop() {
  static const int v = [] {
    const char* e = std::getenv("AHV_TEMPLATE_COOP");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
static int64_t coop_max_sessions() {
  static const int64_t v = [] {
    const char* e = std::getenv("AHV_TEMPLATE_COOP_MAX");
    return e ? std::atoll(e) : int64_t(16384);
  }();
  return v;
}

// Occupancy variant (AHV_TEMPLATE_WAVES = 2, 3 or 4 waves per SIMD; 4 uses a 2-block window).
static int template_waves() {
  static const int v = [] {
    const char* e = std::getenv("AHV_TEMPLATE_WAVES");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}

template <int MinWaves, int W>
__global__ __launch_bounds__(kWaveLanes, MinWaves) void store_template_kernel(TemplateArgs a) {
  const uint32_t lane = threadIdx.x;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaveLanes + lane;
  PipeCounters c{};
  if (i < a.n) {
    TeeWindowSink<W> sink;
    sink.g_win = win_lds<W>();
    sink.lane = lane;
    c = template_session(a, i, sink);
  }
  if (a.stats) {
#pragma unroll
    for (int k = 0; k < kPipeStats; ++k) {
      const uint32_t s = wave_sum(c.v[k]);
      if (lane == 0 && s)
        atomicAdd(a.stats + (blockIdx.x % kStatSpread) * kPipeStats + k, static_cast<unsigned long long>(s));
    }
  }
  if (a.ev.cursor) {
    // one 64-bit atomic reserves the wave's records; lanes write at their exclusive prefix
    uint32_t nev = 0;
    if (i < a.n) nev = template_event_count(c, a.t.s_terminated[template_rows(a, i).s] != 0);
    uint32_t incl = nev;
#pragma unroll
    for (int off = 1; off < kWaveLanes; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, kWaveLanes);
      if (lane >= static_cast<uint32_t>(off)) incl += y;
    }
    const uint32_t total = __shfl(incl, kWaveLanes - 1, kWaveLanes);
    const int seg = static_cast<int>(blockIdx.x % kStatSpread);
    unsigned long long base = 0;
    if (lane == 0 && total) base = atomicAdd(a.ev.cursor + seg, static_cast<unsigned long long>(total));
    base = __shfl(base, 0, kWaveLanes);
    if (i < a.n) {
      const unsigned long long first = base + (incl - nev);
      template_events(a, i, c, [&](uint32_t k, int64_t slot, const EventRec& e) {
        event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
      });
    }
  }
}

// ---- small batches: four cooperating waves per 64 sessions ------------------------
//
// A batch smaller than the chip (config 2: 10⁴ sessions = 157 waves for 1,024 SIMDs)
// is latency-bound: each wave runs alone on its SIMD and its time is its
// instruction stream — one lane per session doing all of the session's serial work
// (three records chained through their parent digests, then a 3-leaf Merkle root:
// 25 compressions).  Here a workgroup of four waves (one per SIMD) shares 64
// sessions, one lane per session in every wave:
//
//   wave 3      the session rows (create → join/K01 → activate → saga/K13 →
//               terminate bookkeeping), counters and events;
//   wave q < D  renders record q into its own LDS window (all records at once; the
//               parent digest a placeholder), hashes the blocks before its parent
//               hole, waits for record q−1's digest, patches its hex in and hashes
//               the rest, writes its delta row and stores the record;
//   Merkle      wave 0 computes node(l0, l1) and the root's first block (hex of that
//               node) while wave 2 finishes record 2; wave 1 then computes
//               node(l2, l2) and the root's last two blocks.
//
// The serial path is record 0 (all blocks) → record 1's tail → record 2's tail →
// node(l2, l2) → root tail: 19 compressions instead of 25, and one record
// emission instead of three.  D ∈ {1, 2, 3}; ≤ W blocks per record (the host
// checks the reservation size).  Same rows, records and digests as
// template_session (one semantics source: template_head, emit_delta_payload).
constexpr int kCoopWaves = 4;

// Workgroup-scope flags between the cooperating waves (LDS).
__device__ __forceinline__ uint32_t coop_get(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void coop_wait(const uint32_t* f, uint32_t v) {
  while (coop_get(f) < v) __builtin_amdgcn_s_sleep(1);
}
// Publish `v`: every LDS write this wave issued before is visible to a wave that
// reads `v` with coop_get (the fence waits for the wave's LDS operations).
__device__ __forceinline__ void coop_set(uint32_t* f, uint32_t v, uint32_t lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// K+W schedule of one message block held in a [word][lane] LDS column (stride 64)
// into a [t][lane] column of the K+W ring.
__device__ __forceinline__ void coop_expand(const uint32_t* w, uint32_t* kw) {
  uint32_t x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    x[k] = w[k * kWaveLanes];
    kw[k * kWaveLanes] = x[k] + sha256_k(k);
  }
#pragma unroll
  for (int k = 16; k < 64; ++k) {
    const uint32_t a = x[(k + 1) & 15], b = x[(k + 14) & 15];
    const uint32_t s0 = xor3(rotr32(a, 7), rotr32(a, 18), a >> 3);
    const uint32_t s1 = xor3(rotr32(b, 17), rotr32(b, 19), b >> 10);
    const uint32_t v = x[k & 15] + s0 + x[(k + 9) & 15] + s1;
    x[k & 15] = v;
    kw[k * kWaveLanes] = v + sha256_k(k);
  }
}

// The 64 rounds over a K+W column (store::sha256_rounds_kw with stride 64).
__device__ __forceinline__ void coop_rounds(uint32_t st[8], const uint32_t* kw) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
  uint32_t q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q[k] = kw[k * kWaveLanes];
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const uint32_t kwi = q[k & 7];
    if (k + 8 < 64) q[k & 7] = kw[(k + 8) * kWaveLanes];
    const uint32_t S1 = xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
    const uint32_t t1 = store::add3u(h + kwi, S1, sha_ch(e, f, g));
    const uint32_t S0 = xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
    const uint32_t na = store::add3u(t1, S0, sha_maj(a, b, c));
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = na;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ __forceinline__ int32_t wave_max(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(v, o, kWaveLanes);
    v = y > v ? y : v;
  }
  return v;
}

// The chain's compressions (record 0 whole, records 1 and 2 after the parent hole)
// run as rounds only: wave 3, once the session rows are written, expands each
// block's message schedule into a two-slot K+W ring in LDS one block ahead of the
// hashing wave (the schedule is a third of a compression).  Waves hand off
// through LDS flags (no workgroup barrier after the first): digests d0..d2,
// segment ready (window final, block ranges set), produced / consumed ring
// blocks, the root's first-block state, the committed flags.
enum CoopFlag : int { CF_DIG = 0, CF_MID = 3, CF_LIVE = 4, CF_SEG = 5, CF_PROD = 8, CF_CONS = 9, CF_N = 10 };

template <int W>
__global__ __launch_bounds__(kCoopWaves * kWaveLanes, 1) void store_template_coop_kernel(TemplateArgs a) {
  constexpr int kWinWords = (W * 16 + 1) * kWaveLanes;
  __shared__ uint32_t win[3 * kWinWords];
  __shared__ uint32_t kwb[2][64 * kWaveLanes];  // K+W ring, [t][lane]
  __shared__ uint32_t dig[3][8][kWaveLanes];    // record digests (Merkle leaves, parents)
  __shared__ uint32_t mid[8][kWaveLanes];       // root state after its first block (D = 3)
  __shared__ int32_t seglo[3][kWaveLanes], seghi[3][kWaveLanes], segK[3];
  __shared__ uint8_t live_c[kWaveLanes];        // the session committed a root (wave 3's answer)
  __shared__ uint32_t flags[CF_N];
  const int wave = static_cast<int>(threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaveLanes + lane;
  const store::Tables& t = a.t;
  const int32_t D = a.deltas;
  const int nrec = D < 3 ? D : 3;
  const TemplateRows R = template_rows(a, i < a.n ? i : 0);
  int ph = 0;  // phase timestamps (measurement: AHV template args "phase_ticks")
  auto mark = [&]() {
    if (a.phase_ticks && blockIdx.x == 0 && lane == 0) a.phase_ticks[16 * wave + ph] = __builtin_amdgcn_s_memrealtime();
    ++ph;
  };
  mark();
  if (threadIdx.x < CF_N) flags[threadIdx.x] = 0;
  // every wave decides liveness before wave 3 writes the row
  const bool live = i < a.n && (R.ring || t.s_state[R.s] == store::kFree8);
  __syncthreads();

  PipeCounters c{};
  uint32_t u[4];
  const int64_t t0 = tp_t0(a);
  if (live) uuid4_words(a.seed, tp_id_base(a) + a.id_stride * static_cast<uint64_t>(i), u);

  if (wave == 3) {
    // ---- session rows, then the schedule producer, then counters and events ----------
    c.v[0] = i < a.n ? 1u : 0u;
    bool committed = false;
    if (live) {
      committed = template_head(a, i, R, c, u);
    } else if (i < a.n && a.status) {
      a.status[i] = TP_ROW_IN_USE;
    }
    live_c[lane] = committed ? 1 : 0;
    coop_set(&flags[CF_LIVE], 1, lane);
    mark();
    uint32_t idx = 0;
    for (int sg = 0; sg < nrec; ++sg) {
      coop_wait(&flags[CF_SEG + sg], 1);
      const int32_t K = segK[sg], lo = seglo[sg][lane], hi = seghi[sg][lane];
      const uint32_t* col = win + sg * kWinWords + lane;
      for (int32_t k = 0; k < K; ++k, ++idx) {
        while (idx - coop_get(&flags[CF_CONS]) >= 2u) __builtin_amdgcn_s_sleep(1);
        if (lo + k < hi) coop_expand(col + (lo + k) * 16 * kWaveLanes, kwb[idx & 1] + lane);
        coop_set(&flags[CF_PROD], idx + 1, lane);
      }
    }
    mark();
    if (a.stats) {
#pragma unroll
      for (int k = 0; k < kPipeStats; ++k) {
        const uint32_t sm = wave_sum(c.v[k]);
        if (lane == 0 && sm)
          atomicAdd(a.stats + (blockIdx.x % kStatSpread) * kPipeStats + k, static_cast<unsigned long long>(sm));
      }
    }
    if (a.ev.cursor) {
      uint32_t nev = 0;
      if (live) nev = template_event_count(c, t.s_terminated[R.s] != 0);
      uint32_t incl = nev;
#pragma unroll
      for (int o = 1; o < kWaveLanes; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, kWaveLanes);
        if (lane >= static_cast<uint32_t>(o)) incl += y;
      }
      const uint32_t tot = __shfl(incl, kWaveLanes - 1, kWaveLanes);
      const int seg = static_cast<int>(blockIdx.x % kStatSpread);
      unsigned long long base = 0;
      if (lane == 0 && tot) base = atomicAdd(a.ev.cursor + seg, static_cast<unsigned long long>(tot));
      base = __shfl(base, 0, kWaveLanes);
      if (live) {
        const unsigned long long first = base + (incl - nev);
        template_events(a, i, c, [&](uint32_t k, int64_t slot, const EventRec& e) {
          event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
        });
      }
    }
    mark();
    return;
  }

  // ---- waves 0..2: record q --------------------------------------------------------------
  WordWindowSink<W> sink;
  sink.g_win = win + wave * kWinWords;
  sink.lane = lane;
  const int q = wave;
  const bool rec = q < nrec;  // this wave owns a record
  const bool mine = live && rec;
  uint32_t st[8];
  uint32_t len = 0;
  int32_t total = 0, hb = 0;
  uint32_t hole = 0;
  const int32_t ag = live ? a.session_agent[i] : 0;
  const int64_t tsd = t0 + 1 + q;
  const uint32_t turn = static_cast<uint32_t>(q + 1);
  const int64_t dr = rec ? R.drow(a, q) : 0;
  const int64_t off = rec ? R.doff(a, q) : 0;
  if (rec) {
    SessionIdent sid;
    sid.str_id = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) sid.uuid[k] = live ? u[k] : 0u;
    const StrRef did = pool_ref(a.pool, a.agent_pool[ag]);
    const StrPool pool = a.pool;
    const uint32_t nch = static_cast<uint32_t>(a.nch);
    const ChangeIds* ch = a.changes + q * nch;
    const uint32_t* fw = a.frag ? a.frag + frag_word(reinterpret_cast<const uint32_t*>(a.frag_off), q) : nullptr;
    const uint32_t fn = a.frag ? frag_word(reinterpret_cast<const uint32_t*>(a.frag_len), q) : 0u;
    Digest ph;  // placeholder parent (patched once the parent's digest is known)
#pragma unroll
    for (int k = 0; k < 8; ++k) ph.v[k] = 0;
    total = sink.render([=](WordWindowSink<W>& k) {
      emit_delta_payload(k, pool, did, ch, nch, -1, turn, q > 0, ph, sid, tsd, fw, fn);
    }, len);
    // the parent's hex starts one byte after the hole's opening quote
    hole = q > 0 ? len - record_suffix_len(tsd, turn) : 0u;
    hb = q > 0 ? static_cast<int32_t>(hole / 64u) : 0;
    // the chain segment: record 0 whole, records 1, 2 from the block holding the hole
    const int32_t lo = mine ? hb : 0, hi = mine ? total / 16 : 0;
    seglo[q][lane] = lo;
    seghi[q][lane] = hi;
    const int32_t K = wave_max(hi - lo);
    if (lane == 0) segK[q] = K;
    mark();
    sha256_init(st);
    if (q > 0) sink.compress_blocks(st, 0, mine ? hb : 0);  // parent-independent blocks
    mark();
  }
  auto publish = [&](void) {  // its digest → LDS (the next record's parent, a leaf)
    if (mine) {
#pragma unroll
      for (int k = 0; k < 8; ++k) dig[q][k][lane] = st[k];
    }
    coop_set(&flags[CF_DIG + q], 1, lane);
  };
  // rows + record bytes (after the digest is handed on: off the chain)
  auto finish = [&](void) {
    if (!mine) return;
    t.d_sess[dr] = static_cast<int32_t>(R.s);
    t.d_turn[dr] = static_cast<int32_t>(turn);
    t.d_prev[dr] = q > 0 ? static_cast<int32_t>(R.drow(a, q - 1)) : -1;
    t.d_ts[dr] = tsd;
    t.d_off[dr] = off;
    t.d_len[dr] = static_cast<int32_t>(len);
    t.d_hole[dr] = q > 0 ? static_cast<int32_t>(hole) : -1;
#pragma unroll
    for (int k = 0; k < 8; ++k) t.d_hash[8 * dr + k] = st[k];
    if (q == D - 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t.s_head[8 * R.s + k] = st[k];
    }
    if (!a.notee) sink.tee(reinterpret_cast<uint32_t*>(t.payload + off), static_cast<int32_t>((len + 3u) >> 2));
  };
  if (rec) {
    if (q > 0) {  // the parent's digest → its hex into the hole
      coop_wait(&flags[CF_DIG + q - 1], 1);
      uint32_t par[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) par[k] = dig[q - 1][k][lane];
      if (mine) sink.patch_hex(hole + 1u, par);
    }
    coop_set(&flags[CF_SEG + q], 1, lane);  // the window is final: the producer may expand it
    // the chain segment as rounds over the producer's K+W ring
    uint32_t base = 0;
    for (int sg = 0; sg < q; ++sg) base += static_cast<uint32_t>(segK[sg]);
    const int32_t K = segK[q], lo = seglo[q][lane], hi = seghi[q][lane];
    for (int32_t k = 0; k < K; ++k) {
      const uint32_t idx = base + static_cast<uint32_t>(k);
      coop_wait(&flags[CF_PROD], idx + 1);
      if (lo + k < hi) coop_rounds(st, kwb[idx & 1] + lane);
      coop_set(&flags[CF_CONS], idx + 1, lane);
    }
    mark();
    publish();
    mark();
    finish();
  }
  if (q == 0 && D == 3) {
    // node(l0, l1) and the root's first block (its hex) while record 2 is hashed
    coop_wait(&flags[CF_DIG + 1], 1);
    uint32_t l0[8], l1[8], n01[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      l0[k] = dig[0][k][lane];
      l1[k] = dig[1][k][lane];
    }
    sink.node(l0, l1, n01);
    uint32_t w[16], m[8];
    digest_to_hex_words(n01, w);
    sha256_init(m);
    sha256_compress(m, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) mid[k][lane] = m[k];
    coop_set(&flags[CF_MID], 1, lane);
    mark();
  }

  // ---- Merkle root (K09) → s_root: wave 1 ------------------------------------------------
  if (wave == 1 && D >= 1) {
    coop_wait(&flags[CF_DIG + nrec - 1], 1);
    coop_wait(&flags[CF_LIVE], 1);
    uint32_t root[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (live && live_c[lane] && !(a.ab & 4)) {
      if (D == 3) {
        uint32_t l2[8], n22[8], w[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) l2[k] = dig[2][k][lane];
        sink.node(l2, l2, n22);
        coop_wait(&flags[CF_MID], 1);
#pragma unroll
        for (int k = 0; k < 8; ++k) root[k] = mid[k][lane];
        digest_to_hex_words(n22, w);
        sha256_compress(root, w);
        sha256_compress_pad_only(root, 128u);
      } else if (D == 2) {
        uint32_t l0[8], l1[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          l0[k] = dig[0][k][lane];
          l1[k] = dig[1][k][lane];
        }
        sink.node(l0, l1, root);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) root[k] = dig[0][k][lane];
      }
    }
    if (live) {
#pragma unroll
      for (int k = 0; k < 8; ++k) t.s_root[8 * R.s + k] = root[k];
    }
    mark();
  }
}

template <class T>
T* P(const py::dict& d, const char* k) {
  return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}

TemplateArgs template_args(const store::Tables& t, const py::dict& d) {
  TemplateArgs a{};
  a.t = t;
  a.n = d["n"].cast<int64_t>();
  a.slot = P<const int32_t>(d, "slot");
  a.gslot = P<const int32_t>(d, "gslot");
  a.tslot = P<const int32_t>(d, "tslot");
  a.drow = P<const int32_t>(d, "drow");
  a.doff = P<const int64_t>(d, "doff");
  a.session_agent = P<const int32_t>(d, "session_agent");
  a.agent_id = P<const int32_t>(d, "agent_id");
  a.agent_pool = P<const int32_t>(d, "agent_pool");
  a.agent_sigma = P<const double>(d, "agent_sigma");
  a.changes = P<const ChangeIds>(d, "changes");
  if (d.contains("frag") && !d["frag"].is_none()) {
    a.frag = P<const uint32_t>(d, "frag");
    a.frag_off = P<const int32_t>(d, "frag_off");
    a.frag_len = P<const int32_t>(d, "frag_len");
  }
  a.pool = StrPool{P<const uint8_t>(d, "pool_bytes"), P<const int64_t>(d, "pool_off"), P<const int32_t>(d, "pool_len")};
  a.deltas = d["deltas"].cast<int32_t>();
  a.nch = d["nch"].cast<int32_t>();
  a.creator = d["creator"].cast<int32_t>();
  a.maxpart = d["maxpart"].cast<int32_t>();
  a.minsig = d["minsig"].cast<double>();
  a.audit = d["audit"].cast<int32_t>();
  a.t0 = d["t0"].cast<int64_t>();
  a.seed = d["seed"].cast<uint64_t>();
  a.id_base = d["id_base"].cast<uint64_t>();
  a.gc_retention_us = d["gc_retention_us"].cast<int64_t>();
  auto opt = [&](const char* k) { return d.contains(k) && !d[k].is_none(); };
  a.status = opt("status") ? P<int32_t>(d, "status") : nullptr;
  a.stats = opt("stats") ? P<unsigned long long>(d, "stats") : nullptr;
  a.ring_cap = opt("ring_cap") ? d["ring_cap"].cast<int64_t>() : 0;
  a.slot_base = opt("slot_base") ? d["slot_base"].cast<int64_t>() : 0;
  a.dstride = opt("dstride") ? d["dstride"].cast<int32_t>() : 0;
  a.rec_bytes = opt("rec_bytes") ? d["rec_bytes"].cast<int64_t>() : 0;
  a.off_base = opt("off_base") ? d["off_base"].cast<int64_t>() : 0;
  a.id_stride = opt("id_stride") ? d["id_stride"].cast<uint64_t>() : 1;
  a.cursor = opt("cursor") ? P<const int64_t>(d, "cursor") : nullptr;
  a.phase_ticks = opt("phase_ticks") ? P<uint64_t>(d, "phase_ticks") : nullptr;
  if (opt("ev_cursor")) {
    a.ev = EventRing{P<uint8_t>(d, "ev_type"), P<int32_t>(d, "ev_slot"), P<int32_t>(d, "ev_agent"),
                     P<int64_t>(d, "ev_ts_us"), P<int32_t>(d, "ev_aux"), P<unsigned long long>(d, "ev_cursor"),
                     d["ev_capacity"].cast<int64_t>()};
  }
  if (a.ring_cap > 0) {
    if (a.dstride < a.deltas || a.rec_bytes <= 0 || a.rec_bytes % 64 || a.off_base % 64)
      throw std::invalid_argument("ring mode: dstride ≥ deltas, rec_bytes a positive multiple of 64");
    if (a.ring_cap > t.cap.S || a.ring_cap > t.cap.G || a.ring_cap > t.cap.T || a.ring_cap * a.dstride > t.cap.D ||
        a.off_base + a.ring_cap * a.dstride * a.rec_bytes > t.cap.B)
      throw std::invalid_argument("ring mode: the ring does not fit the store's tables");
    if (a.n > a.ring_cap) throw std::invalid_argument("ring mode: batch larger than the ring");
  }
  if (a.deltas < 0 || a.deltas > kMaxDeltasPipeline) throw std::invalid_argument("deltas must be in [0, 8]");
  if (a.nch < 0 || a.nch > kMaxChanges) throw std::invalid_argument("changes per delta must be in [0, 4]");
  return a;
}

}  // namespace

// Launch on `stream` (device tables) or run the host twin (host tables).
void store_template_run(const store::Tables& t, bool gpu, const py::dict& d, uintptr_t stream) {
  const TemplateArgs a = template_args(t, d);
  if (!gpu) {
    HostTeeSink sink;
    for (int64_t i = 0; i < a.n; ++i) {
      const PipeCounters c = template_session(a, i, sink);
      const int seg = static_cast<int>((i / kWaveLanes) % kStatSpread);  // the device's workgroup mapping
      if (a.stats)
        for (int k = 0; k < kPipeStats; ++k) a.stats[seg * kPipeStats + k] += c.v[k];
      if (a.ev.cursor) {
        const unsigned long long first = a.ev.cursor[seg];
        a.ev.cursor[seg] += template_event_count(c, a.t.s_terminated[template_rows(a, i).s] != 0);
        template_events(a, i, c, [&](uint32_t k, int64_t slot, const EventRec& e) {
          event_store(a.ev, seg, first + k, static_cast<int32_t>(slot), e);
        });
      }
    }
    return;
  }
  if (a.n <= 0) return;
  TemplateArgs b = a;
  const int ab = template_ab();
  if (ab & 1) b.notee = 1;
  b.ab = ab & (4 | 8 | 64);
  if (ab & 2) {
    static uint8_t* scratch = nullptr;
    static int64_t scratch_cap = 0;
    if (scratch_cap < t.cap.B) {
      if (scratch) (void)hipFree(scratch);
      check_hip(hipMalloc(reinterpret_cast<void**>(&scratch), static_cast<size_t>(t.cap.B)), "template AB scratch");
      scratch_cap = t.cap.B;
    }
    b.t.payload = scratch;
  }
  // variant selection: per call ("waves" / "small" in the argument dict: oracle tests of
  // every variant in one process) or per process (AHV_TEMPLATE_WAVES / AHV_TEMPLATE_SMALL)
  const int waves = d.contains("waves") && !d["waves"].is_none() ? d["waves"].cast<int>() : template_waves();
  const int64_t small = d.contains("small") && !d["small"].is_none() ? d["small"].cast<int64_t>() : template_small();
  // cooperative small-batch kernel: D ≤ 3 records of ≤ 8 blocks (the caller's record
  // reservation `max_rec` bytes, or the ring's), at most one workgroup per CU
  // (ring mode: the slot size bounds it; the caller's exact bound wins when given)
  const int64_t max_rec = d.contains("max_rec") && !d["max_rec"].is_none() ? d["max_rec"].cast<int64_t>()
                          : (a.ring_cap > 0 ? a.rec_bytes : 0);
  const int coop = template_coop();
  const bool use_coop = coop != 0 && a.n <= coop_max_sessions() && a.deltas >= 1 && a.deltas <= 3 && max_rec > 0 &&
                        max_rec <= 512 && !(b.ab & 64) &&
                        !(d.contains("waves") && !d["waves"].is_none() && d["waves"].cast<int>() == -1);
  py::gil_scoped_release nogil;
  const dim3 grid(static_cast<uint32_t>((a.n + kWaveLanes - 1) / kWaveLanes)), block(kWaveLanes);
  if (use_coop) {
    const dim3 cblock(kCoopWaves * kWaveLanes);
    if (max_rec <= 384)
      hipLaunchKernelGGL((store_template_coop_kernel<6>), grid, cblock, 0, reinterpret_cast<hipStream_t>(stream), b);
    else
      hipLaunchKernelGGL((store_template_coop_kernel<8>), grid, cblock, 0, reinterpret_cast<hipStream_t>(stream), b);
  } else if (a.n <= small)  // latency-bound: one pass per record
    hipLaunchKernelGGL((store_template_kernel<1, 6>), grid, block, 0, reinterpret_cast<hipStream_t>(stream), b);
  else if (waves == 2)  // 231 VGPRs, no scratch
    hipLaunchKernelGGL((store_template_kernel<2, 3>), grid, block, 0, reinterpret_cast<hipStream_t>(stream), b);
  else if (waves == 4)  // 2-block window (8.5 KiB LDS): 4 waves per SIMD, one more emission pass
    hipLaunchKernelGGL((store_template_kernel<4, 2>), grid, block, 0, reinterpret_cast<hipStream_t>(stream), b);
  else  // 168 VGPRs (3 waves/SIMD) with a small spill
    hipLaunchKernelGGL((store_template_kernel<3, 3>), grid, block, 0, reinterpret_cast<hipStream_t>(stream), b);
  check_hip(hipGetLastError(), "store_template_kernel launch");
}

void kernels_store_template(std::vector<KernelEntry>& out) {
  out.push_back({"store_template_kernel<3,3>", reinterpret_cast<const void*>(&store_template_kernel<3, 3>)});
  out.push_back({"store_template_kernel<2,3>", reinterpret_cast<const void*>(&store_template_kernel<2, 3>)});
  out.push_back({"store_template_kernel<1,6>", reinterpret_cast<const void*>(&store_template_kernel<1, 6>)});
  out.push_back({"store_template_kernel<4,2>", reinterpret_cast<const void*>(&store_template_kernel<4, 2>)});
  out.push_back({"store_template_coop_kernel<6>", reinterpret_cast<const void*>(&store_template_coop_kernel<6>)});
  out.push_back({"store_template_coop_kernel<8>", reinterpret_cast<const void*>(&store_template_coop_kernel<8>)});
}

}  // namespace ahv
