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
  py::gil_scoped_release nogil;
  const dim3 grid(static_cast<uint32_t>((a.n + kWaveLanes - 1) / kWaveLanes)), block(kWaveLanes);
  if (a.n <= small)  // latency-bound: one pass per record
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
}

}  // namespace ahv
