// Agent-global liability kernels for session-sharded multi-GPU runs (SURVEY
// §2.13 X01/X02): the per-rank partials that the cross-rank collectives combine.
//
//   agent_exposure  (K04, global form) — exposure[a] = Σ live bonded amounts of
//                   the edges agent a vouches with (reference vouching.py:157-166
//                   summed over every session the rank owns).  Edges are stored
//                   CSR by voucher in creation order — a resident voucher-sorted
//                   layout, so the agent sums are a segmented reduction with no
//                   atomics: a wave owns 64 consecutive rows, stages their edge
//                   range (live bond or +0.0) in LDS with coalesced loads — every
//                   chunk requested before the first is stored — and each lane
//                   then adds its row in creation order (the exact fp64 sum;
//                   adding +0.0 for a dead edge leaves a +0.0-started sum
//                   unchanged).  The [A] vector is then all-reduced over ranks
//                   (X01: 8 MB for 1 M agents, RCCL over xGMI).  The same kernel
//                   gathers an agent's per-session exposure rows through an index
//                   (X01 input of the fused MFMA pass, ops.liability.bond_fused).
//   slash_clip      (K06 stage) — for a storm of k slashed vouchees: every live
//                   incoming edge (CSR by vouchee) is released and its voucher
//                   gets a clip factor (1 − ω) (reference slashing.py:89-99).  Each
//                   lane owns one vouchee and appends (voucher, factor) pairs into a
//                   fixed-capacity buffer through one atomic cursor; unused
//                   entries keep id −1 / factor 1.  The pairs are all-gathered and
//                   PROD-scattered (X02 sparse merge, collectives.merge_slash_fixed).
//
// Both are memory-streaming kernels: 256-thread workgroups, grid-stride, and a
// grid of ≥ 4 workgroups per CU so all 8 XCDs stay busy.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <vector>

#include "ahv/hd.h"
#include "ahv/launch.h"

namespace py = pybind11;

namespace ahv {
namespace {

struct ExposureArgs {
  int64_t agents;
  int64_t now_us;
  const int64_t* offsets;  // [A+1] CSR by voucher
  const double* bonded;    // [V] values (bond amounts, or per-session exposure rows)
  const uint8_t* active;   // [V] (null: every entry live)
  const int64_t* expiry;   // [V] (-1 = never; null: no expiry)
  double* out;             // [A]
  const int32_t* index;    // [E] value index of entry e (null: e itself)
};

AHV_HD double exposure_value(const ExposureArgs& a, int64_t e) {
  const int64_t v = a.index ? a.index[e] : e;
  // every word loaded unconditionally (no short-circuit: one round trip, not three)
  const double x = a.bonded[v];
  const uint8_t act = a.active ? a.active[v] : 1;
  const int64_t ex = a.expiry ? a.expiry[v] : -1;
  return act != 0 && (ex < 0 || a.now_us <= ex) ? x : 0.0;
}

AHV_HD double exposure_row(const ExposureArgs& a, int64_t r) {
  double s = 0.0;
  for (int64_t e = a.offsets[r]; e < a.offsets[r + 1]; ++e) s += exposure_value(a, e);
  return s;
}

constexpr int kSegWaves = 4;
constexpr int kSegChunks = 8;                      // staged chunks of 64 entries per wave
constexpr int kSegLds = kSegChunks * 64;           // 512 entries (4 KB) per wave

__global__ __launch_bounds__(64 * kSegWaves) void agent_exposure_kernel(ExposureArgs a) {
  __shared__ double s_v[kSegWaves][kSegLds];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t r0 = (static_cast<int64_t>(blockIdx.x) * kSegWaves + w) * 64;
  const int64_t r = r0 + l;
  const int64_t lo = a.offsets[r < a.agents ? r : a.agents];
  const int64_t hi = a.offsets[r + 1 < a.agents ? r + 1 : a.agents];
  const int64_t E0 = __shfl(lo, 0), E1 = __shfl(hi, 63);  // the wave's contiguous edge range
  const int64_t n = E1 - E0;
  double* v = s_v[w];
  const bool staged = n <= kSegLds;                   // wave-uniform
  if (staged) {
    double x[kSegChunks];
#pragma unroll
    for (int c = 0; c < kSegChunks; ++c) {           // all loads first, then the LDS stores
      const int64_t i = c * 64 + l;
      x[c] = i < n ? exposure_value(a, E0 + i) : 0.0;
    }
#pragma unroll
    for (int c = 0; c < kSegChunks; ++c)
      if (c * 64 < n) v[c * 64 + l] = x[c];
  }
  __syncthreads();
  if (r >= a.agents) return;
  double s = 0.0;
  if (staged) {
    for (int64_t k = lo - E0; k < hi - E0; ++k) s += v[k];
  } else {  // a wave whose 64 rows hold more than 512 entries: walk them in place
    for (int64_t e = lo; e < hi; ++e) s += exposure_value(a, e);
  }
  a.out[r] = s;
}

struct ClipArgs {
  int64_t k;                // slashed vouchees
  int64_t cap;              // pair buffer capacity
  int64_t now_us;
  double omega;
  const int32_t* ids;       // [k] vouchee agent ids
  const int64_t* offsets;   // [A+1] CSR by vouchee (incoming edges)
  const int32_t* src;       // [E] voucher of each incoming edge
  const int32_t* edge;      // [E] edge id in the voucher-major table
  uint8_t* active;          // [E] voucher-major active flags (released here)
  int64_t* released;        // [E]
  const int64_t* expiry;    // [E] voucher-major
  int32_t* pair_id;         // [cap] out (−1 = unused)
  double* pair_factor;      // [cap] out (1 = unused)
  unsigned long long* cursor;  // [1] pairs written (may exceed cap: overflow is counted, not written)
};

// Each lane owns one slashed vouchee and walks its in-edges kClipUnroll at a
// time: the edge ids, then their liveness words, are requested for the whole
// group at once (two round trips per group instead of two per edge); the claim
// (atomicAnd on the active byte) keeps the release-once semantics, and the
// wave's released edges take their pair slots with one cursor atomic per wave
// (ballot + mbcnt prefix) instead of one per edge.
constexpr int kClipUnroll = 8;

__global__ __launch_bounds__(256) void slash_clip_kernel(ClipArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (int64_t i0 = base - threadIdx.x % 64; i0 < a.k; i0 += stride) {  // wave-uniform trip count
    const int64_t i = i0 + threadIdx.x % 64;
    const bool mine = i < a.k;
    const int32_t v = mine ? a.ids[i] : 0;
    int64_t j = mine ? a.offsets[v] : 0;
    const int64_t j1 = mine ? a.offsets[v + 1] : 0;
    while (__any(j < j1)) {
      int32_t e[kClipUnroll], src[kClipUnroll];
#pragma unroll
      for (int u = 0; u < kClipUnroll; ++u) {
        const bool in = j + u < j1;
        e[u] = in ? a.edge[j + u] : -1;
        src[u] = in ? a.src[j + u] : -1;
      }
      bool take[kClipUnroll];
#pragma unroll
      for (int u = 0; u < kClipUnroll; ++u) {
        take[u] = false;
        if (e[u] < 0) continue;
        const uint8_t act = a.active[e[u]];
        const int64_t ex = a.expiry[e[u]];
        take[u] = act && !(ex >= 0 && a.now_us > ex);
      }
#pragma unroll
      for (int u = 0; u < kClipUnroll; ++u) {
        if (!take[u]) continue;
        // claim the bond: the same vouchee may appear twice in one storm, and a bond
        // is released (and its voucher clipped) once — as the sequential engine does
        const uintptr_t addr = reinterpret_cast<uintptr_t>(a.active + e[u]);
        unsigned int* word = reinterpret_cast<unsigned int*>(addr & ~uintptr_t(3));
        const unsigned int shift = static_cast<unsigned int>(addr & 3u) * 8u;
        const unsigned int old = atomicAnd(word, ~(0xffu << shift));
        take[u] = ((old >> shift) & 0xffu) != 0u;
        if (take[u]) a.released[e[u]] = a.now_us;
      }
      int mine_n = 0;
#pragma unroll
      for (int u = 0; u < kClipUnroll; ++u) mine_n += take[u] ? 1 : 0;
      // wave-aggregated slots: prefix over lanes of their release counts
      int pre = mine_n;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(pre, d, 64);
        if ((threadIdx.x % 64) >= d) pre += y;
      }
      const int total = __shfl(pre, 63, 64);
      unsigned long long slot0 = 0;
      if ((threadIdx.x % 64) == 63 && total > 0) slot0 = atomicAdd(a.cursor, static_cast<unsigned long long>(total));
      slot0 = __shfl(slot0, 63, 64);
      unsigned long long slot = slot0 + static_cast<unsigned long long>(pre - mine_n);
#pragma unroll
      for (int u = 0; u < kClipUnroll; ++u) {
        if (!take[u]) continue;
        if (slot < static_cast<unsigned long long>(a.cap)) {
          a.pair_id[slot] = src[u];
          a.pair_factor[slot] = 1.0 - a.omega;
        }
        ++slot;
      }
      j += kClipUnroll;
    }
  }
}

// X02 apply, sparse: only the touched agents are read or written.  Phase 1
// multiplies each gathered clip factor into a persistent all-ones factor vector
// (CAS loop: fp64 has no atomic multiply); phase 2 takes each product back with
// an exchange to 1.0 — the first taker of an agent applies σ = max(σ·Π, floor)
// and later takers see 1.0 and skip — leaving the factor vector all-ones for the
// next step; phase 3 zeroes the blacklisted agents.  Product order across
// duplicate pairs is not fixed (fp64 rounding may differ in the last bit from a
// sequential product; the exact path is collectives.merge_slash_sparse).
struct X02Args {
  int64_t npairs, nbl;
  double floor;
  const int32_t* pair_id;    // [npairs] (−1 = unused)
  const double* pair_f;      // [npairs]
  const int32_t* bl;         // [nbl] (−1 = unused)
  double* factor;            // [A] all ones between calls
  double* sigma;             // [A]
  const int32_t* bl_code;    // [nbl] merge code per blacklist entry (null: all 2), see below
  int32_t phase;             // x02_blacklist_kernel pass: 1 floors code-1 entries, 2 zeroes code-2 entries
};

__device__ void atomic_mul(double* p, double f) {
  unsigned long long* a = reinterpret_cast<unsigned long long*>(p);
  unsigned long long old = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), assumed;
  do {
    assumed = old;
    const double nv = __longlong_as_double(static_cast<long long>(assumed)) * f;
    old = atomicCAS(a, assumed, static_cast<unsigned long long>(__double_as_longlong(nv)));
  } while (assumed != old);
}

__global__ __launch_bounds__(256) void x02_mul_kernel(X02Args a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.npairs && a.pair_id[i] >= 0) atomic_mul(a.factor + a.pair_id[i], a.pair_f[i]);
}

__global__ __launch_bounds__(256) void x02_apply_kernel(X02Args a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.npairs && a.pair_id[i] >= 0) {
    const int32_t id = a.pair_id[i];
    const double prod = __longlong_as_double(static_cast<long long>(
        atomicExch(reinterpret_cast<unsigned long long*>(a.factor + id),
                   static_cast<unsigned long long>(__double_as_longlong(1.0)))));
    if (prod < 1.0) {
      const double v = a.sigma[id] * prod;
      a.sigma[id] = v < a.floor ? a.floor : v;
    }
  }
}

// Blacklist codes (the exact merge's convention, collectives.merge_slash_effects):
// 2 = blacklisted → σ 0; 1 = blacklisted and then clipped on its rank → the floor.
// Across ranks the larger code wins (MAX): pass 1 floors the code-1 agents, pass 2
// zeroes the code-2 agents afterwards.
__host__ __device__ __forceinline__ int32_t x02_code(const X02Args& a, int64_t i) { return a.bl_code ? a.bl_code[i] : 2; }

__global__ __launch_bounds__(256) void x02_blacklist_kernel(X02Args a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.nbl && a.bl[i] >= 0) {
    const int32_t c = x02_code(a, i);
    if (a.phase == 1 && c == 1) a.sigma[a.bl[i]] = a.floor;
    if (a.phase == 2 && c >= 2) a.sigma[a.bl[i]] = 0.0;
  }
}

int grid_for(int64_t n) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) cus = p.multiProcessorCount;
  }
  const int64_t need = (n + 255) / 256;
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(need, 4LL * cus)));
}

template <class T>
T* P(const py::dict& d, const char* k) {
  return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}

template <class T>
T* Popt(const py::dict& d, const char* k) {
  return d.contains(k) && !d[k].is_none() ? P<T>(d, k) : nullptr;
}

ExposureArgs to_exposure(const py::dict& d) {
  return ExposureArgs{d["agents"].cast<int64_t>(), d["now_us"].cast<int64_t>(), P<const int64_t>(d, "offsets"),
                      P<const double>(d, "bonded"), Popt<const uint8_t>(d, "active"),
                      Popt<const int64_t>(d, "expiry"), P<double>(d, "out"), Popt<const int32_t>(d, "index")};
}

ClipArgs to_clip(const py::dict& d) {
  return ClipArgs{d["k"].cast<int64_t>(), d["cap"].cast<int64_t>(), d["now_us"].cast<int64_t>(),
                  d["omega"].cast<double>(), P<const int32_t>(d, "ids"), P<const int64_t>(d, "offsets"),
                  P<const int32_t>(d, "src"), P<const int32_t>(d, "edge"), P<uint8_t>(d, "active"),
                  P<int64_t>(d, "released"), P<const int64_t>(d, "expiry"), P<int32_t>(d, "pair_id"),
                  P<double>(d, "pair_factor"), P<unsigned long long>(d, "cursor")};
}

X02Args to_x02(const py::dict& d) {
  return X02Args{d["npairs"].cast<int64_t>(), d["nbl"].cast<int64_t>(), d["floor"].cast<double>(),
                 P<const int32_t>(d, "pair_id"), P<const double>(d, "pair_f"), P<const int32_t>(d, "bl"),
                 P<double>(d, "factor"), P<double>(d, "sigma"),
                 d.contains("bl_code") ? P<const int32_t>(d, "bl_code") : nullptr, 0};
}

}  // namespace

namespace host {

void register_global_liability(py::module_& m) {
  m.def(
      "agent_exposure",
      [](const py::dict& d, uintptr_t stream) {
        const ExposureArgs a = to_exposure(d);
        py::gil_scoped_release nogil;
        if (a.agents <= 0) return;
        const int64_t blocks = (a.agents + 64 * kSegWaves - 1) / (64 * kSegWaves);
        hipLaunchKernelGGL(agent_exposure_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(64 * kSegWaves), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "agent_exposure");
      },
      py::arg("args"), py::arg("stream"));
  m.def("agent_exposure_host", [](const py::dict& d) {
    const ExposureArgs a = to_exposure(d);
    for (int64_t r = 0; r < a.agents; ++r) a.out[r] = exposure_row(a, r);
  });
  m.def(
      "slash_clip",
      [](const py::dict& d, uintptr_t stream) {
        const ClipArgs a = to_clip(d);
        py::gil_scoped_release nogil;
        hipLaunchKernelGGL(slash_clip_kernel, dim3(grid_for(a.k)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "slash_clip");
      },
      py::arg("args"), py::arg("stream"));
  m.def(
      "x02_apply",
      [](const py::dict& d, uintptr_t stream) {
        const X02Args a = to_x02(d);
        py::gil_scoped_release nogil;
        hipStream_t st = reinterpret_cast<hipStream_t>(stream);
        const int gp = static_cast<int>((std::max<int64_t>(a.npairs, 1) + 255) / 256);
        const int gb = static_cast<int>((std::max<int64_t>(a.nbl, 1) + 255) / 256);
        hipLaunchKernelGGL(x02_mul_kernel, dim3(gp), dim3(256), 0, st, a);
        hipLaunchKernelGGL(x02_apply_kernel, dim3(gp), dim3(256), 0, st, a);
        X02Args b = a;
        if (a.bl_code) {
          b.phase = 1;
          hipLaunchKernelGGL(x02_blacklist_kernel, dim3(gb), dim3(256), 0, st, b);
        }
        b.phase = 2;
        hipLaunchKernelGGL(x02_blacklist_kernel, dim3(gb), dim3(256), 0, st, b);
        check_hip(hipGetLastError(), "x02_apply");
      },
      py::arg("args"), py::arg("stream"));
  m.def("x02_apply_host", [](const py::dict& d) {
    const X02Args a = to_x02(d);
    for (int64_t i = 0; i < a.npairs; ++i)
      if (a.pair_id[i] >= 0) a.factor[a.pair_id[i]] *= a.pair_f[i];
    for (int64_t i = 0; i < a.npairs; ++i) {
      if (a.pair_id[i] < 0) continue;
      const int32_t id = a.pair_id[i];
      const double prod = a.factor[id];
      a.factor[id] = 1.0;
      if (prod < 1.0) {
        const double v = a.sigma[id] * prod;
        a.sigma[id] = v < a.floor ? a.floor : v;
      }
    }
    for (int phase = 1; phase <= 2; ++phase)
      for (int64_t i = 0; i < a.nbl; ++i) {
        if (a.bl[i] < 0) continue;
        const int32_t c = x02_code(a, i);
        if (phase == 1 && c == 1) a.sigma[a.bl[i]] = a.floor;
        if (phase == 2 && c >= 2) a.sigma[a.bl[i]] = 0.0;
      }
  });
  m.def("slash_clip_host", [](const py::dict& d) {
    const ClipArgs a = to_clip(d);
    for (int64_t i = 0; i < a.k; ++i) {
      const int32_t v = a.ids[i];
      for (int64_t j = a.offsets[v]; j < a.offsets[v + 1]; ++j) {
        const int32_t e = a.edge[j];
        if (!a.active[e] || (a.expiry[e] >= 0 && a.now_us > a.expiry[e])) continue;
        a.active[e] = 0;
        a.released[e] = a.now_us;
        const unsigned long long slot = (*a.cursor)++;
        if (slot < static_cast<unsigned long long>(a.cap)) {
          a.pair_id[slot] = a.src[j];
          a.pair_factor[slot] = 1.0 - a.omega;
        }
      }
    }
  });
}

}  // namespace host
}  // namespace ahv
