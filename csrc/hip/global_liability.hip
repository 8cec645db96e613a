// Agent-global liability kernels for session-sharded multi-GPU runs (SURVEY
// §2.13 X01/X02): the per-rank partials that the cross-rank collectives combine.
//
//   agent_exposure  (K04, global form) — exposure[a] = Σ live bonded amounts of
//                   the edges agent a vouches with (reference vouching.py:157-166
//                   summed over every session the rank owns).  Edges are stored
//                   CSR by voucher in creation order; one lane per agent walks its
//                   row sequentially, so each partial is the exact creation-order
//                   fp64 sum.  The [A] fp64 vector is then all-reduced over ranks
//                   (X01: 8 MB for 1 M agents, RCCL over xGMI).
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
  const double* bonded;    // [E]
  const uint8_t* active;   // [E]
  const int64_t* expiry;   // [E] (-1 = never)
  double* out;             // [A]
};

AHV_HD double exposure_row(const ExposureArgs& a, int64_t r) {
  double s = 0.0;
  for (int64_t e = a.offsets[r]; e < a.offsets[r + 1]; ++e)
    if (a.active[e] && (a.expiry[e] < 0 || a.now_us <= a.expiry[e])) s += a.bonded[e];
  return s;
}

__global__ __launch_bounds__(256) void agent_exposure_kernel(ExposureArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < a.agents; r += stride)
    a.out[r] = exposure_row(a, r);
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

__global__ __launch_bounds__(256) void slash_clip_kernel(ClipArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.k; i += stride) {
    const int32_t v = a.ids[i];
    for (int64_t j = a.offsets[v]; j < a.offsets[v + 1]; ++j) {
      const int32_t e = a.edge[j];
      if (!a.active[e] || (a.expiry[e] >= 0 && a.now_us > a.expiry[e])) continue;
      a.active[e] = 0;
      a.released[e] = a.now_us;
      const unsigned long long slot = atomicAdd(a.cursor, 1ull);
      if (slot < static_cast<unsigned long long>(a.cap)) {
        a.pair_id[slot] = a.src[j];
        a.pair_factor[slot] = 1.0 - a.omega;
      }
    }
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

ExposureArgs to_exposure(const py::dict& d) {
  return ExposureArgs{d["agents"].cast<int64_t>(), d["now_us"].cast<int64_t>(), P<const int64_t>(d, "offsets"),
                      P<const double>(d, "bonded"), P<const uint8_t>(d, "active"), P<const int64_t>(d, "expiry"),
                      P<double>(d, "out")};
}

ClipArgs to_clip(const py::dict& d) {
  return ClipArgs{d["k"].cast<int64_t>(), d["cap"].cast<int64_t>(), d["now_us"].cast<int64_t>(),
                  d["omega"].cast<double>(), P<const int32_t>(d, "ids"), P<const int64_t>(d, "offsets"),
                  P<const int32_t>(d, "src"), P<const int32_t>(d, "edge"), P<uint8_t>(d, "active"),
                  P<int64_t>(d, "released"), P<const int64_t>(d, "expiry"), P<int32_t>(d, "pair_id"),
                  P<double>(d, "pair_factor"), P<unsigned long long>(d, "cursor")};
}

}  // namespace

namespace host {

void register_global_liability(py::module_& m) {
  m.def(
      "agent_exposure",
      [](const py::dict& d, uintptr_t stream) {
        const ExposureArgs a = to_exposure(d);
        py::gil_scoped_release nogil;
        hipLaunchKernelGGL(agent_exposure_kernel, dim3(grid_for(a.agents)), dim3(256), 0,
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
