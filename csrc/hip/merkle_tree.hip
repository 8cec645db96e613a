// K09 — work-parallel Merkle root of one long audit chain (reference
// audit/delta.py:117-134).
//
// The reference pairs nodes level by level and duplicates the last node of an
// odd level.  Level k of that tree has ceil(n / 2^k) nodes, and an aligned block
// of 2^L leaves is a complete subtree — except the last block, whose odd local
// levels are exactly the global odd levels.  So a pass reduces L levels at once:
// workgroup b turns leaves [b·2^L, (b+1)·2^L) into node b of level L, hashing
// the last block's unpaired node with itself at every level where its count is
// odd (a single trailing leaf is lifted L levels by self-pairing, as the global
// tree does).  Passes repeat on the level-L nodes with L = min(9, ⌈log2 count⌉)
// until one node is left; the last pass stops exactly at the root.
//
// Geometry (gfx950): 256 threads (4 waves) per workgroup, 2^L ≤ 512 leaves.
// Level 0 reads the leaf digests straight from HBM (each thread two 32-byte
// leaves as 16-byte loads) and writes its parent into LDS; levels 1..L-1 run in
// LDS with a workgroup barrier per level.  A node is sha256(hex(l) || hex(r)):
// 128 ASCII bytes = 3 compressions, digest → hex words in registers.  Active
// lanes halve per level (256, 128, 64, 32, …): with several workgroups resident
// per CU the idle waves' slots go to other blocks, so passes run near the VALU
// issue rate — this kernel is compute-bound on the SHA rounds.
//
// LDS layout: node j at word 9·j (a 36-byte stride) — consecutive lanes read
// nodes 2t and 2t+1, and the odd stride spreads each lane's eight words over
// different banks.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>

#include "ahv/launch.h"
#include "ahv/sha256.h"

namespace py = pybind11;

namespace ahv {
namespace {

constexpr int kTreeThreads = 256;
constexpr int kMaxLevels = 9;  // 512 leaves per workgroup
constexpr int kStride = 9;     // LDS words per node

struct TreeArgs {
  int64_t count;        // nodes at the input level
  int32_t levels;       // levels reduced by this pass (1..9)
  const uint32_t* in;   // [count][8]
  uint32_t* out;        // [ceil(count / 2^levels)][8]
};

AHV_HD int64_t ceil_shift(int64_t n, int s) { return (n + (int64_t(1) << s) - 1) >> s; }

__global__ __launch_bounds__(kTreeThreads) void merkle_tree_pass_kernel(TreeArgs a) {
  __shared__ uint32_t lds[kTreeThreads * kStride];
  const int64_t span = int64_t(1) << a.levels;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * span;
  const int t = threadIdx.x;
  int64_t c = std::min<int64_t>(span, a.count - base);  // nodes at the current local level
  // level 0: leaves from HBM → parents in LDS
  {
    const int64_t m = (c + 1) / 2;
    if (t < m) {
      uint32_t l[8], r[8], o[8];
      const uint4* pl = reinterpret_cast<const uint4*>(a.in + (base + 2 * t) * 8);
      const uint4 l0 = pl[0], l1 = pl[1];
      l[0] = l0.x; l[1] = l0.y; l[2] = l0.z; l[3] = l0.w; l[4] = l1.x; l[5] = l1.y; l[6] = l1.z; l[7] = l1.w;
      if (2 * t + 1 < c) {
        const uint4 r0 = pl[2], r1 = pl[3];
        r[0] = r0.x; r[1] = r0.y; r[2] = r0.z; r[3] = r0.w; r[4] = r1.x; r[5] = r1.y; r[6] = r1.z; r[7] = r1.w;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = l[k];
      }
      merkle_node(l, r, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) lds[t * kStride + k] = o[k];
    }
    c = m;
  }
  __syncthreads();
  for (int lev = 1; lev < a.levels; ++lev) {
    const int64_t m = (c + 1) / 2;
    uint32_t o[8];
    if (t < m) {
      uint32_t l[8], r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) l[k] = lds[(2 * t) * kStride + k];
      if (2 * t + 1 < c) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = lds[(2 * t + 1) * kStride + k];
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = l[k];
      }
      merkle_node(l, r, o);
    }
    __syncthreads();  // every read of this level precedes the overwrite
    if (t < m) {
#pragma unroll
      for (int k = 0; k < 8; ++k) lds[t * kStride + k] = o[k];
    }
    __syncthreads();
    c = m;
  }
  if (t < 2) {  // the block's node: 8 words, two 16-byte stores
    uint4 v;
    v.x = lds[4 * t + 0];
    v.y = lds[4 * t + 1];
    v.z = lds[4 * t + 2];
    v.w = lds[4 * t + 3];
    reinterpret_cast<uint4*>(a.out + static_cast<int64_t>(blockIdx.x) * 8)[t] = v;
  }
}

// Host twin: the same pass, one block at a time (CPU tests; the semantic oracle
// is the reference algorithm in hypervisor.audit / _C.merkle_root).
void merkle_tree_pass_host(const TreeArgs& a) {
  const int64_t span = int64_t(1) << a.levels;
  const int64_t nb = ceil_shift(a.count, a.levels);
  std::vector<uint32_t> cur;
  for (int64_t b = 0; b < nb; ++b) {
    int64_t c = std::min<int64_t>(span, a.count - b * span);
    cur.assign(a.in + b * span * 8, a.in + (b * span + c) * 8);
    for (int lev = 0; lev < a.levels; ++lev) {
      const int64_t m = (c + 1) / 2;
      for (int64_t i = 0; i < m; ++i) {
        uint32_t o[8];
        const uint32_t* l = &cur[2 * i * 8];
        const uint32_t* r = (2 * i + 1 < c) ? &cur[(2 * i + 1) * 8] : l;
        merkle_node(l, r, o);
        std::copy(o, o + 8, &cur[i * 8]);
      }
      c = m;
    }
    std::copy(cur.begin(), cur.begin() + 8, a.out + b * 8);
  }
}

TreeArgs to_tree(const py::dict& d) {
  TreeArgs a{d["count"].cast<int64_t>(), d["levels"].cast<int32_t>(),
             reinterpret_cast<const uint32_t*>(d["in"].cast<uintptr_t>()),
             reinterpret_cast<uint32_t*>(d["out"].cast<uintptr_t>())};
  if (a.levels < 1 || a.levels > kMaxLevels) throw py::value_error("merkle_tree_pass: levels must be 1..9");
  if (a.count < 1) throw py::value_error("merkle_tree_pass: empty level");
  return a;
}

}  // namespace

void kernels_merkle_tree(std::vector<KernelEntry>& out) {
  out.push_back({"merkle_tree_pass_kernel", reinterpret_cast<const void*>(&merkle_tree_pass_kernel)});
}

namespace host {

void register_merkle_tree(py::module_& m) {
  m.def(
      "merkle_tree_pass",
      [](const py::dict& d, uintptr_t stream) {
        const TreeArgs a = to_tree(d);
        py::gil_scoped_release nogil;
        const int64_t blocks = ceil_shift(a.count, a.levels);
        hipLaunchKernelGGL(merkle_tree_pass_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kTreeThreads), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "merkle_tree_pass");
      },
      py::arg("args"), py::arg("stream"));
  m.def("merkle_tree_pass_host", [](const py::dict& d) {
    const TreeArgs a = to_tree(d);
    py::gil_scoped_release nogil;
    merkle_tree_pass_host(a);
  });
}

}  // namespace host
}  // namespace ahv
