// Batched kernels over the device store's resident tables (one device state).
//
// The public API's audit chain lives in the store (csrc/include/ahv/store.h):
// delta rows (d_off/d_len/d_prev/d_hole/d_sess/d_turn + d_hash) and the
// canonical-JSON records in the payload arena.  `store_verify` is K10 over those
// rows as they are — no host re-render, no upload of payload bytes: one lane per
// delta re-hashes its arena record (system-scope loads: the arena is
// host-written fine-grained memory), compares the digest with the row's d_hash,
// and checks the parent link — the row's d_prev is the previous row of its chain
// (same session, turn − 1) and the 66 bytes at d_hole are exactly the quoted hex
// of that row's digest (or there is no hole and no predecessor for turn 1).
//
// Reference semantics: audit/delta.py:117-152 (verify_chain without the
// reference's re-hash-then-compare self-repair, Q02).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <algorithm>

#include "ahv/launch.h"
#include "ahv/store.h"

namespace py = pybind11;

namespace ahv {
namespace {

using store::ld32f;

struct VerifyRowsArgs {
  int64_t n;                 // rows to check
  const int32_t* rows;       // [n] delta rows, chains consecutive, each in turn order
  const uint8_t* first;      // [n] 1 where a chain starts
  const uint8_t* payload;    // arena
  int64_t payload_cap;
  const int64_t* d_off;
  const int32_t* d_len;
  const int32_t* d_prev;
  const int32_t* d_hole;
  const int32_t* d_sess;
  const int32_t* d_turn;
  const uint32_t* d_hash;    // [D, 8]
  int64_t cap_d;
  uint8_t* ok;               // [n] out: 1 = digest and parent link verified
};

AHV_HD uint8_t verify_row(const VerifyRowsArgs& a, int64_t i) {
  const int32_t d = a.rows[i];
  if (d < 0 || d >= a.cap_d) return 0;
  const int64_t off = a.d_off[d];
  const int64_t len = a.d_len[d];
  if (off < 0 || len <= 0 || off + len > a.payload_cap) return 0;
  uint32_t h[8];
  store::sha256_fine(a.payload + off, static_cast<uint64_t>(len), h);
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) ok = ok && h[k] == a.d_hash[8 * static_cast<int64_t>(d) + k];
  const int32_t hole = a.d_hole[d];
  if (a.first[i]) {
    ok = ok && a.d_prev[d] < 0 && hole < 0 && a.d_turn[d] == 1;
  } else {
    const int32_t p = a.rows[i - 1];
    ok = ok && a.d_prev[d] == p && p >= 0 && a.d_sess[p] == a.d_sess[d] && a.d_turn[p] + 1 == a.d_turn[d] &&
         hole >= 0 && hole + 66 <= len;
    if (ok) {
      // the record's quoted parent: '"' + 64 lowercase hex + '"' at byte `hole`
      const uint8_t* q = a.payload + off + hole;
      for (int k = 0; k < 66 && ok; ++k) {
        const uint64_t b = static_cast<uint64_t>(off + hole + k);
        const uint32_t w = ld32f(a.payload + (b & ~uint64_t(3)));
        const uint32_t ch = (w >> (8 * (b & 3))) & 0xffu;
        uint32_t want = 0x22u;
        if (k > 0 && k < 65) {
          const int nib = k - 1;
          want = hex_nibble((a.d_hash[8 * static_cast<int64_t>(p) + (nib >> 3)] >> (28 - 4 * (nib & 7))) & 15u);
        }
        ok = ch == want;
      }
      (void)q;
    }
  }
  return ok ? 1 : 0;
}

__global__ __launch_bounds__(256) void store_verify_kernel(VerifyRowsArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += stride)
    a.ok[i] = verify_row(a, i);
}

// K03/K04 over resident vouch lists: one lane per request walks the request's
// liability-session edge list in creation order (the store's linked list), so
// each sum has exactly the order of the scalar OP_SIGMA_EFF / OP_EXPOSURE
// commands (bit-identical fp64): mode 0 σ_eff = min(σ + ω·Σ bonded of live edges
// *into* `agent`, 1); mode 1 exposure = Σ bonded of live edges *from* `agent`.
struct SigmaBatchArgs {
  int64_t n;
  int32_t mode;
  int64_t now_us;
  const int32_t* vsess;    // [n] liability-session rows (-1: no bonds yet)
  const int32_t* agent;    // [n] vouchee (mode 0) / voucher (mode 1) agent ids
  const double* sigma;     // [n] σ (mode 0)
  const double* omega;     // [n] ω (mode 0)
  const int32_t* v_head;
  const int32_t* e_next;
  const int32_t* e_voucher;
  const int32_t* e_vouchee;
  const uint8_t* e_active;
  const int64_t* e_expiry;
  const double* e_bonded;
  int64_t cap_v;
  double* out;             // [n]
};

AHV_HD double sigma_batch_row(const SigmaBatchArgs& a, int64_t i) {
  const int32_t v = a.vsess[i];
  const int32_t who = a.agent[i];
  double acc = 0.0;
  if (v >= 0 && v < a.cap_v) {
    for (int32_t e = a.v_head[v]; e >= 0; e = a.e_next[e]) {
      const uint8_t act = a.e_active[e];
      const int64_t ex = a.e_expiry[e];
      const bool live = act && (ex < 0 || a.now_us <= ex);
      const int32_t x = a.mode == 0 ? a.e_vouchee[e] : a.e_voucher[e];
      if (live && x == who) acc += a.e_bonded[e];
    }
  }
  if (a.mode != 0) return acc;
  double s = a.sigma[i] + a.omega[i] * acc;
  return s > 1.0 ? 1.0 : s;
}

__global__ __launch_bounds__(256) void store_sigma_kernel(SigmaBatchArgs a) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += stride)
    a.out[i] = sigma_batch_row(a, i);
}

// Record moves between the payload arena and a contiguous device buffer (session
// migration between ranks, P08): record i is the `lens[i]` bytes at arena offset
// `offs[i]` ↔ buffer position `pos[i]`.  One 64-lane wave per record; the arena
// is fine-grained (host-visible) memory, read with system-scope word loads.
struct RecordMoveArgs {
  int64_t n;
  uint8_t* payload;
  int64_t payload_cap;
  const int64_t* offs;
  const int64_t* lens;
  const int64_t* pos;
  uint8_t* buf;
  int32_t to_arena;  // 0: arena → buf (pack), 1: buf → arena (unpack)
};

AHV_HD bool record_ok(const RecordMoveArgs& a, int64_t i) {
  return a.offs[i] >= 0 && a.lens[i] >= 0 && a.offs[i] + a.lens[i] <= a.payload_cap;
}

__global__ __launch_bounds__(256) void store_records_kernel(RecordMoveArgs a) {
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const int lane = threadIdx.x & 63;
  for (int64_t i = wave; i < a.n; i += nwaves) {
    if (!record_ok(a, i)) continue;
    const int64_t off = a.offs[i], len = a.lens[i], p = a.pos[i];
    for (int64_t j = lane; j < len; j += 64) {
      if (a.to_arena) {
        a.payload[off + j] = a.buf[p + j];
      } else {
        const uint64_t b = static_cast<uint64_t>(off + j);
        const uint32_t w = ld32f(a.payload + (b & ~uint64_t(3)));
        a.buf[p + j] = static_cast<uint8_t>((w >> (8 * (b & 3))) & 0xffu);
      }
    }
  }
}

void records_host(const RecordMoveArgs& a) {
  for (int64_t i = 0; i < a.n; ++i) {
    if (!record_ok(a, i)) continue;
    if (a.to_arena) std::copy(a.buf + a.pos[i], a.buf + a.pos[i] + a.lens[i], a.payload + a.offs[i]);
    else std::copy(a.payload + a.offs[i], a.payload + a.offs[i] + a.lens[i], a.buf + a.pos[i]);
  }
}

template <class T>
T* P(const py::dict& d, const char* k) {
  return reinterpret_cast<T*>(d[k].cast<uintptr_t>());
}

VerifyRowsArgs to_verify(const py::dict& d) {
  return VerifyRowsArgs{d["n"].cast<int64_t>(), P<const int32_t>(d, "rows"), P<const uint8_t>(d, "first"),
                        P<const uint8_t>(d, "payload"), d["payload_cap"].cast<int64_t>(), P<const int64_t>(d, "d_off"),
                        P<const int32_t>(d, "d_len"), P<const int32_t>(d, "d_prev"), P<const int32_t>(d, "d_hole"),
                        P<const int32_t>(d, "d_sess"), P<const int32_t>(d, "d_turn"), P<const uint32_t>(d, "d_hash"),
                        d["cap_d"].cast<int64_t>(), P<uint8_t>(d, "ok")};
}

SigmaBatchArgs to_sigma(const py::dict& d) {
  return SigmaBatchArgs{d["n"].cast<int64_t>(), d["mode"].cast<int32_t>(), d["now_us"].cast<int64_t>(),
                        P<const int32_t>(d, "vsess"), P<const int32_t>(d, "agent"), P<const double>(d, "sigma"),
                        P<const double>(d, "omega"), P<const int32_t>(d, "v_head"), P<const int32_t>(d, "e_next"),
                        P<const int32_t>(d, "e_voucher"), P<const int32_t>(d, "e_vouchee"),
                        P<const uint8_t>(d, "e_active"), P<const int64_t>(d, "e_expiry"),
                        P<const double>(d, "e_bonded"), d["cap_v"].cast<int64_t>(), P<double>(d, "out")};
}

RecordMoveArgs to_records(const py::dict& d) {
  return RecordMoveArgs{d["n"].cast<int64_t>(), P<uint8_t>(d, "payload"), d["payload_cap"].cast<int64_t>(),
                        P<const int64_t>(d, "offs"), P<const int64_t>(d, "lens"), P<const int64_t>(d, "pos"),
                        P<uint8_t>(d, "buf"), d["to_arena"].cast<int32_t>()};
}

}  // namespace

namespace host {

void register_store_views(py::module_& m) {
  m.def(
      "store_verify",
      [](const py::dict& d, uintptr_t stream) {
        const VerifyRowsArgs a = to_verify(d);
        py::gil_scoped_release nogil;
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((a.n + 255) / 256, 8192));
        hipLaunchKernelGGL(store_verify_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "store_verify");
      },
      py::arg("args"), py::arg("stream"));
  m.def(
      "store_sigma",
      [](const py::dict& d, uintptr_t stream) {
        const SigmaBatchArgs a = to_sigma(d);
        py::gil_scoped_release nogil;
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((a.n + 255) / 256, 8192));
        hipLaunchKernelGGL(store_sigma_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "store_sigma");
      },
      py::arg("args"), py::arg("stream"));
  m.def(
      "store_records",
      [](const py::dict& d, uintptr_t stream) {
        const RecordMoveArgs a = to_records(d);
        py::gil_scoped_release nogil;
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((a.n + 3) / 4, 16384));  // 4 waves per block
        hipLaunchKernelGGL(store_records_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                           reinterpret_cast<hipStream_t>(stream), a);
        check_hip(hipGetLastError(), "store_records");
      },
      py::arg("args"), py::arg("stream"));
  m.def("store_records_host", [](const py::dict& d) { records_host(to_records(d)); });
  m.def("store_sigma_host", [](const py::dict& d) {
    const SigmaBatchArgs a = to_sigma(d);
    for (int64_t i = 0; i < a.n; ++i) a.out[i] = sigma_batch_row(a, i);
  });
  m.def("store_verify_host", [](const py::dict& d) {
    const VerifyRowsArgs a = to_verify(d);
    for (int64_t i = 0; i < a.n; ++i) a.ok[i] = verify_row(a, i);
  });
}

}  // namespace host
}  // namespace ahv
