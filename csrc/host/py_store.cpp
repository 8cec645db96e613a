// Host runtime of the device state store (csrc/include/ahv/store.h).
//
// `Store` owns the transport between the Python API and the store tables:
//
//   gfx950:  command ring + staging area + audit payload arena in fine-grained
//            device memory (host writes them through the PCIe BAR), result slots
//            and bulk outputs in pinned host memory, and the resident worker
//            wave (csrc/hip/store_worker.hip) that executes commands.  The
//            worker idles out after a short quiet period and is relaunched on
//            demand, so it never holds its hardware queue for long.
//   cpu:     the same `store_exec` body runs inline on host-memory tables (the
//            CPU twin used by the CPU test suite and the reference oracle).
//
// The tables themselves are PyTorch tensors (allocated by
// agent_hypervisor_amd/models/store.py) passed in by data pointer.
#include <Python.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ahv/store.h"

namespace py = pybind11;

extern "C" int ahv_store_launch_worker(const ahv::store::Tables* t, const uint64_t* ring, int64_t nslots,
                                       uint64_t* res, uint8_t* bulk, uint64_t* alive, int64_t* tail,
                                       uint64_t idle_ticks, uint64_t max_ticks, int speculate, hipStream_t stream);

namespace ahv {
namespace host {

bool render_delta(PyObject* d, std::string& out, size_t* null_parent_at);

namespace {

using namespace ahv::store;

// The result slot of a sequence number was recycled by a later command.
struct ResultGone : std::exception {
  const char* what() const noexcept override { return "store result slot recycled"; }
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class Store {
 public:
  Store(int device, const py::dict& ptrs, const py::dict& caps, int64_t nslots, int64_t staging_bytes,
        int64_t bulk_bytes, int64_t idle_us, int64_t max_ms)
      : gpu_(device >= 0), device_(device), nslots_(nslots), staging_cap_(staging_bytes), bulk_cap_(bulk_bytes) {
    auto cap = [&](const char* k) { return caps[k].cast<int64_t>(); };
    t_.cap = Caps{cap("S"), cap("P"), cap("D"), cap("E"), cap("V"), cap("G"), cap("T"), cap("X"), cap("B")};
#define AHV_PTR(name, type, ext) t_.name = reinterpret_cast<type*>(ptrs[#name].cast<uintptr_t>());
    AHV_STORE_COLUMNS(AHV_PTR)
#undef AHV_PTR
    const size_t ring_bytes = static_cast<size_t>(nslots_) * kSlotWords * 8;
    const size_t res_bytes = static_cast<size_t>(nslots_) * kResWords * 8;
    if (gpu_) {
      hip_check(hipSetDevice(device_), "hipSetDevice");
      hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&ring_), ring_bytes, hipDeviceMallocFinegrained),
                "store ring");
      hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&staging_), static_cast<size_t>(staging_cap_),
                                      hipDeviceMallocFinegrained),
                "store staging");
      hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&payload_), static_cast<size_t>(t_.cap.B),
                                      hipDeviceMallocFinegrained),
                "store payload arena");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&res_), res_bytes, hipHostMallocCoherent), "store results");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&bulk_), static_cast<size_t>(bulk_cap_), hipHostMallocCoherent),
                "store bulk");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&alive_), 64, hipHostMallocCoherent), "store ctl");
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&tail_), 64, hipHostMallocCoherent), "store tail");
      hip_check(hipMemset(ring_, 0, ring_bytes), "memset ring");
      *tail_ = 0;
      hip_check(hipDeviceSynchronize(), "store init sync");
      hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "store stream");
      idle_ticks_ = static_cast<uint64_t>(idle_us) * 100;   // s_memrealtime: 100 MHz
      // worker feature bits: 1 = provisional Merkle roots on the idle hash engine,
      // 2 = capture prefix midstates on the command wave
      const char* sp = std::getenv("AHV_STORE_SPECULATE");
      const char* pf = std::getenv("AHV_STORE_PREFIX");
      speculate_ = ((sp == nullptr || std::atoi(sp) != 0) ? 1 : 0) | ((pf == nullptr || std::atoi(pf) != 0) ? 2 : 0);
      max_ticks_ = static_cast<uint64_t>(max_ms) * 100000;
    } else {
      ring_ = static_cast<uint64_t*>(std::calloc(ring_bytes / 8, 8));
      staging_ = static_cast<uint8_t*>(std::calloc(static_cast<size_t>(staging_cap_), 1));
      payload_ = static_cast<uint8_t*>(std::calloc(static_cast<size_t>(t_.cap.B), 1));
      res_ = static_cast<uint64_t*>(std::calloc(res_bytes / 8, 8));
      bulk_ = static_cast<uint8_t*>(std::calloc(static_cast<size_t>(bulk_cap_), 1));
      alive_ = static_cast<uint64_t*>(std::calloc(8, 8));
      if (!ring_ || !staging_ || !payload_ || !res_ || !bulk_ || !alive_) throw std::bad_alloc();
    }
    std::memset(res_, 0, res_bytes);
    *alive_ = 0;
    t_.payload = payload_;
    t_.staging = staging_;
  }

  ~Store() {
    try {
      close();
    } catch (...) {
    }
    if (gpu_) {
      (void)hipFree(ring_);
      (void)hipFree(staging_);
      (void)hipFree(payload_);
      (void)hipHostFree(res_);
      (void)hipHostFree(bulk_);
      (void)hipHostFree(alive_);
      (void)hipHostFree(tail_);
      if (stream_) (void)hipStreamDestroy(stream_);
    } else {
      std::free(ring_);
      std::free(staging_);
      std::free(payload_);
      std::free(res_);
      std::free(bulk_);
      std::free(alive_);
    }
  }

  // Stop the worker (if resident) and wait for its wave to drain.
  void close() {
    if (closed_) return;
    closed_ = true;
    if (gpu_ && launches_ > 0) {
      if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) != 0) {
        const uint64_t q = post_raw(OP_STOP, nullptr, 0, nullptr, 0);
        wait(q);
      }
      hip_check(hipStreamSynchronize(stream_), "store worker drain");
    }
  }

  // ------------------------------------------------------------ transport

  uint64_t post_raw(uint32_t op, const uint64_t* args, size_t nargs, const uint8_t* inl, size_t inl_bytes) {
    if (nargs > static_cast<size_t>(kArgs)) throw std::invalid_argument("too many store args");
    if (inl_bytes > static_cast<size_t>(kInlineWords) * 8) throw std::invalid_argument("inline payload too large");
    const uint64_t q = next_++;
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    // the slot's previous occupant must have completed
    if (q >= static_cast<uint64_t>(nslots_)) wait(q - static_cast<uint64_t>(nslots_));
    uint64_t w[kSlotWords];
    std::memset(w, 0, sizeof w);
    w[1] = op;
    for (size_t k = 0; k < nargs; ++k) w[3 + k] = args[k];
    if (inl_bytes) std::memcpy(w + 16, inl, inl_bytes);
    uint64_t x = w[1];
    for (int k = 3; k < kSlotWords; ++k) x ^= w[k];
    w[2] = x;
    ++posted_;
    if (!gpu_) {
      uint64_t* slot = ring_ + idx * kSlotWords;
      std::memcpy(slot, w, sizeof w);
      Cmd c;
      c.op = op;
      for (int k = 0; k < kArgs; ++k) c.a[k] = w[3 + k];
      c.inl = slot + 16;
      uint64_t* r = res_ + idx * kResWords;
      thread_local uint32_t lds[kLdsWords];
      const Lanes L{0, 1, lds};
      store_exec(L, t_, c, q, r, bulk_, nullptr);
      r[0] = q + 1;
      return q;
    }
    volatile uint64_t* slot = ring_ + idx * kSlotWords;
    for (int k = 1; k < kSlotWords; ++k) slot[k] = w[k];
    _mm_sfence();
    slot[0] = q + 1;
    _mm_sfence();
    ensure_worker();
    return q;
  }

  void ensure_worker() {
    if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) != 0) return;
    __atomic_store_n(alive_, 1ull, __ATOMIC_RELEASE);
    const int rc = ahv_store_launch_worker(&t_, ring_, nslots_, res_, bulk_, alive_, tail_, idle_ticks_, max_ticks_, speculate_,
                                           stream_);
    if (rc != 0) {
      __atomic_store_n(alive_, 0ull, __ATOMIC_RELEASE);
      throw std::runtime_error(std::string("store worker launch failed: ") +
                               hipGetErrorString(static_cast<hipError_t>(rc)));
    }
    ++launches_;
  }

  const uint64_t* wait(uint64_t q) {
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    volatile uint64_t* r = res_ + idx * kResWords;
    if (q >= next_) throw std::out_of_range("store: sequence number not posted");
    if (r[0] >= q + 1 + static_cast<uint64_t>(nslots_)) throw ResultGone();
    if (r[0] >= q + 1) return const_cast<uint64_t*>(r);
    if (!gpu_) throw std::logic_error("store: result missing on the host twin");
    uint64_t spins = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const uint64_t v = r[0];
      if (v >= q + 1) break;
      if ((++spins & 1023u) == 0) {
        // the worker idled out between our post and its last poll: relaunch
        if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) == 0) ensure_worker();
        if ((spins & 0xfffffu) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s_)) {
          throw std::runtime_error("store: command " + std::to_string(q) + " timed out (worker not responding)");
        }
      }
      _mm_pause();
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return const_cast<uint64_t*>(r);
  }

  // ------------------------------------------------------------ Python API

  uint64_t post(uint32_t op, const std::vector<int64_t>& args, const py::object& inl) {
    std::string buf;
    if (!inl.is_none()) buf = inl.cast<std::string>();
    return post_raw(op, reinterpret_cast<const uint64_t*>(args.data()), args.size(),
                    reinterpret_cast<const uint8_t*>(buf.data()), buf.size());
  }

  // post + wait; returns (r[1], r[2], ..., r[nres]) as ints (status first)
  py::tuple call(uint32_t op, const std::vector<int64_t>& args, int nres, const py::object& inl) {
    const uint64_t q = post(op, args, inl);
    const uint64_t* r = wait(q);
    py::tuple out(nres);
    for (int k = 0; k < nres; ++k) out[k] = py::int_(static_cast<int64_t>(r[1 + k]));
    return out;
  }

  // Results of an earlier post, or None once its slot has been recycled.
  py::object result(uint64_t q, int nres) {
    const uint64_t* r;
    try {
      r = wait(q);
    } catch (const ResultGone&) {
      return py::none();
    }
    py::tuple out(nres);
    for (int k = 0; k < nres; ++k) out[k] = py::int_(static_cast<int64_t>(r[1 + k]));
    return out;
  }

  // Everything posted so far has completed: on the device a NOP is executed only
  // after the hash engine's queue has drained, and results complete in order
  // otherwise.
  void drain() {
    if (next_ == 0) return;
    if (!gpu_) return;
    wait(post_raw(OP_NOP, nullptr, 0, nullptr, 0));
  }

  // Copy bytes into the staging area; returns their offset.  Wrapping first
  // drains the queue, so no pending command still reads the overwritten bytes.
  int64_t stage(const py::bytes& b) {
    std::string_view v = b;
    return stage_raw(reinterpret_cast<const uint8_t*>(v.data()), v.size());
  }

  int64_t stage_raw(const uint8_t* p, size_t n) {
    const size_t need = (n + 63) & ~size_t(63);
    if (need > static_cast<size_t>(staging_cap_)) throw std::length_error("staging area too small");
    if (stage_head_ + need > static_cast<size_t>(staging_cap_)) {
      drain();
      stage_head_ = 0;
    }
    const size_t off = stage_head_;
    stage_head_ += need;
    std::memcpy(staging_ + off, p, n);
    if (gpu_) _mm_sfence();
    return static_cast<int64_t>(off);
  }

  py::bytes bulk(int64_t off, int64_t n) const {
    if (off < 0 || n < 0 || off + n > bulk_cap_) throw std::out_of_range("bulk range");
    return py::bytes(reinterpret_cast<const char*>(bulk_ + off), static_cast<size_t>(n));
  }

  py::bytes payload(int64_t off, int64_t n) const {
    if (off < 0 || n < 0 || off + n > t_.cap.B) throw std::out_of_range("payload range");
    std::string out(static_cast<size_t>(n), '\0');
    if (gpu_) {
      hip_check(hipMemcpy(out.data(), payload_ + off, static_cast<size_t>(n), hipMemcpyDeviceToHost), "payload read");
    } else {
      std::memcpy(out.data(), payload_ + off, static_cast<size_t>(n));
    }
    return py::bytes(out);
  }

  // DeltaEngine.capture on the device: render the canonical payload around a
  // null parent, lay it out in the payload arena with a 66-byte hole for the
  // quoted parent digest (turn > 1), and post OP_DELTA_CAPTURE.  The device
  // splices the chain head into the hole and hashes (K08).
  // Returns (delta index, payload offset, payload length, sequence).
  py::tuple capture(int64_t slot, int64_t turn, int64_t ts_us, py::handle delta) {
    thread_local std::string buf;
    size_t at = 0;
    if (!render_delta(delta.ptr(), buf, &at)) return py::make_tuple(-1, -1, -1, -1);
    return capture_rendered(slot, turn, ts_us, buf, at);
  }

  // Same, for a payload the caller rendered (json.dumps fallback for exotic field
  // types): `null_at` is the offset of the parent's `null`.
  py::tuple capture_bytes(int64_t slot, int64_t turn, int64_t ts_us, const py::bytes& payload, int64_t null_at) {
    std::string buf = payload;
    if (null_at < 0 || static_cast<size_t>(null_at) + 4 > buf.size() || buf.compare(null_at, 4, "null") != 0)
      throw std::invalid_argument("capture_bytes: null_at does not point at the parent's null");
    return capture_rendered(slot, turn, ts_us, buf, static_cast<size_t>(null_at));
  }

  py::tuple capture_rendered(int64_t slot, int64_t turn, int64_t ts_us, const std::string& buf, size_t at) {
    const bool hole = turn > 1;
    const size_t len = hole ? buf.size() - 4 + 66 : buf.size();
    if (static_cast<int64_t>(len) > t_.cap.B) throw std::length_error("audit payload larger than the arena");
    if (payload_head_ + static_cast<int64_t>(len) > t_.cap.B) payload_head_ = 0;  // ring: oldest records recycled
    const int64_t off = payload_head_;
    payload_head_ += static_cast<int64_t>((len + 63) & ~size_t(63));
    uint8_t* dst = payload_ + off;
    if (hole) {
      std::memcpy(dst, buf.data(), at);
      std::memcpy(dst + at + 66, buf.data() + at + 4, buf.size() - at - 4);
    } else {
      std::memcpy(dst, buf.data(), buf.size());
    }
    if (gpu_) _mm_sfence();
    const int64_t didx = delta_head_;
    delta_head_ = (delta_head_ + 1) % t_.cap.D;
    uint64_t a[7] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(didx), static_cast<uint64_t>(turn),
                     static_cast<uint64_t>(ts_us), static_cast<uint64_t>(off), static_cast<uint64_t>(len),
                     hole ? static_cast<uint64_t>(at) : ~0ull};
    const uint64_t q = post_raw(OP_DELTA_CAPTURE, a, 7, nullptr, 0);
    return py::make_tuple(didx, off, static_cast<int64_t>(len), q);
  }

  // Append a complete record to the payload arena (checkpoint restore); returns
  // its offset.  The device re-hashes restored records before they are trusted.
  int64_t payload_append(const py::bytes& b) {
    std::string_view v = b;
    const int64_t len = static_cast<int64_t>(v.size());
    if (len > t_.cap.B) throw std::length_error("audit payload larger than the arena");
    if (payload_head_ + len > t_.cap.B) payload_head_ = 0;
    const int64_t off = payload_head_;
    payload_head_ += (len + 63) & ~int64_t(63);
    std::memcpy(payload_ + off, v.data(), v.size());
    if (gpu_) _mm_sfence();
    return off;
  }

  int64_t alloc_delta() {
    const int64_t d = delta_head_;
    delta_head_ = (delta_head_ + 1) % t_.cap.D;
    return d;
  }

  py::dict info() const {
    py::dict d;
    d["gpu"] = gpu_;
    d["device"] = device_;
    d["posted"] = posted_;
    d["launches"] = launches_;
    d["nslots"] = nslots_;
    d["payload_head"] = payload_head_;
    d["delta_head"] = delta_head_;
    return d;
  }

  int64_t delta_head() const { return delta_head_; }
  void set_delta_head(int64_t v) { delta_head_ = v; }
  int64_t payload_head() const { return payload_head_; }
  void set_payload_head(int64_t v) { payload_head_ = v; }
  void set_timeout(int s) { timeout_s_ = s; }
  bool gpu() const { return gpu_; }

 private:
  bool gpu_;
  int device_;
  int64_t nslots_;
  int64_t staging_cap_;
  int64_t bulk_cap_;
  Tables t_{};
  uint64_t* ring_ = nullptr;
  uint8_t* staging_ = nullptr;
  uint8_t* payload_ = nullptr;
  uint64_t* res_ = nullptr;
  uint8_t* bulk_ = nullptr;
  uint64_t* alive_ = nullptr;
  int64_t* tail_ = nullptr;
  hipStream_t stream_ = nullptr;
  uint64_t idle_ticks_ = 0, max_ticks_ = 0;
  int speculate_ = 1;
  uint64_t next_ = 0;
  uint64_t posted_ = 0;
  uint64_t launches_ = 0;
  size_t stage_head_ = 0;
  int64_t payload_head_ = 0;
  int64_t delta_head_ = 0;
  int timeout_s_ = 30;
  bool closed_ = false;
};

}  // namespace

void register_store(py::module_& m) {
  py::class_<Store>(m, "Store", "Device-authoritative governance state store (gfx950 worker or CPU twin)")
      .def(py::init<int, const py::dict&, const py::dict&, int64_t, int64_t, int64_t, int64_t, int64_t>(),
           py::arg("device"), py::arg("ptrs"), py::arg("caps"), py::arg("nslots") = 256,
           py::arg("staging_bytes") = 1 << 22, py::arg("bulk_bytes") = 1 << 22, py::arg("idle_us") = 500,
           py::arg("max_ms") = 2000)
      .def("post", &Store::post, py::arg("op"), py::arg("args"), py::arg("inline") = py::none())
      .def("call", &Store::call, py::arg("op"), py::arg("args"), py::arg("nres") = 4, py::arg("inline") = py::none())
      .def("result", &Store::result, py::arg("seq"), py::arg("nres") = 4)
      .def("drain", &Store::drain)
      .def("stage", &Store::stage)
      .def("bulk", &Store::bulk)
      .def("payload", &Store::payload)
      .def("capture", &Store::capture)
      .def("capture_bytes", &Store::capture_bytes)
      .def("payload_append", &Store::payload_append)
      .def("alloc_delta", &Store::alloc_delta)
      .def("close", &Store::close)
      .def("info", &Store::info)
      .def("set_timeout", &Store::set_timeout)
      .def_property("delta_head", &Store::delta_head, &Store::set_delta_head)
      .def_property("payload_head", &Store::payload_head, &Store::set_payload_head)
      .def_property_readonly("gpu", &Store::gpu);
  py::dict ops;
#define AHV_OP(n) ops[#n] = static_cast<int>(ahv::store::n);
  AHV_OP(OP_NOP) AHV_OP(OP_STOP) AHV_OP(OP_FLUSH) AHV_OP(OP_ACQUIRE) AHV_OP(OP_SESS_CREATE) AHV_OP(OP_SESS_JOIN)
  AHV_OP(OP_SESS_LEAVE) AHV_OP(OP_SESS_ACTIVATE) AHV_OP(OP_SESS_TERMINATE) AHV_OP(OP_SESS_ARCHIVE)
  AHV_OP(OP_SESS_UPDATE_RING) AHV_OP(OP_SESS_SET_MODE) AHV_OP(OP_SESS_READ) AHV_OP(OP_SESS_SET_SIGMA)
  AHV_OP(OP_SESS_CLOSE) AHV_OP(OP_SESS_HANDSHAKE) AHV_OP(OP_DELTA_CAPTURE) AHV_OP(OP_DELTA_MERKLE)
  AHV_OP(OP_DELTA_VERIFY) AHV_OP(OP_DELTA_READ) AHV_OP(OP_VOUCH) AHV_OP(OP_SIGMA_EFF) AHV_OP(OP_EXPOSURE)
  AHV_OP(OP_RELEASE_BOND) AHV_OP(OP_RELEASE_SESSION) AHV_OP(OP_VOUCH_LIST) AHV_OP(OP_EDGE_READ) AHV_OP(OP_SLASH)
  AHV_OP(OP_SAGA_CREATE) AHV_OP(OP_STEP_READ)
  AHV_OP(OP_STEP_ADD) AHV_OP(OP_STEP_TRANSITION) AHV_OP(OP_STEP_SET) AHV_OP(OP_SAGA_TRANSITION)
  AHV_OP(OP_SAGA_READ) AHV_OP(OP_SAGA_PLAN)
#undef AHV_OP
  m.attr("STORE_OPS") = ops;
  py::list cols;
#define AHV_COL(name, type, ext) cols.append(py::make_tuple(#name, #type, #ext));
  AHV_STORE_COLUMNS(AHV_COL)
#undef AHV_COL
  m.attr("STORE_COLUMNS") = cols;
}

}  // namespace host
}  // namespace ahv
