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
#include <pybind11/numpy.h>
#include <pybind11/stl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <unordered_map>
#include <array>
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
void store_pipeline_run(const store::Tables& t, bool gpu, const pybind11::dict& d, uintptr_t stream);

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

// Allocator of the audit payload arena: 64-byte granules, exact-fit free lists
// per granule count (records are a few hundred bytes, so a handful of classes
// see nearly all traffic), a best-fit map for large records, a bump pointer, and
// splitting of larger free blocks when both run dry.  A record's bytes are
// reclaimed together with its delta row (free_deltas), never overwritten while
// the row is live.
class ArenaAlloc {
 public:
  static constexpr int64_t kGran = 64;
  static constexpr int64_t kClasses = 256;

  void reset(int64_t cap) {
    cap_ = cap;
    head_ = 0;
    live_ = 0;
    for (auto& v : cls_) v.clear();
    big_.clear();
  }
  void grow(int64_t cap) { cap_ = cap; }
  static int64_t granules(int64_t bytes) { return bytes <= 0 ? 1 : (bytes + kGran - 1) / kGran; }

  // Offset of a block of `bytes`, or -1 when the arena is full.
  int64_t alloc(int64_t bytes) {
    const int64_t g = granules(bytes);
    int64_t off = -1;
    if (g < kClasses && !cls_[g].empty()) {
      off = cls_[g].back();
      cls_[g].pop_back();
    } else if (head_ + g * kGran <= cap_) {
      off = head_;
      head_ += g * kGran;
    } else {
      for (int64_t k = g + 1; k < kClasses && off < 0; ++k) {
        if (cls_[k].empty()) continue;
        off = cls_[k].back();
        cls_[k].pop_back();
        put(off + g * kGran, k - g);
      }
      if (off < 0) {
        auto it = big_.lower_bound(g);
        if (it == big_.end()) return -1;
        const int64_t k = it->first;
        off = it->second;
        big_.erase(it);
        if (k > g) put(off + g * kGran, k - g);
      }
    }
    live_ += g * kGran;
    return off;
  }
  void free(int64_t off, int64_t bytes) {
    const int64_t g = granules(bytes);
    put(off, g);
    live_ -= g * kGran;
  }
  int64_t live() const { return live_; }
  int64_t head() const { return head_; }

 private:
  void put(int64_t off, int64_t g) {
    if (g < kClasses) cls_[g].push_back(off);
    else big_.emplace(g, off);
  }
  std::vector<int64_t> cls_[kClasses];
  std::multimap<int64_t, int64_t> big_;
  int64_t head_ = 0, cap_ = 0, live_ = 0;
};

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
      std::memset(tail_, 0, 64);  // [0] next sequence, [1..4] worker telemetry
      hip_check(hipDeviceSynchronize(), "store init sync");
      hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "store stream");
      idle_ticks_ = static_cast<uint64_t>(idle_us) * 100;   // s_memrealtime: 100 MHz
      // worker feature bits: 1 = provisional Merkle roots on the idle hash engine,
      // 2 = capture prefix midstates on the command wave,
      const char* sp = std::getenv("AHV_STORE_SPECULATE");
      const char* pf = std::getenv("AHV_STORE_PREFIX");
      // 4 = batched hashing: queued captures of distinct sessions hashed one per lane
      const char* bt = std::getenv("AHV_STORE_BATCH");
      // 8 = compute the capture prefix even when the next command is already waiting (off by
      //     default: it shortens the engine's later captures but the command wave's SHA work
      //     slows the engine's current one — both waves issue on one CU; p50 measured equal or
      //     slightly worse, profiles/r3/prefix_always_ab_r3aj.*)
      const char* pw = std::getenv("AHV_STORE_PREFIX_ALWAYS");
      speculate_ = ((sp == nullptr || std::atoi(sp) != 0) ? 1 : 0) | ((pf == nullptr || std::atoi(pf) != 0) ? 2 : 0) |
                   ((bt == nullptr || std::atoi(bt) != 0) ? 4 : 0) | ((pw != nullptr && std::atoi(pw) != 0) ? 8 : 0);
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
    arena_.reset(t_.cap.B);
    pools_[0].cap = t_.cap.S;
    pools_[1].cap = t_.cap.G;
    pools_[2].cap = t_.cap.T;
    pools_[3].cap = t_.cap.E;
    pools_[4].cap = t_.cap.V;
    d_off_.assign(static_cast<size_t>(t_.cap.D), -1);
    d_len_.assign(static_cast<size_t>(t_.cap.D), 0);
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
    quiesce();
  }

  // Every posted command has completed and no worker wave is resident (its
  // table writes are visible to other kernels); the next post relaunches it.
  void quiesce() {
    if (gpu_ && launches_ > 0) {
      if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) != 0) {
        const uint64_t q = post_raw(OP_STOP, nullptr, 0, nullptr, 0);
        wait(q);
      }
      hip_check(hipStreamSynchronize(stream_), "store worker drain");
    }
  }

  // New table pointers / capacities (table growth).  The caller quiesced the
  // worker and copied the old rows into the new tensors.
  void rebind(const py::dict& ptrs, const py::dict& caps) {
    quiesce();
    auto cap = [&](const char* k) { return caps[k].cast<int64_t>(); };
    const int64_t oldB = t_.cap.B;
    t_.cap = Caps{cap("S"), cap("P"), cap("D"), cap("E"), cap("V"), cap("G"), cap("T"), cap("X"), oldB};
#define AHV_PTR(name, type, ext) t_.name = reinterpret_cast<type*>(ptrs[#name].cast<uintptr_t>());
    AHV_STORE_COLUMNS(AHV_PTR)
#undef AHV_PTR
    d_off_.resize(static_cast<size_t>(t_.cap.D), -1);
    d_len_.resize(static_cast<size_t>(t_.cap.D), 0);
    pools_[0].cap = t_.cap.S;
    pools_[1].cap = t_.cap.G;
    pools_[2].cap = t_.cap.T;
    pools_[3].cap = t_.cap.E;
    pools_[4].cap = t_.cap.V;
  }

  // Double (at least) the payload arena, keeping every record at its offset.
  void grow_payload(int64_t new_bytes) {
    if (new_bytes <= t_.cap.B) return;
    quiesce();
    uint8_t* p = nullptr;
    if (gpu_) {
      hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&p), static_cast<size_t>(new_bytes),
                                      hipDeviceMallocFinegrained),
                "store payload arena (grow)");
      hip_check(hipMemcpy(p, payload_, static_cast<size_t>(arena_.head()), hipMemcpyDeviceToDevice), "arena copy");
      hip_check(hipDeviceSynchronize(), "arena grow sync");
      (void)hipFree(payload_);
    } else {
      p = static_cast<uint8_t*>(std::realloc(payload_, static_cast<size_t>(new_bytes)));
      if (!p) throw std::bad_alloc();
    }
    payload_ = p;
    t_.payload = p;
    t_.cap.B = new_bytes;
    arena_.grow(new_bytes);
  }

  // ------------------------------------------------------------ transport

  uint64_t post_raw(uint32_t op, const uint64_t* args, size_t nargs, const uint8_t* inl, size_t inl_bytes) {
    if (nargs > static_cast<size_t>(kArgs)) throw std::invalid_argument("too many store args");
    if (inl_bytes > static_cast<size_t>(kInlineWords) * 8) throw std::invalid_argument("inline payload too large");
    const uint64_t q = next_++;
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    // the slot's previous occupant must have completed; if an asyncio waiter
    // has not collected its results yet, they are kept aside first
    if (q >= static_cast<uint64_t>(nslots_)) {
      const uint64_t p = q - static_cast<uint64_t>(nslots_);
      const uint64_t* pr = wait(p);
      if (!watched_.empty()) {
        auto it = watched_.find(p);
        if (it != watched_.end()) {
          std::array<uint64_t, kSaveWords> a;
          for (int k = 0; k < kSaveWords; ++k) a[k] = pr[k];
          saved_[p] = a;
          watched_.erase(it);
        }
      }
    }
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

  // Keep the results of `q` even if its slot is recycled before they are read
  // (a posted command whose result is awaited later, after an unbounded number
  // of other sessions' posts — e.g. the saga step's posted EXECUTING transition
  // under thousands of concurrent pipelines).  Consumed by try_result/result.
  void keep(uint64_t q) {
    if (q >= next_) throw std::out_of_range("store: sequence number not posted");
    if (q + static_cast<uint64_t>(nslots_) >= next_) watched_[q] = 1;
  }

  // Drop a kept result that will never be read (its awaiting call was cancelled).
  void discard(uint64_t q) {
    watched_.erase(q);
    saved_.erase(q);
  }

  // Non-blocking form for the asyncio API: the results of `q` if it completed
  // within `spin_ns` (0: just look), else None.  A worker that idled out
  // between the post and now is relaunched.
  py::object try_result(uint64_t q, int nres, int64_t spin_ns) {
    if (nres > kSaveWords - 1) throw std::invalid_argument("try_result: at most 15 result words");
    if (!saved_.empty()) {
      auto it = saved_.find(q);
      if (it != saved_.end()) {
        py::tuple out(nres);
        for (int k = 0; k < nres; ++k) out[k] = py::int_(static_cast<int64_t>(it->second[1 + k]));
        saved_.erase(it);
        return out;
      }
    }
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    volatile uint64_t* r = res_ + idx * kResWords;
    if (q >= next_) throw std::out_of_range("store: sequence number not posted");
    if (r[0] < q + 1 && gpu_) {
      auto t0 = std::chrono::steady_clock::now();
      uint32_t spins = 0;
      while (r[0] < q + 1) {
        if ((++spins & 255u) == 0) {
          if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) == 0) ensure_worker();
          if (std::chrono::steady_clock::now() - t0 >= std::chrono::nanoseconds(spin_ns)) break;
        }
        _mm_pause();
      }
      if (r[0] < q + 1) {
        if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) == 0) ensure_worker();
        watched_[q] = 1;  // keep the results if the slot is recycled before they are collected
        return py::none();
      }
    }
    if (!watched_.empty()) watched_.erase(q);
    if (r[0] >= q + 1 + static_cast<uint64_t>(nslots_)) throw ResultGone();
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
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

  // Returns (-2, ...) when the delta table is full and (-3, ...) when the payload
  // arena is: the Python layer reclaims / grows and retries.  Nothing is
  // recycled while it is live.
  py::tuple capture_rendered(int64_t slot, int64_t turn, int64_t ts_us, const std::string& buf, size_t at) {
    const bool hole = turn > 1;
    const size_t len = hole ? buf.size() - 4 + 66 : buf.size();
    const int64_t didx = take_delta_row();
    if (didx < 0) return py::make_tuple(-2, -1, static_cast<int64_t>(len), -1);
    const int64_t off = arena_.alloc(static_cast<int64_t>(len));
    if (off < 0) {
      dfree_.push_back(static_cast<int32_t>(didx));
      return py::make_tuple(-3, -1, static_cast<int64_t>(len), -1);
    }
    d_off_[static_cast<size_t>(didx)] = off;
    d_len_[static_cast<size_t>(didx)] = static_cast<int64_t>(len);
    uint8_t* dst = payload_ + off;
    if (hole) {
      std::memcpy(dst, buf.data(), at);
      std::memcpy(dst + at + 66, buf.data() + at + 4, buf.size() - at - 4);
    } else {
      std::memcpy(dst, buf.data(), buf.size());
    }
    if (gpu_) _mm_sfence();
    uint64_t a[7] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(didx), static_cast<uint64_t>(turn),
                     static_cast<uint64_t>(ts_us), static_cast<uint64_t>(off), static_cast<uint64_t>(len),
                     hole ? static_cast<uint64_t>(at) : ~0ull};
    const uint64_t q = post_raw(OP_DELTA_CAPTURE, a, 7, nullptr, 0);
    return py::make_tuple(didx, off, static_cast<int64_t>(len), q);
  }

  // Append a complete record to the payload arena (checkpoint restore); returns
  // its offset.  The device re-hashes restored records before they are trusted.
  // Checkpoint restore: a delta row plus its record in the arena (the caller
  // writes the row's columns).  Returns (delta index, offset); -2 / -3 as capture.
  py::tuple restore_delta(const py::bytes& b) {
    std::string_view v = b;
    const int64_t len = static_cast<int64_t>(v.size());
    const int64_t didx = take_delta_row();
    if (didx < 0) return py::make_tuple(-2, -1);
    const int64_t off = arena_.alloc(len);
    if (off < 0) {
      dfree_.push_back(static_cast<int32_t>(didx));
      return py::make_tuple(-3, -1);
    }
    d_off_[static_cast<size_t>(didx)] = off;
    d_len_[static_cast<size_t>(didx)] = len;
    std::memcpy(payload_ + off, v.data(), v.size());
    if (gpu_) _mm_sfence();
    return py::make_tuple(didx, off);
  }

  // Delta rows + arena reservations for a batch of records (the batched store
  // pipeline renders into them): `caps` = int32 bytes per record.  Returns
  // (int32 rows bytes, int64 offsets bytes), or (code, None) with code -2 (delta
  // table full) / -3 (arena full) after releasing what it took.
  py::tuple reserve_deltas(const py::bytes& caps) {
    std::string_view v = caps;
    const size_t n = v.size() / 4;
    const int32_t* c = reinterpret_cast<const int32_t*>(v.data());
    std::string rows(n * 4, '\0'), offs(n * 8, '\0');
    int32_t* r = reinterpret_cast<int32_t*>(rows.data());
    int64_t* o = reinterpret_cast<int64_t*>(offs.data());
    for (size_t i = 0; i < n; ++i) {
      const int64_t d = take_delta_row();
      const int64_t off = d < 0 ? -1 : arena_.alloc(c[i]);
      if (d < 0 || off < 0) {
        if (d >= 0) dfree_.push_back(static_cast<int32_t>(d));
        for (size_t k = 0; k < i; ++k) {
          arena_.free(o[k], c[k]);
          d_off_[static_cast<size_t>(r[k])] = -1;
          d_len_[static_cast<size_t>(r[k])] = 0;
          dfree_.push_back(r[k]);
        }
        return py::make_tuple(d < 0 ? -2 : -3, py::none());
      }
      r[i] = static_cast<int32_t>(d);
      o[i] = off;
      d_off_[static_cast<size_t>(d)] = off;
      d_len_[static_cast<size_t>(d)] = c[i];  // the reservation is what a free returns
    }
    return py::make_tuple(py::bytes(rows), py::bytes(offs));
  }

  // The batched store pipeline (csrc/hip/store_pipeline.hip) over this store's
  // tables on `stream`; the caller released the worker's writes (OP_FLUSH)
  // before and has it acquire the new rows (OP_ACQUIRE) after the stream drains.
  void run_pipeline(const py::dict& d, uintptr_t stream) { store_pipeline_run(t_, gpu_, d, stream); }

  // Reclaim delta rows (and their arena records) no API object refers to any
  // more: OP_FREE_ROWS marks them free on the device after the hash engine has
  // drained, then the rows and bytes return to the host free lists.
  void free_deltas(const std::vector<int32_t>& rows) {
    if (rows.empty()) return;
    for (int32_t d : rows)
      if (d < 0 || d >= t_.cap.D || d_off_[static_cast<size_t>(d)] < 0)
        throw std::invalid_argument("free_deltas: row " + std::to_string(d) + " is not allocated");
    free_rows_cmd(RK_D, rows);
    for (int32_t d : rows) {
      arena_.free(d_off_[static_cast<size_t>(d)], d_len_[static_cast<size_t>(d)]);
      d_off_[static_cast<size_t>(d)] = -1;
      d_len_[static_cast<size_t>(d)] = 0;
      dfree_.push_back(d);
    }
  }

  // OP_FREE_ROWS for any table; waits for completion.
  void free_rows_cmd(uint64_t kind, const std::vector<int32_t>& rows) {
    const size_t per = static_cast<size_t>(staging_cap_ / 8);  // one staged list per command
    for (size_t i = 0; i < rows.size(); i += per) {
      const size_t n = std::min(per, rows.size() - i);
      uint64_t a[3] = {kind, static_cast<uint64_t>(n), 0};
      const uint8_t* raw = reinterpret_cast<const uint8_t*>(rows.data() + i);
      uint64_t q;
      if (n <= static_cast<size_t>(2 * kInlineWords)) {
        q = post_raw(OP_FREE_ROWS, a, 3, raw, 4 * n);
      } else {
        a[2] = static_cast<uint64_t>(stage_raw(raw, 4 * n));
        q = post_raw(OP_FREE_ROWS, a, 3, nullptr, 0);
      }
      const uint64_t* r = wait(q);
      if (r[1] != ST_OK) throw std::runtime_error("OP_FREE_ROWS failed with status " + std::to_string(r[1]));
    }
  }

  // ------------------------------------------------------------ row allocator
  //
  // Free lists of the session / saga / step / vouch-edge / liability-session
  // tables (RowKind S G T E V; delta rows have their own, with their arena
  // records).  A row is *live* from alloc_row until its last API view releases
  // it (release_row, cheap enough for a finaliser); released rows queue in
  // `pend` and are reclaimed in small batches — OP_FREE_ROWS marks them free on
  // the device, then they return to the free list.  The host does not wait for
  // that command: every later command that could reuse a row executes after it
  // (the worker runs commands in order, and batched kernels drain the worker
  // first), so the rows are handed out again at once; the command's status is
  // checked when the next reclaim of any table runs.  Delta rows are different:
  // their arena bytes are rewritten by the host at the next capture's post, so
  // they wait for the FREE_ROWS (which drains the hash engine) to complete.
  struct RowPool {
    int64_t cap = 0, hw = 0;
    std::vector<int32_t> free, pend;
  };

  static size_t pool_index(uint64_t kind) {
    switch (kind) {
      case RK_S: return 0;
      case RK_G: return 1;
      case RK_T: return 2;
      case RK_E: return 3;
      case RK_V: return 4;
      default: throw std::invalid_argument("row kind has no row pool: " + std::to_string(kind));
    }
  }
  RowPool& pool(uint64_t kind) { return pools_[pool_index(kind)]; }

  void set_row_cap(uint64_t kind, int64_t cap) { pool(kind).cap = cap; }

  // Queued rows that trigger a reclaim: 256, or an eighth of a small table.
  static size_t reclaim_at(const RowPool& p) {
    return static_cast<size_t>(std::max<int64_t>(8, std::min<int64_t>(256, p.cap >> 3)));
  }

  // A free row of `kind`, or -1 when the table is full (the caller grows it).
  int64_t alloc_row(uint64_t kind) {
    RowPool& p = pool(kind);
    if (p.pend.size() >= reclaim_at(p)) reclaim_pool(kind);
    if (p.free.empty() && p.hw >= p.cap && !p.pend.empty()) reclaim_pool(kind);
    if (!p.free.empty()) {
      const int32_t r = p.free.back();
      p.free.pop_back();
      return r;
    }
    if (p.hw < p.cap) return p.hw++;
    return -1;
  }

  // `n` free rows of `kind` (int32), or None when the table cannot hold them (nothing taken).
  py::object alloc_rows(uint64_t kind, int64_t n) {
    RowPool& p = pool(kind);
    if (!p.pend.empty()) reclaim_pool(kind);
    if (static_cast<int64_t>(p.free.size()) + (p.cap - p.hw) < n) return py::none();
    py::array_t<int32_t> out(n);
    int32_t* o = out.mutable_data();
    int64_t k = 0;
    while (k < n && !p.free.empty()) {
      o[k++] = p.free.back();
      p.free.pop_back();
    }
    while (k < n) o[k++] = static_cast<int32_t>(p.hw++);
    return std::move(out);
  }

  void release_row(uint64_t kind, int64_t row) {
    if (kind == RK_D) {
      dpend_.push_back(static_cast<int32_t>(row));
      return;
    }
    pool(kind).pend.push_back(static_cast<int32_t>(row));
  }

  // A row that was allocated but never written on the device (a refused vouch):
  // straight back to the free list.
  void return_row(uint64_t kind, int64_t row) { pool(kind).free.push_back(static_cast<int32_t>(row)); }

  void release_rows(uint64_t kind, py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
    std::vector<int32_t>& v = kind == RK_D ? dpend_ : pool(kind).pend;
    v.insert(v.end(), a.data(), a.data() + a.size());
  }

  // Return the queued rows of `kind` to its free list; returns their count.
  int64_t reclaim_pool(uint64_t kind) {
    if (kind == RK_D) {
      if (dpend_.empty()) return 0;
      std::vector<int32_t> rows;
      rows.swap(dpend_);
      free_deltas(rows);
      return static_cast<int64_t>(rows.size());
    }
    RowPool& p = pool(kind);
    if (p.pend.empty()) return 0;
    check_frees();
    std::vector<int32_t> rows;
    rows.swap(p.pend);
    post_frees(kind, rows);
    p.free.insert(p.free.end(), rows.begin(), rows.end());
    return static_cast<int64_t>(rows.size());
  }

  int64_t npend(uint64_t kind) const {
    return static_cast<int64_t>(kind == RK_D ? dpend_.size() : pools_[pool_index(kind)].pend.size());
  }
  int64_t live_rows(uint64_t kind) const {
    if (kind == RK_D) return delta_live() - static_cast<int64_t>(dpend_.size());
    const RowPool& p = pools_[pool_index(kind)];
    return p.hw - static_cast<int64_t>(p.free.size() + p.pend.size());
  }

  // OP_FREE_ROWS without waiting; statuses are checked by check_frees.
  void post_frees(uint64_t kind, const std::vector<int32_t>& rows) {
    const size_t per = static_cast<size_t>(staging_cap_ / 8);
    for (size_t i = 0; i < rows.size(); i += per) {
      const size_t n = std::min(per, rows.size() - i);
      uint64_t a[3] = {kind, static_cast<uint64_t>(n), 0};
      const uint8_t* raw = reinterpret_cast<const uint8_t*>(rows.data() + i);
      uint64_t q;
      if (n <= static_cast<size_t>(2 * kInlineWords)) {
        q = post_raw(OP_FREE_ROWS, a, 3, raw, 4 * n);
      } else {
        a[2] = static_cast<uint64_t>(stage_raw(raw, 4 * n));
        q = post_raw(OP_FREE_ROWS, a, 3, nullptr, 0);
      }
      keep(q);
      frees_.push_back(q);
    }
  }

  // Statuses of the FREE_ROWS posted so far whose results are in (`block`: all).
  void check_frees(bool block = false) {
    size_t k = 0;
    for (; k < frees_.size(); ++k) {
      const uint64_t q = frees_[k];
      uint64_t st;
      auto it = saved_.find(q);
      if (it != saved_.end()) {
        st = it->second[1];
        saved_.erase(it);
      } else {
        volatile uint64_t* r = res_ + (q % static_cast<uint64_t>(nslots_)) * kResWords;
        if (r[0] < q + 1 && !block) break;
        st = wait(q)[1];
        watched_.erase(q);
      }
      if (st != ST_OK) {
        frees_.erase(frees_.begin(), frees_.begin() + static_cast<std::ptrdiff_t>(k + 1));
        throw std::runtime_error("OP_FREE_ROWS failed with status " + std::to_string(st));
      }
    }
    frees_.erase(frees_.begin(), frees_.begin() + static_cast<std::ptrdiff_t>(k));
  }

  int64_t take_delta_row() {
    if (!dfree_.empty()) {
      const int32_t d = dfree_.back();
      dfree_.pop_back();
      return d;
    }
    if (dhw_ < t_.cap.D) return dhw_++;
    return -1;
  }

  py::dict info() const {
    py::dict d;
    d["gpu"] = gpu_;
    d["device"] = device_;
    d["posted"] = posted_;
    d["launches"] = launches_;
    d["nslots"] = nslots_;
    d["payload_live"] = arena_.live();
    d["payload_head"] = arena_.head();
    d["payload_cap"] = t_.cap.B;
    d["delta_rows"] = dhw_ - static_cast<int64_t>(dfree_.size());
    d["delta_hw"] = dhw_;
    d["delta_cap"] = t_.cap.D;
    d["kept"] = static_cast<int64_t>(watched_.size() + saved_.size());  // posted results awaiting their reader
    if (gpu_) {  // worker utilisation telemetry (store_worker.hip; s_memrealtime ticks are 10 ns)
      d["worker_busy_us"] = static_cast<double>(__atomic_load_n(tail_ + 1, __ATOMIC_RELAXED)) / 100.0;
      d["worker_commands"] = __atomic_load_n(tail_ + 2, __ATOMIC_RELAXED);
      d["engine_busy_us"] = static_cast<double>(__atomic_load_n(tail_ + 3, __ATOMIC_RELAXED)) / 100.0;
      d["engine_jobs"] = __atomic_load_n(tail_ + 4, __ATOMIC_RELAXED);
    }
    return d;
  }

  int64_t delta_live() const { return dhw_ - static_cast<int64_t>(dfree_.size()); }
  int64_t payload_cap() const { return t_.cap.B; }
  int64_t bulk_cap() const { return bulk_cap_; }
  uintptr_t payload_ptr() const { return reinterpret_cast<uintptr_t>(payload_); }
  int64_t staging_cap() const { return staging_cap_; }
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
  ArenaAlloc arena_;
  static constexpr int kSaveWords = 16;
  std::unordered_map<uint64_t, int> watched_;                             // seqs with a pending async waiter
  std::unordered_map<uint64_t, std::array<uint64_t, kSaveWords>> saved_;  // their results, once recycled
  std::vector<int64_t> d_off_, d_len_;  // arena record of each delta row (-1: row free)
  std::vector<int32_t> dfree_;          // reclaimed delta rows
  std::vector<int32_t> dpend_;          // delta rows released by their views, not reclaimed yet
  RowPool pools_[5];                    // S G T E V row allocators
  std::vector<uint64_t> frees_;         // FREE_ROWS posted without waiting, status unchecked
  int64_t dhw_ = 0;                      // delta rows ever handed out (high-water mark)
  int timeout_s_ = 30;
  bool closed_ = false;
};

}  // namespace

void register_store(py::module_& m) {
  py::class_<Store>(m, "Store", "Device-authoritative governance state store (gfx950 worker or CPU twin)")
      .def(py::init<int, const py::dict&, const py::dict&, int64_t, int64_t, int64_t, int64_t, int64_t>(),
           py::arg("device"), py::arg("ptrs"), py::arg("caps"), py::arg("nslots") = 4096,
           py::arg("staging_bytes") = 1 << 22, py::arg("bulk_bytes") = 1 << 24, py::arg("idle_us") = 500,
           py::arg("max_ms") = 2000)
      .def("post", &Store::post, py::arg("op"), py::arg("args"), py::arg("inline") = py::none())
      .def("keep", &Store::keep, py::arg("seq"))
      .def("discard", &Store::discard, py::arg("seq"))
      .def("call", &Store::call, py::arg("op"), py::arg("args"), py::arg("nres") = 4, py::arg("inline") = py::none())
      .def("result", &Store::result, py::arg("seq"), py::arg("nres") = 4)
      .def("try_result", &Store::try_result, py::arg("seq"), py::arg("nres") = 4, py::arg("spin_ns") = 0)
      .def("drain", &Store::drain)
      .def("stage", &Store::stage)
      .def("bulk", &Store::bulk)
      .def("payload", &Store::payload)
      .def("capture", &Store::capture)
      .def("capture_bytes", &Store::capture_bytes)
      .def("restore_delta", &Store::restore_delta)
      .def("free_deltas", &Store::free_deltas)
      .def("free_deltas_arr",
           [](Store& st, py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
             st.free_deltas(std::vector<int32_t>(a.data(), a.data() + a.size()));
           })
      .def("free_rows_arr",
           [](Store& st, uint64_t kind, py::array_t<int32_t, py::array::c_style | py::array::forcecast> a) {
             st.free_rows_cmd(kind, std::vector<int32_t>(a.data(), a.data() + a.size()));
           })
      .def("reserve_deltas", &Store::reserve_deltas)
      .def("alloc_row", &Store::alloc_row)
      .def("alloc_rows", &Store::alloc_rows)
      .def("release_row", &Store::release_row)
      .def("release_rows", &Store::release_rows)
      .def("return_row", &Store::return_row)
      .def("reclaim_pool", &Store::reclaim_pool)
      .def("check_frees", &Store::check_frees, py::arg("block") = false)
      .def("npend", &Store::npend)
      .def("live_rows", &Store::live_rows)
      .def("set_row_cap", &Store::set_row_cap)
      .def("run_pipeline", &Store::run_pipeline)
      .def("free_rows", &Store::free_rows_cmd)
      .def("quiesce", &Store::quiesce)
      .def("rebind", &Store::rebind)
      .def("grow_payload", &Store::grow_payload)
      .def("close", &Store::close)
      .def("info", &Store::info)
      .def("set_timeout", &Store::set_timeout)
      .def_property_readonly("delta_live", &Store::delta_live)
      .def_property_readonly("payload_cap", &Store::payload_cap)
      .def_property_readonly("bulk_cap", &Store::bulk_cap)
      .def_property_readonly("payload_ptr", &Store::payload_ptr)
      .def_property_readonly("staging_cap", &Store::staging_cap)
      .def_property_readonly("gpu", &Store::gpu);
  py::dict ops;
#define AHV_OP(n) ops[#n] = static_cast<int>(ahv::store::n);
  AHV_OP(OP_NOP) AHV_OP(OP_STOP) AHV_OP(OP_FLUSH) AHV_OP(OP_ACQUIRE) AHV_OP(OP_FREE_ROWS) AHV_OP(OP_SESS_READ_MANY) AHV_OP(OP_V_RETIRE) AHV_OP(OP_SESS_CREATE) AHV_OP(OP_SESS_JOIN)
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
  m.attr("STORE_HDR_WORDS") = static_cast<int>(ahv::store::kHdrWords);
  py::list cols;
#define AHV_COL(name, type, ext) cols.append(py::make_tuple(#name, #type, #ext));
  AHV_STORE_COLUMNS(AHV_COL)
#undef AHV_COL
  m.attr("STORE_COLUMNS") = cols;
}

}  // namespace host
}  // namespace ahv
