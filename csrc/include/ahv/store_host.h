// Host runtime of the device state store (ahv/store.h), free of Python: the
// transport between the API layer and the store tables, and the host-side
// allocators.  csrc/host/py_store.cpp binds it to Python; the host self test
// (csrc/tests/host_selftest.cpp) drives it directly under ASan/UBSan.
//
//   gfx950:  command ring + staging area + audit payload arena in fine-grained
//            device memory (host writes them through the PCIe BAR), result slots
//            and bulk outputs in pinned host memory, and the resident worker
//            (csrc/hip/store_worker.hip) that executes commands.  The worker idles
//            out after a short quiet period and is relaunched on demand, so it
//            never holds its hardware queue for long.
//   cpu:     the same `store_exec` body runs inline on host-memory tables (the
//            CPU twin used by the CPU test suite and the reference oracle).
//
// The tables themselves are owned by the caller (PyTorch tensors in
// agent_hypervisor_amd/models/store.py) and passed in by address.
#pragma once

#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "ahv/store.h"

extern "C" int ahv_store_launch_worker(const ahv::store::Tables* t, const uint64_t* ring, int64_t nslots,
                                       uint64_t* res, uint8_t* bulk, uint64_t* alive, int64_t* tail,
                                       uint64_t idle_ticks, uint64_t max_ticks, int speculate, uint64_t* trace,
                                       int64_t trace_cap, hipStream_t stream);

namespace ahv {
namespace host {

using store::Caps;
using store::Tables;

// The result slot of a sequence number was recycled by a later command.
struct ResultGone : std::exception {
  const char* what() const noexcept override { return "store result slot recycled"; }
};

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Column addresses by name (the X-macro's names).
using ColumnPtrs = std::unordered_map<std::string, uintptr_t>;

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

// A capture's placement: delta row, arena offset, record length, command sequence
// (code -2: delta table full, -3: arena full — nothing taken).
struct Placed {
  int64_t didx, off, len, seq;
};

class StoreCore {
 public:
  static constexpr int kSaveWords = 16;

  StoreCore(int device, const ColumnPtrs& ptrs, const Caps& caps, int64_t nslots, int64_t staging_bytes,
            int64_t bulk_bytes, int64_t idle_us, int64_t max_ms)
      : gpu_(device >= 0), device_(device), nslots_(nslots), staging_cap_(staging_bytes), bulk_cap_(bulk_bytes) {
    t_.cap = caps;
    bind(ptrs);
    const size_t ring_bytes = static_cast<size_t>(nslots_) * store::kSlotWords * 8;
    const size_t res_bytes = static_cast<size_t>(nslots_) * store::kResWords * 8;
    if (gpu_) {
      hip_check(hipSetDevice(device_), "hipSetDevice");
      // The command ring: fine-grained device memory by default, written through
      // the BAR with 32-byte stores, so the worker's slot reads stay in HBM.
      // AHV_STORE_RING=host puts it in pinned host memory (cached host stores,
      // but every worker read crosses PCIe: measured 2.47 us vs 1.77 us per NOP
      // of worker throughput, profiles/r4/worker_probe_r4h_*.json).
      const char* rm = std::getenv("AHV_STORE_RING");
      ring_host_ = rm != nullptr && std::string(rm) == "host";
      if (ring_host_) {
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&ring_), ring_bytes, hipHostMallocCoherent), "store ring");
      } else {
        hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&ring_), ring_bytes, hipDeviceMallocFinegrained),
                  "store ring");
      }
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
      if (ring_host_) std::memset(ring_, 0, ring_bytes);
      else hip_check(hipMemset(ring_, 0, ring_bytes), "memset ring");
      std::memset(tail_, 0, 64);  // [0] next sequence, [1..4] worker telemetry
      hip_check(hipDeviceSynchronize(), "store init sync");
      hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "store stream");
      idle_ticks_ = static_cast<uint64_t>(idle_us) * 100;  // s_memrealtime: 100 MHz
      // worker feature bits: 1 = provisional Merkle roots on the idle hash engine,
      // 2 = capture prefix midstates on the prefix wave (wave 2),
      const char* sp = std::getenv("AHV_STORE_SPECULATE");
      const char* pf = std::getenv("AHV_STORE_PREFIX");
      // 4 = batched hashing: queued captures of distinct sessions hashed one per lane
      const char* bt = std::getenv("AHV_STORE_BATCH");
      // 16 = FREE_ROWS waits only for the queued captures of the rows it frees (S, D) or
      //      not at all (G, T, E, V), instead of draining the hash engine
      const char* nf = std::getenv("AHV_STORE_NARROW_FREE");
      // 32 = results published with a wait for the worker's stores, not a system release
      //      (wholesale commands keep the full release; see publish_fence)
      const char* lp = std::getenv("AHV_STORE_LIGHT_PUBLISH");
      // 64 = prefetch the next command slot while the current command executes
      const char* pf2 = std::getenv("AHV_STORE_SLOT_PREFETCH");
      // 128 = helper waves hash a capture whose parent the host predicted (hole prefilled)
      //       as a whole record, off the chain; the engine checks the parent and takes it
      const char* sc = std::getenv("AHV_STORE_SPEC_CHAIN");
      // 256 = helper waves hash captures straight from the command ring, ahead of the
      //       command wave (turn-1 records and predicted-parent links).  Off by default
      //       (AHV_STORE_LOOKAHEAD=1 on): measured slower — the waves of the one worker CU
      //       hash at 3.2-3.4 µs per block side by side against 2.4 µs for the engine alone
      //       (per-call p50 76.4 vs 69.4 µs, profiles/r6/lookahead_ab_r6v.txt)
      const char* la = std::getenv("AHV_STORE_LOOKAHEAD");
      // 512 = the next slot's prefetch is issued after the current command's result is
      //       published (not before its execution: the publication's wait covers it)
      const char* lp2 = std::getenv("AHV_STORE_LATE_PREFETCH");
      speculate_ = ((la != nullptr && std::atoi(la) != 0) ? 256 : 0) |
                   ((lp2 != nullptr && std::atoi(lp2) != 0) ? 512 : 0) |
                   ((sc == nullptr || std::atoi(sc) != 0) ? 128 : 0) | ((sp == nullptr || std::atoi(sp) != 0) ? 1 : 0) | ((pf == nullptr || std::atoi(pf) != 0) ? 2 : 0) |
                   ((bt == nullptr || std::atoi(bt) != 0) ? 4 : 0) |
                   ((nf == nullptr || std::atoi(nf) != 0) ? 16 : 0) |
                   ((lp == nullptr || std::atoi(lp) != 0) ? 32 : 0) |
                   ((pf2 == nullptr || std::atoi(pf2) != 0) ? 64 : 0);
      max_ticks_ = static_cast<uint64_t>(max_ms) * 100000;
      // command / hash-engine timeline (AHV_STORE_TRACE=<entries>, off by default)
      const char* tr = std::getenv("AHV_STORE_TRACE");
      if (tr != nullptr && std::atoll(tr) > 0) {
        trace_cap_ = std::atoll(tr);
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&trace_), static_cast<size_t>(trace_cap_) * 128,
                                hipHostMallocCoherent),
                  "store trace");
        std::memset(trace_, 0, static_cast<size_t>(trace_cap_) * 128);
        post_ns_.assign(static_cast<size_t>(trace_cap_), 0);
      }
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
    set_pool_caps();
    d_off_.assign(static_cast<size_t>(t_.cap.D), -1);
    d_len_.assign(static_cast<size_t>(t_.cap.D), 0);
    watch_.assign(static_cast<size_t>(nslots_), 0);
  }

  StoreCore(const StoreCore&) = delete;
  StoreCore& operator=(const StoreCore&) = delete;

  virtual ~StoreCore() {
    try {
      close();
    } catch (...) {
    }
    if (gpu_) {
      if (ring_host_) (void)hipHostFree(ring_);
      else (void)hipFree(ring_);
      (void)hipFree(staging_);
      (void)hipFree(payload_);
      (void)hipHostFree(res_);
      (void)hipHostFree(bulk_);
      (void)hipHostFree(alive_);
      (void)hipHostFree(tail_);
      if (trace_) (void)hipHostFree(trace_);
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
        const uint64_t q = post_raw(store::OP_STOP, nullptr, 0, nullptr, 0);
        wait(q);
      }
      hip_check(hipStreamSynchronize(stream_), "store worker drain");
    }
  }

  // New table pointers / capacities (table growth).  The caller quiesced the
  // worker and copied the old rows into the new tensors.
  void rebind(const ColumnPtrs& ptrs, const Caps& caps) {
    quiesce();
    const int64_t oldB = t_.cap.B;
    t_.cap = caps;
    t_.cap.B = oldB;
    bind(ptrs);
    d_off_.resize(static_cast<size_t>(t_.cap.D), -1);
    d_len_.resize(static_cast<size_t>(t_.cap.D), 0);
    set_pool_caps();
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
      // the whole old arena: besides the allocator's records it may hold regions a
      // batched kernel wrote at caller-chosen offsets (GovernanceEngine's ring)
      hip_check(hipMemcpy(p, payload_, static_cast<size_t>(t_.cap.B), hipMemcpyDeviceToDevice), "arena copy");
      hip_check(hipDeviceSynchronize(), "arena grow sync");
      (void)hipFree(payload_);
    } else {
      p = static_cast<uint8_t*>(std::realloc(payload_, static_cast<size_t>(new_bytes)));
      if (!p) throw std::bad_alloc();
      std::memset(p + t_.cap.B, 0, static_cast<size_t>(new_bytes - t_.cap.B));
    }
    payload_ = p;
    t_.payload = p;
    t_.cap.B = new_bytes;
    arena_.grow(new_bytes);
  }

  // ------------------------------------------------------------ transport

  uint64_t post_raw(uint32_t op, const uint64_t* args, size_t nargs, const uint8_t* inl, size_t inl_bytes) {
    using namespace store;
    if (nargs > static_cast<size_t>(kArgs)) throw std::invalid_argument("too many store args");
    if (inl_bytes > static_cast<size_t>(kInlineWords) * 8) throw std::invalid_argument("inline payload too large");
    const uint64_t q = next_++;
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    // the slot's previous occupant must have completed; if an asyncio waiter
    // has not collected its results yet, they are kept aside first
    if (q >= static_cast<uint64_t>(nslots_)) {
      const uint64_t p = q - static_cast<uint64_t>(nslots_);
      const uint64_t* pr;
      if (gpu_ && *reinterpret_cast<volatile uint64_t*>(res_ + (p % static_cast<uint64_t>(nslots_)) * store::kResWords) <
                      p + 1) {
        // the ring is full: the worker is a whole ring behind (telemetry: host back-pressure)
        const auto t0 = std::chrono::steady_clock::now();
        pr = wait(p);
        ring_wait_ns_ += static_cast<uint64_t>(
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
        ++ring_waits_;
      } else {
        pr = wait(p);
      }
      if (nwatch_ && watched(p)) {
        std::array<uint64_t, kSaveWords> a;
        for (int k = 0; k < kSaveWords; ++k) a[k] = pr[k];
        saved_[p] = a;
        unwatch(p);
      }
    }
    uint64_t w[kSlotWords];
    // words in use (header, arguments, inline payload): only these cross the BAR;
    // the worker reads the count from w[1]'s high half and treats the rest as zero
    // (zero words add nothing to the checksum: slot_mix(0, k) = 0)
    const uint32_t nw = inl_bytes ? 16u + static_cast<uint32_t>((inl_bytes + 7) / 8) : 3u + static_cast<uint32_t>(nargs);
    const uint32_t nz = gpu_ ? std::min<uint32_t>((nw + 3u) & ~3u, kSlotWords) : kSlotWords;  // the BAR chunks' words
    std::memset(w, 0, 8 * static_cast<size_t>(nz));
    w[1] = op | (static_cast<uint64_t>(nw) << 32);
    for (size_t k = 0; k < nargs; ++k) w[3 + k] = args[k];
    if (inl_bytes) std::memcpy(w + 16, inl, inl_bytes);
    uint64_t x = slot_mix(w[1], 1);
    for (uint32_t k = 3; k < nw; ++k) x ^= slot_mix(w[k], static_cast<uint64_t>(k));
    w[2] = x;
    ++posted_;
    if (trace_cap_ > 0)
      post_ns_[static_cast<size_t>(q % static_cast<uint64_t>(trace_cap_))] = static_cast<uint64_t>(
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
              .count());
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
    uint64_t* slot = ring_ + idx * kSlotWords;
    if (ring_host_) {
      // cached stores; x86 keeps them in order, and the worker rejects a torn read
      // through the checksum, so the sequence word goes last
      std::memcpy(slot + 1, w + 1, 8 * (nw - 1));
      __atomic_store_n(slot, q + 1, __ATOMIC_RELEASE);
    } else if (__builtin_cpu_supports("avx2")) {
      write_slot_bar(slot, w, q + 1, nw);
    } else {
      volatile uint64_t* v = slot;
      for (uint32_t k = 1; k < nw; ++k) v[k] = w[k];
      _mm_sfence();
      v[0] = q + 1;
      _mm_sfence();
    }
    ensure_worker();
    return q;
  }

  // A slot in device memory through the BAR: 32-byte stores of the `nw` words in
  // use (a typical command is 1–4 PCIe writes, not the 16 of the whole 512-byte
  // slot): the argument / payload chunks, then the first chunk with the sequence
  // word, then one fence.  Write-combined stores may reach the device in any
  // order; a worker that sees the sequence word before the rest rejects the read
  // through the checksum and polls again (store_worker.hip).
  __attribute__((target("avx2"))) static void write_slot_bar(uint64_t* slot, const uint64_t* w, uint64_t seq,
                                                             uint32_t nw) {
    for (uint32_t k = 4; k < nw; k += 4)
      _mm256_storeu_si256(reinterpret_cast<__m256i*>(slot + k),
                          _mm256_loadu_si256(reinterpret_cast<const __m256i*>(w + k)));
    const uint64_t first[4] = {seq, w[1], w[2], w[3]};
    _mm256_storeu_si256(reinterpret_cast<__m256i*>(slot), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(first)));
    _mm_sfence();
  }

  void ensure_worker() {
    if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) != 0) return;
    __atomic_store_n(alive_, 1ull, __ATOMIC_RELEASE);
    const int rc = ahv_store_launch_worker(&t_, ring_, nslots_, res_, bulk_, alive_, tail_, idle_ticks_, max_ticks_,
                                           speculate_, trace_, trace_cap_, stream_);
    if (rc != 0) {
      __atomic_store_n(alive_, 0ull, __ATOMIC_RELEASE);
      throw std::runtime_error(std::string("store worker launch failed: ") +
                               hipGetErrorString(static_cast<hipError_t>(rc)));
    }
    ++launches_;
  }

  const uint64_t* wait(uint64_t q) {
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    volatile uint64_t* r = res_ + idx * store::kResWords;
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

  // Keep the results of `q` even if its slot is recycled before they are read
  // (a posted command whose result is awaited later, after an unbounded number
  // of other sessions' posts — e.g. the saga step's posted EXECUTING transition
  // under thousands of concurrent pipelines).  Consumed by try_result/result.
  void keep(uint64_t q) {
    if (q >= next_) throw std::out_of_range("store: sequence number not posted");
    if (q + static_cast<uint64_t>(nslots_) >= next_) watch(q);
  }

  // Drop a kept result that will never be read (its awaiting call was cancelled).
  void discard(uint64_t q) {
    unwatch(q);
    saved_.erase(q);
  }

  // The result words of `q` in place when it has completed and its slot still holds
  // it (nullptr otherwise: not done yet, recycled into `saved_`, or posted later) —
  // the expectation check's fast path, no copy of the result words.
  const uint64_t* peek_done(uint64_t q) {
    if (q >= next_) return nullptr;
    volatile uint64_t* r = res_ + (q % static_cast<uint64_t>(nslots_)) * store::kResWords;
    const uint64_t v = r[0];
    if (v < q + 1 || v >= q + 1 + static_cast<uint64_t>(nslots_)) return nullptr;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (nwatch_) unwatch(q);
    return const_cast<const uint64_t*>(r);
  }

  // Non-blocking form for asyncio callers: copies the first kSaveWords result
  // words of `q` into `out` and returns true if it completed within `spin_ns`
  // (0: just look).  A worker that idled out between the post and now is relaunched.
  bool try_result_raw(uint64_t q, int64_t spin_ns, uint64_t out[kSaveWords]) {
    if (!saved_.empty()) {
      auto it = saved_.find(q);
      if (it != saved_.end()) {
        for (int k = 0; k < kSaveWords; ++k) out[k] = it->second[k];
        saved_.erase(it);
        return true;
      }
    }
    const uint64_t idx = q % static_cast<uint64_t>(nslots_);
    volatile uint64_t* r = res_ + idx * store::kResWords;
    if (q >= next_) throw std::out_of_range("store: sequence number not posted");
    if (r[0] < q + 1 && gpu_ && spin_ns <= 0) {
      // just look: no spin (a 256-pause spin before the first clock check cost ≈3 µs
      // on every speculation check and asyncio poll of a command still in flight)
      if (__atomic_load_n(alive_, __ATOMIC_ACQUIRE) == 0) ensure_worker();
      watch(q);
      return false;
    }
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
        watch(q);  // keep the results if the slot is recycled before they are collected
        return false;
      }
    }
    if (nwatch_) unwatch(q);
    if (r[0] >= q + 1 + static_cast<uint64_t>(nslots_)) throw ResultGone();
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    for (int k = 0; k < kSaveWords; ++k) out[k] = r[k];
    return true;
  }

  // Everything posted so far has completed: on the device a NOP is executed only
  // after the hash engine's queue has drained, and results complete in order
  // otherwise.
  void drain() {
    if (next_ == 0) return;
    if (!gpu_) return;
    wait(post_raw(store::OP_NOP, nullptr, 0, nullptr, 0));
  }

  // Copy bytes into the staging area; returns their offset.  Wrapping first
  // drains the queue, so no pending command still reads the overwritten bytes.
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

  const uint8_t* bulk_ptr(int64_t off, int64_t n) const {
    if (off < 0 || n < 0 || off + n > bulk_cap_) throw std::out_of_range("bulk range");
    return bulk_ + off;
  }

  void payload_read(int64_t off, int64_t n, void* dst) const {
    if (off < 0 || n < 0 || off + n > t_.cap.B) throw std::out_of_range("payload range");
    if (gpu_) {
      hip_check(hipMemcpy(dst, payload_ + off, static_cast<size_t>(n), hipMemcpyDeviceToHost), "payload read");
    } else {
      std::memcpy(dst, payload_ + off, static_cast<size_t>(n));
    }
  }

  // Bulk copy into the payload arena (checkpoint restore of whole arena regions);
  // the caller drained the worker, and records are re-verified (K10) afterwards.
  void write_payload_raw(int64_t off, const void* src, size_t n) {
    if (off < 0 || off + static_cast<int64_t>(n) > t_.cap.B) throw std::out_of_range("payload range");
    if (gpu_) {
      hip_check(hipMemcpy(payload_ + off, src, n, hipMemcpyHostToDevice), "payload write");
    } else {
      std::memcpy(payload_ + off, src, n);
    }
  }

  // Records at arena offsets `offs` with lengths `lens`, concatenated in `blob`
  // (checkpoint restore into freshly reserved rows).
  void write_records_raw(const int64_t* o, const int64_t* l, int64_t n, const uint8_t* blob, size_t blob_n) {
    int64_t pos = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (o[i] < 0 || l[i] < 0 || o[i] + l[i] > t_.cap.B || pos + l[i] > static_cast<int64_t>(blob_n))
        throw std::out_of_range("write_records: record out of range");
      pos += l[i];
    }
    pos = 0;
    for (int64_t i = 0; i < n; ++i) {
      std::memcpy(payload_ + o[i], blob + pos, static_cast<size_t>(l[i]));  // host-visible arena (BAR on gfx950)
      pos += l[i];
    }
    if (gpu_) _mm_sfence();
  }

  // The records at arena offsets `o` / lengths `l`, concatenated into `dst`
  // (checkpoint save).  On the GPU the used span is copied to the host once.
  void gather_records_raw(const int64_t* o, const int64_t* l, int64_t n, uint8_t* dst) const {
    int64_t lo = INT64_MAX, hi = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (o[i] < 0 || l[i] < 0 || o[i] + l[i] > t_.cap.B) throw std::out_of_range("gather_records: record out of range");
      lo = std::min(lo, o[i]);
      hi = std::max(hi, o[i] + l[i]);
    }
    if (n == 0 || hi <= lo) return;
    std::vector<uint8_t> tmp;
    const uint8_t* base = payload_ + lo;
    if (gpu_) {
      tmp.resize(static_cast<size_t>(hi - lo));
      hip_check(hipMemcpy(tmp.data(), payload_ + lo, tmp.size(), hipMemcpyDeviceToHost), "payload gather");
      base = tmp.data();
    }
    size_t pos = 0;
    for (int64_t i = 0; i < n; ++i) {
      std::memcpy(dst + pos, base + (o[i] - lo), static_cast<size_t>(l[i]));
      pos += static_cast<size_t>(l[i]);
    }
  }

  // Same, for a payload the caller rendered (`at`: offset of the parent's `null`).
  // DeltaEngine.capture on the device: lay the record out in the payload arena
  // with a 66-byte hole for the quoted parent digest (turn > 1), and post
  // OP_DELTA_CAPTURE.  The device splices the chain head into the hole and hashes
  // (K08).  Nothing is recycled while it is live; full tables report -2 / -3.
  // `phex` (or null): the parent's predicted digest as 64 lowercase hex chars.  It
  // is written into the hole (quoted) and flagged in the command (a7 bit 0), so the
  // worker's helper waves can hash the whole record at once instead of waiting for
  // the parent's digest; the hash engine still splices and re-hashes when the
  // parent it computed differs (store_worker.hip, spec jobs).
  Placed capture_rendered(int64_t slot, int64_t turn, int64_t ts_us, const std::string& buf, size_t at,
                          const char* phex = nullptr) {
    const bool hole = turn > 1;
    const size_t len = hole ? buf.size() - 4 + 66 : buf.size();
    const int64_t didx = take_delta_row();
    if (didx < 0) return Placed{-2, -1, static_cast<int64_t>(len), -1};
    const int64_t off = arena_.alloc(static_cast<int64_t>(len));
    if (off < 0) {
      dfree_.push_back(static_cast<int32_t>(didx));
      return Placed{-3, -1, static_cast<int64_t>(len), -1};
    }
    d_off_[static_cast<size_t>(didx)] = off;
    d_len_[static_cast<size_t>(didx)] = static_cast<int64_t>(len);
    uint8_t* dst = payload_ + off;
    if (hole) {
      std::memcpy(dst, buf.data(), at);
      if (phex != nullptr) {
        dst[at] = '"';
        std::memcpy(dst + at + 1, phex, 64);
        dst[at + 65] = '"';
      }
      std::memcpy(dst + at + 66, buf.data() + at + 4, buf.size() - at - 4);
    } else {
      std::memcpy(dst, buf.data(), buf.size());
    }
    if (gpu_) _mm_sfence();
    const bool spec = hole && phex != nullptr;
    uint64_t a[8] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(didx), static_cast<uint64_t>(turn),
                     static_cast<uint64_t>(ts_us), static_cast<uint64_t>(off), static_cast<uint64_t>(len),
                     hole ? static_cast<uint64_t>(at) : ~0ull, spec ? 1ull : 0ull};
    const uint64_t q = post_raw(store::OP_DELTA_CAPTURE, a, spec ? 8 : 7, nullptr, 0);
    return Placed{didx, off, static_cast<int64_t>(len), static_cast<int64_t>(q)};
  }

  // Checkpoint restore: a delta row plus its record in the arena (the caller
  // writes the row's columns).  Returns {delta index, offset}; -2 / -3 as capture.
  std::pair<int64_t, int64_t> restore_delta_raw(const uint8_t* p, size_t n) {
    const int64_t len = static_cast<int64_t>(n);
    const int64_t didx = take_delta_row();
    if (didx < 0) return {-2, -1};
    const int64_t off = arena_.alloc(len);
    if (off < 0) {
      dfree_.push_back(static_cast<int32_t>(didx));
      return {-3, -1};
    }
    d_off_[static_cast<size_t>(didx)] = off;
    d_len_[static_cast<size_t>(didx)] = len;
    std::memcpy(payload_ + off, p, n);
    if (gpu_) _mm_sfence();
    return {didx, off};
  }

  // Delta rows + arena reservations for a batch of records (the batched store
  // pipelines render into them): `caps[i]` bytes each.  Fills rows/offs and returns
  // 0, or -2 (delta table full) / -3 (arena full) after releasing what it took.
  int reserve_deltas_raw(const int32_t* c, size_t n, int32_t* r, int64_t* o) {
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
        return d < 0 ? -2 : -3;
      }
      r[i] = static_cast<int32_t>(d);
      o[i] = off;
      d_off_[static_cast<size_t>(d)] = off;
      d_len_[static_cast<size_t>(d)] = c[i];  // the reservation is what a free returns
    }
    return 0;
  }

  // Reclaim delta rows (and their arena records) no API object refers to any
  // more: OP_FREE_ROWS marks them free on the device after the hash engine has
  // drained, then the rows and bytes return to the host free lists.
  void free_deltas(const std::vector<int32_t>& rows) {
    if (rows.empty()) return;
    for (int32_t d : rows)
      if (d < 0 || d >= t_.cap.D || d_off_[static_cast<size_t>(d)] < 0)
        throw std::invalid_argument("free_deltas: row " + std::to_string(d) + " is not allocated");
    free_rows_cmd(store::RK_D, rows);
    for (int32_t d : rows) {
      mark(dreleased_, d, 0);
      arena_.free(d_off_[static_cast<size_t>(d)], d_len_[static_cast<size_t>(d)]);
      d_off_[static_cast<size_t>(d)] = -1;
      d_len_[static_cast<size_t>(d)] = 0;
      dfree_.push_back(d);
    }
  }

  // OP_FREE_ROWS for any table; waits for completion.
  void free_rows_cmd(uint64_t kind, const std::vector<int32_t>& rows) {
    using namespace store;
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
      volatile uint64_t* rs = res_ + (q % static_cast<uint64_t>(nslots_)) * store::kResWords;
      if (rs[0] < q + 1) ++reclaim_waits_;  // not answered yet: this wait blocks
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
    std::vector<uint8_t> live;  // 1 while handed out and not released (double-release guard)
  };

  static void mark(std::vector<uint8_t>& v, int64_t row, uint8_t x) {
    if (row < 0) return;
    if (static_cast<size_t>(row) >= v.size()) v.resize(std::max<size_t>(static_cast<size_t>(row) + 1, 2 * v.size()), 0);
    v[static_cast<size_t>(row)] = x;
  }
  static bool is_set(const std::vector<uint8_t>& v, int64_t row) {
    return row >= 0 && static_cast<size_t>(row) < v.size() && v[static_cast<size_t>(row)] != 0;
  }

  static size_t pool_index(uint64_t kind) {
    switch (kind) {
      case store::RK_S: return 0;
      case store::RK_G: return 1;
      case store::RK_T: return 2;
      case store::RK_E: return 3;
      case store::RK_V: return 4;
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
      mark(p.live, r, 1);
      return r;
    }
    if (p.hw < p.cap) {
      mark(p.live, p.hw, 1);
      return p.hw++;
    }
    return -1;
  }

  // `n` free rows of `kind` into `out`, or false when the table cannot hold them (nothing taken).
  bool alloc_rows_raw(uint64_t kind, int64_t n, int32_t* out) {
    RowPool& p = pool(kind);
    if (!p.pend.empty()) reclaim_pool(kind);
    if (static_cast<int64_t>(p.free.size()) + (p.cap - p.hw) < n) return false;
    int64_t k = 0;
    while (k < n && !p.free.empty()) {
      out[k++] = p.free.back();
      p.free.pop_back();
    }
    while (k < n) out[k++] = static_cast<int32_t>(p.hw++);
    for (int64_t i = 0; i < n; ++i) mark(p.live, out[i], 1);
    return true;
  }

  // A released row leaves the live set once: a second release of the same row (two
  // views that both believed they owned it) is counted and ignored, so a row can
  // never enter the free list twice and be handed to two sessions.
  void release_row(uint64_t kind, int64_t row) {
    if (kind == store::RK_D) {
      if (row < 0 || row >= dhw_ || d_off_[static_cast<size_t>(row)] < 0 || is_set(dreleased_, row)) {
        ++double_releases_;
        return;
      }
      mark(dreleased_, row, 1);
      dpend_.push_back(static_cast<int32_t>(row));
      return;
    }
    RowPool& p = pool(kind);
    if (!is_set(p.live, row)) {
      ++double_releases_;
      return;
    }
    mark(p.live, row, 0);
    p.pend.push_back(static_cast<int32_t>(row));
  }

  void release_rows_raw(uint64_t kind, const int32_t* rows, int64_t n) {
    for (int64_t i = 0; i < n; ++i) release_row(kind, rows[i]);
  }

  // A row that was allocated but never written on the device (a refused vouch):
  // straight back to the free list.
  void return_row(uint64_t kind, int64_t row) {
    RowPool& p = pool(kind);
    mark(p.live, row, 0);
    p.free.push_back(static_cast<int32_t>(row));
  }

  // Return the queued rows of `kind` to its free list; returns their count.
  int64_t reclaim_pool(uint64_t kind) {
    if (kind == store::RK_D) {
      if (dpend_.empty()) return 0;
      std::vector<int32_t> rows;
      rows.swap(dpend_);
      ++reclaims_;
      free_deltas(rows);
      return static_cast<int64_t>(rows.size());
    }
    RowPool& p = pool(kind);
    if (p.pend.empty()) return 0;
    check_frees();
    std::vector<int32_t> rows;
    rows.swap(p.pend);
    ++reclaims_;
    post_frees(kind, rows);
    p.free.insert(p.free.end(), rows.begin(), rows.end());
    return static_cast<int64_t>(rows.size());
  }

  int64_t npend(uint64_t kind) const {
    return static_cast<int64_t>(kind == store::RK_D ? dpend_.size() : pools_[pool_index(kind)].pend.size());
  }
  int64_t live_rows(uint64_t kind) const {
    if (kind == store::RK_D) return delta_live() - static_cast<int64_t>(dpend_.size());
    const RowPool& p = pools_[pool_index(kind)];
    return p.hw - static_cast<int64_t>(p.free.size() + p.pend.size());
  }

  // OP_FREE_ROWS without waiting; statuses are checked by check_frees.
  void post_frees(uint64_t kind, const std::vector<int32_t>& rows) {
    using namespace store;
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
        volatile uint64_t* r = res_ + (q % static_cast<uint64_t>(nslots_)) * store::kResWords;
        if (r[0] < q + 1 && !block) break;
        if (r[0] < q + 1) ++reclaim_waits_;
        st = wait(q)[1];
        unwatch(q);
      }
      if (st != store::ST_OK) {
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

  // ------------------------------------------------------------ accessors
  const Tables& tables() const { return t_; }
  int64_t delta_live() const { return dhw_ - static_cast<int64_t>(dfree_.size()); }
  int64_t delta_hw() const { return dhw_; }
  int64_t payload_cap() const { return t_.cap.B; }
  int64_t payload_live() const { return arena_.live(); }
  int64_t payload_head() const { return arena_.head(); }
  int64_t bulk_cap() const { return bulk_cap_; }
  uintptr_t payload_ptr() const { return reinterpret_cast<uintptr_t>(payload_); }
  int64_t staging_cap() const { return staging_cap_; }
  void set_timeout(int s) { timeout_s_ = s; }
  bool gpu() const { return gpu_; }
  int device() const { return device_; }
  uint64_t posted() const { return posted_; }
  uint64_t ring_waits() const { return ring_waits_; }
  uint64_t ring_wait_ns() const { return ring_wait_ns_; }
  uint64_t launches() const { return launches_; }
  uint64_t reclaims() const { return reclaims_; }
  uint64_t reclaim_waits() const { return reclaim_waits_; }
  uint64_t double_releases() const { return double_releases_; }
  const uint64_t* trace_buf() const { return trace_; }
  int64_t trace_cap() const { return trace_cap_; }
  const std::vector<uint64_t>& post_ns() const { return post_ns_; }
  int64_t nslots() const { return nslots_; }
  size_t kept() const { return nwatch_ + saved_.size(); }
  const int64_t* tail() const { return tail_; }

 protected:
  void bind(const ColumnPtrs& ptrs) {
    auto get = [&](const char* k) -> uintptr_t {
      auto it = ptrs.find(k);
      if (it == ptrs.end()) throw std::invalid_argument(std::string("store column missing: ") + k);
      return it->second;
    };
#define AHV_PTR(name, type, ext) t_.name = reinterpret_cast<type*>(get(#name));
    AHV_STORE_COLUMNS(AHV_PTR)
#undef AHV_PTR
  }
  void set_pool_caps() {
    pools_[0].cap = t_.cap.S;
    pools_[1].cap = t_.cap.G;
    pools_[2].cap = t_.cap.T;
    pools_[3].cap = t_.cap.E;
    pools_[4].cap = t_.cap.V;
  }

  bool gpu_;
  int device_;
  int64_t nslots_;
  int64_t staging_cap_;
  int64_t bulk_cap_;
  Tables t_{};
  uint64_t* ring_ = nullptr;
  bool ring_host_ = false;  // command ring in pinned host memory (else fine-grained device memory)
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
  uint64_t ring_waits_ = 0;    // posts that found the ring full (waited for the worker)
  uint64_t ring_wait_ns_ = 0;  // host time spent in those waits
  uint64_t launches_ = 0;
  uint64_t double_releases_ = 0;  // releases of rows that were not live (ignored)
  std::vector<uint8_t> dreleased_;  // delta rows released and not yet reclaimed
  uint64_t* trace_ = nullptr;       // worker timeline (AHV_STORE_TRACE): [4·cap][4] words, pinned
  int64_t trace_cap_ = 0;
  std::vector<uint64_t> post_ns_;   // host post time of each traced sequence number (steady clock)
  uint64_t reclaims_ = 0;        // reclaim_pool passes that returned queued rows (any table)
  uint64_t reclaim_waits_ = 0;   // times a reclaim blocked on a FREE_ROWS result
  size_t stage_head_ = 0;
  ArenaAlloc arena_;
  // Per ring slot: seq + 1 of a kept result still in that slot (0: none) — a slot
  // holds one command at a time, so keeping / releasing a result is an array store
  // (the per-command hash-map node it replaced showed up under 10^4 concurrent pipelines)
  std::vector<uint64_t> watch_;
  size_t nwatch_ = 0;
  void watch(uint64_t q) {
    uint64_t& w = watch_[q % static_cast<uint64_t>(nslots_)];
    if (w != q + 1) {
      if (w == 0) ++nwatch_;
      w = q + 1;
    }
  }
  bool watched(uint64_t q) const { return watch_[q % static_cast<uint64_t>(nslots_)] == q + 1; }
  void unwatch(uint64_t q) {
    uint64_t& w = watch_[q % static_cast<uint64_t>(nslots_)];
    if (w == q + 1) {
      w = 0;
      --nwatch_;
    }
  }
  std::unordered_map<uint64_t, std::array<uint64_t, kSaveWords>> saved_;  // their results, once recycled
  std::vector<int64_t> d_off_, d_len_;  // arena record of each delta row (-1: row free)
  std::vector<int32_t> dfree_;          // reclaimed delta rows
  std::vector<int32_t> dpend_;          // delta rows released by their views, not reclaimed yet
  RowPool pools_[5];                    // S G T E V row allocators
  std::vector<uint64_t> frees_;         // FREE_ROWS posted without waiting, status unchecked
  int64_t dhw_ = 0;                     // delta rows ever handed out (high-water mark)
  int timeout_s_ = 30;
  bool closed_ = false;
};

}  // namespace host
}  // namespace ahv
