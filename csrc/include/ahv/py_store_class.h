// The Python-facing device store (pybind11 class `_C.Store`): argument
// conversion over `StoreCore` (ahv/store_host.h), the speculation expectations,
// and the capture path.  Shared by its bindings (csrc/host/py_store.cpp) and the
// native per-call control plane (csrc/host/py_control.cpp), which drives the same
// object without a Python frame per command.
#pragma once

#include <Python.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <deque>

#include "ahv/host_sha.h"
#include "ahv/store_host.h"

namespace py = pybind11;

namespace ahv {
void store_pipeline_run(const store::Tables& t, bool gpu, const pybind11::dict& d, uintptr_t stream);
void store_template_run(const store::Tables& t, bool gpu, const pybind11::dict& d, uintptr_t stream);

namespace host {

bool render_delta(PyObject* d, std::string& out, size_t* null_parent_at);

namespace storebind {

using namespace ahv::store;
using I32Array = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using I64Array = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

inline ColumnPtrs column_ptrs(const py::dict& d) {
  ColumnPtrs out;
  for (auto kv : d) out[kv.first.cast<std::string>()] = kv.second.cast<uintptr_t>();
  return out;
}

inline Caps caps_of(const py::dict& caps) {
  auto cap = [&](const char* k) { return caps[k].cast<int64_t>(); };
  return Caps{cap("S"), cap("P"), cap("D"), cap("E"), cap("V"), cap("G"), cap("T"), cap("X"), cap("B")};
}

inline py::tuple words(const uint64_t* r, int nres) {
  py::tuple out(nres);
  for (int k = 0; k < nres; ++k) out[k] = py::int_(static_cast<int64_t>(r[1 + k]));
  return out;
}

class Store : public StoreCore {
 public:
  Store(int device, const py::dict& ptrs, const py::dict& caps, int64_t nslots, int64_t staging_bytes,
        int64_t bulk_bytes, int64_t idle_us, int64_t max_ms)
      : StoreCore(device, column_ptrs(ptrs), caps_of(caps), nslots, staging_bytes, bulk_bytes, idle_us, max_ms) {}

  void rebind_py(const py::dict& ptrs, const py::dict& caps) {
    Caps c = caps_of_partial(caps);
    rebind(column_ptrs(ptrs), c);
  }

  uint64_t post(uint32_t op, const std::vector<int64_t>& args, const py::object& inl) {
    std::string buf;
    if (!inl.is_none()) buf = inl.cast<std::string>();
    return post_raw(op, reinterpret_cast<const uint64_t*>(args.data()), args.size(),
                    reinterpret_cast<const uint8_t*>(buf.data()), buf.size());
  }

  // post + wait; returns (r[1], r[2], ..., r[nres]) as ints (status first)
  py::tuple call(uint32_t op, const std::vector<int64_t>& args, int nres, const py::object& inl) {
    const uint64_t q = post(op, args, inl);
    return words(wait(q), nres);
  }

  py::object try_result(uint64_t q, int nres, int64_t spin_ns) {
    if (nres > kSaveWords - 1) throw std::invalid_argument("try_result: at most 15 result words");
    uint64_t r[kSaveWords];
    if (!try_result_raw(q, spin_ns, r)) return py::none();
    return words(r, nres);
  }

  // Results of an earlier post, or None once its slot has been recycled.
  py::object result(uint64_t q, int nres) {
    const uint64_t* r;
    try {
      r = wait(q);
    } catch (const ResultGone&) {
      return py::none();
    }
    return words(r, nres);
  }

  // ---- speculation: posted commands whose results the caller predicted ----
  //
  // An expectation is the leading result words a kept post must produce (None:
  // any value).  They are checked here, in post order, without a Python call per
  // result; only a mismatch hands its token (and the device's words) back to the
  // caller, which turns it into the prediction owner's error.
  struct Expect {
    uint64_t seq;
    uint32_t mask;
    uint64_t want[kSaveWords - 1];
    py::object token;
  };
  std::deque<Expect> expects_;
  py::list expect_bad_;  // mismatches found by an automatic blocking pass
  // Pending expectations past which each new one first checks the completed ones
  // (a non-blocking pass: it stops at the first result not in yet), and past which
  // it waits for them.  Under 10^4 concurrent pipelines thousands of speculated
  // posts are in flight; waiting at 512 made the posting thread spin on the worker.
  static constexpr size_t kExpectMax = 512;
  static constexpr size_t kExpectHard = size_t(1) << 16;

  void expect(uint64_t q, const py::tuple& want, py::object token) {
    uint64_t w[kSaveWords - 1] = {};
    uint32_t mask = 0;
    const size_t n = std::min<size_t>(want.size(), kSaveWords - 1);
    for (size_t k = 0; k < n; ++k) {
      py::handle x = want[k];
      if (x.is_none()) continue;
      mask |= 1u << k;
      w[k] = static_cast<uint64_t>(x.cast<int64_t>());
    }
    expect_mask(q, mask, w, std::move(token));
  }

  // The expectation of `q` as a mask of checked result words (bit k: word k must
  // equal want[k]) — the form the native control plane registers without tuples.
  void expect_mask(uint64_t q, uint32_t mask, const uint64_t* want, py::object token) {
    keep(q);
    Expect e;
    e.seq = q;
    e.mask = mask;
    for (int k = 0; k < kSaveWords - 1; ++k) e.want[k] = (mask >> k) & 1u ? want[k] : 0;
    e.token = std::move(token);
    expects_.push_back(std::move(e));
    if (expects_.size() >= kExpectMax) {
      py::object bad = verify_expects(expects_.size() >= kExpectHard);
      if (!bad.is_none())
        for (auto b : py::reinterpret_borrow<py::list>(bad)) expect_bad_.append(b);
    }
  }

  uint64_t post_expect_raw(uint32_t op, const uint64_t* args, size_t nargs, uint32_t mask, const uint64_t* want,
                           py::object token) {
    const uint64_t q = post_raw(op, args, nargs, nullptr, 0);
    expect_mask(q, mask, want, std::move(token));
    return q;
  }

  int64_t cap_participants() const { return t_.cap.P; }

  uint64_t post_expect(uint32_t op, const std::vector<int64_t>& args, const py::object& inl, const py::tuple& want,
                       py::object token) {
    const uint64_t q = post(op, args, inl);
    expect(q, want, std::move(token));
    return q;
  }

  // Check the expectations whose results are in (all of them with `block`);
  // returns [(token, result words)] for the mismatches, or None.
  py::object verify_expects(bool block) {
    if (expects_.empty() && expect_bad_.size() == 0) return py::none();
    py::object bad = py::none();  // a list only once there is a mismatch
    if (expect_bad_.size()) {
      bad = expect_bad_;
      expect_bad_ = py::list();
    }
    while (!expects_.empty()) {
      Expect& e = expects_.front();
      uint64_t buf[kSaveWords];
      // completed and still in its slot: compare the expected words in place
      const uint64_t* r = peek_done(e.seq);
      if (r == nullptr) {
        if (!try_result_raw(e.seq, 0, buf)) {
          if (!block) break;
          const auto t0 = std::chrono::steady_clock::now();
          while (!try_result_raw(e.seq, 1000000, buf)) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
              throw std::runtime_error("store: speculated command " + std::to_string(e.seq) + " never completed");
          }
        }
        r = buf;
      }
      bool ok = true;
      for (uint32_t m = e.mask; m && ok; m &= m - 1) {
        const int k = __builtin_ctz(m);
        ok = r[1 + k] == e.want[k];
      }
      if (!ok) {
        if (bad.is_none()) bad = py::list();
        py::reinterpret_borrow<py::list>(bad).append(py::make_tuple(e.token, words(r, kSaveWords - 1)));
      }
      expects_.pop_front();
    }
    return bad;
  }

  size_t n_expects() const { return expects_.size(); }

  int64_t stage(const py::bytes& b) {
    std::string_view v = b;
    return stage_raw(reinterpret_cast<const uint8_t*>(v.data()), v.size());
  }

  py::bytes bulk(int64_t off, int64_t n) const {
    return py::bytes(reinterpret_cast<const char*>(bulk_ptr(off, n)), static_cast<size_t>(n));
  }

  py::bytes payload(int64_t off, int64_t n) const {
    std::string out(static_cast<size_t>(std::max<int64_t>(n, 0)), '\0');
    payload_read(off, n, out.data());
    return py::bytes(out);
  }

  void write_payload(int64_t off, const py::bytes& b) {
    std::string_view v = b;
    write_payload_raw(off, v.data(), v.size());
  }

  void write_records(I64Array offs, I64Array lens, py::buffer blob) {
    if (lens.size() != offs.size()) throw std::invalid_argument("write_records: offs and lens differ in length");
    const py::buffer_info bi = blob.request();
    py::gil_scoped_release nogil;
    write_records_raw(offs.data(), lens.data(), offs.size(), static_cast<const uint8_t*>(bi.ptr),
                      static_cast<size_t>(bi.size * bi.itemsize));
  }

  // The records at `offs` / `lens`, concatenated (checkpoint save; no store command).
  py::bytes payload_gather(I64Array offs, I64Array lens) {
    if (lens.size() != offs.size()) throw std::invalid_argument("payload_gather: offs and lens differ in length");
    int64_t total = 0;
    for (py::ssize_t i = 0; i < lens.size(); ++i) total += std::max<int64_t>(lens.data()[i], 0);
    PyObject* out = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(total));
    if (!out) throw py::error_already_set();
    py::bytes res = py::reinterpret_steal<py::bytes>(out);
    uint8_t* dst = reinterpret_cast<uint8_t*>(PyBytes_AS_STRING(out));
    {
      py::gil_scoped_release nogil;
      gather_records_raw(offs.data(), lens.data(), offs.size(), dst);
    }
    return res;
  }

  // DeltaEngine.capture: render the canonical payload around a null parent
  // (py_audit.cpp), then place it (StoreCore::capture_rendered).
  // Returns (delta index, payload offset, payload length, sequence, predicted
  // digest): the digest the device will compute, hashed here with SHA-NI over
  // the same bytes (turn 1: the record as rendered; later turns: with `parent`,
  // the previous capture's predicted hex digest, spliced in quoted) — None when
  // the parent is not known.  The caller verifies it against the device later.
  py::tuple capture(int64_t slot, int64_t turn, int64_t ts_us, py::handle delta, const py::object& parent) {
    if (npend(store::RK_D) >= kReclaimDeltas) reclaim_pool(store::RK_D);  // released delta rows back in bulk
    thread_local std::string buf;
    size_t at = 0;
    if (!render_delta(delta.ptr(), buf, &at)) return py::make_tuple(-1, -1, -1, -1, py::none());
    const Placed p = capture_rendered(slot, turn, ts_us, buf, at, parent_hex(turn, parent));
    return py::make_tuple(p.didx, p.off, p.len, p.seq, p.didx >= 0 ? predict(buf, at, turn, parent) : py::none());
  }

  // The predicted parent digest's 64 hex chars (turn > 1 and a canonical hex str), or null.
  static const char* parent_hex(int64_t turn, const py::object& parent) {
    if (turn <= 1 || parent.is_none() || !PyUnicode_Check(parent.ptr())) return nullptr;
    PyObject* o = parent.ptr();
    if (PyUnicode_GET_LENGTH(o) != 64 || !PyUnicode_IS_COMPACT_ASCII(o)) return nullptr;
    const char* ph = static_cast<const char*>(PyUnicode_DATA(o));
    for (int k = 0; k < 64; ++k)
      if (!((ph[k] >= '0' && ph[k] <= '9') || (ph[k] >= 'a' && ph[k] <= 'f'))) return nullptr;
    return ph;
  }

  // Released delta rows reclaimed per batch.  The reclaim's OP_FREE_ROWS waits for the
  // hash engine to drain (its records must be hashed before their arena bytes are
  // reused), which under a steady capture stream is the engine's whole backlog
  // (≈1.5 ms): batches of 4,096 rows pay it once per ≈1,400 pipelines instead of once
  // per ≈85 (256 rows: a +19 µs mean on the per-call path, profiles/r4/
  // percall_outliers_r4y_before_async_reclaim.txt).
  static constexpr int64_t kReclaimDeltas = 4096;  // == GovernanceStore.RECLAIM_BATCH

  py::tuple capture_bytes(int64_t slot, int64_t turn, int64_t ts_us, const py::bytes& payload, int64_t null_at,
                          const py::object& parent) {
    if (npend(store::RK_D) >= kReclaimDeltas) reclaim_pool(store::RK_D);
    std::string buf = payload;
    if (null_at < 0 || static_cast<size_t>(null_at) + 4 > buf.size() || buf.compare(null_at, 4, "null") != 0)
      throw std::invalid_argument("capture_bytes: null_at does not point at the parent's null");
    const Placed p = capture_rendered(slot, turn, ts_us, buf, static_cast<size_t>(null_at), parent_hex(turn, parent));
    return py::make_tuple(p.didx, p.off, p.len, p.seq,
                          p.didx >= 0 ? predict(buf, static_cast<size_t>(null_at), turn, parent) : py::none());
  }

  static py::object predict(const std::string& buf, size_t at, int64_t turn, const py::object& parent) {
    uint32_t h[8];
    if (turn <= 1) {
      host::sha256_bytes(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), h);
    } else {
      if (parent.is_none() || !PyUnicode_Check(parent.ptr())) return py::none();
      Py_ssize_t n = 0;
      const char* ph = PyUnicode_AsUTF8AndSize(parent.ptr(), &n);
      if (ph == nullptr || n != 64) {
        PyErr_Clear();
        return py::none();
      }
      thread_local std::string rec;
      rec.assign(buf.data(), at);
      rec.push_back('"');
      rec.append(ph, 64);
      rec.push_back('"');
      rec.append(buf.data() + at + 4, buf.size() - at - 4);
      host::sha256_bytes(reinterpret_cast<const uint8_t*>(rec.data()), rec.size(), h);
    }
    PyObject* out = PyUnicode_New(64, 127);
    if (out == nullptr) throw py::error_already_set();
    host::hex_bytes(h, PyUnicode_1BYTE_DATA(out));
    return py::reinterpret_steal<py::object>(out);
  }

  // Reference Merkle root over predicted hex digests (SHA-NI), or None when one
  // is missing or not canonical hex.
  static py::object merkle_predict(const py::list& leaves) {
    const size_t n = leaves.size();
    if (n == 0) return py::none();
    std::vector<uint32_t> level(8 * n);
    for (size_t i = 0; i < n; ++i) {
      PyObject* o = leaves[i].ptr();
      if (!PyUnicode_Check(o) || PyUnicode_GET_LENGTH(o) != 64 || PyUnicode_KIND(o) != PyUnicode_1BYTE_KIND)
        return py::none();
      const uint8_t* c = PyUnicode_1BYTE_DATA(o);
      for (int w = 0; w < 8; ++w) {
        uint32_t x = 0;
        for (int k = 0; k < 8; ++k) {
          const uint8_t ch = c[8 * w + k];
          uint32_t v;
          if (ch >= '0' && ch <= '9') v = ch - '0';
          else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
          else return py::none();
          x = (x << 4) | v;
        }
        level[8 * i + w] = x;
      }
    }
    if (n == 1) return leaves[0];
    uint32_t root[8];
    host::merkle_root_host(level.data(), n, root);
    PyObject* out = PyUnicode_New(64, 127);
    if (out == nullptr) throw py::error_already_set();
    host::hex_bytes(root, PyUnicode_1BYTE_DATA(out));
    return py::reinterpret_steal<py::object>(out);
  }

  py::tuple restore_delta(const py::bytes& b) {
    std::string_view v = b;
    const auto r = restore_delta_raw(reinterpret_cast<const uint8_t*>(v.data()), v.size());
    return py::make_tuple(r.first, r.second);
  }

  // (int32 rows bytes, int64 offsets bytes), or (code, None).
  py::tuple reserve_deltas(const py::bytes& caps) {
    std::string_view v = caps;
    const size_t n = v.size() / 4;
    std::string rows(n * 4, '\0'), offs(n * 8, '\0');
    const int rc = reserve_deltas_raw(reinterpret_cast<const int32_t*>(v.data()), n,
                                      reinterpret_cast<int32_t*>(rows.data()), reinterpret_cast<int64_t*>(offs.data()));
    if (rc) return py::make_tuple(rc, py::none());
    return py::make_tuple(py::bytes(rows), py::bytes(offs));
  }

  // The batched store pipelines (csrc/hip/store_pipeline.hip, store_template.hip)
  // over this store's tables on `stream`; the caller released the worker's writes
  // (OP_FLUSH) before and has it acquire the new rows (OP_ACQUIRE) after.
  void run_pipeline(const py::dict& d, uintptr_t stream) { store_pipeline_run(t_, gpu_, d, stream); }
  void run_template(const py::dict& d, uintptr_t stream) { store_template_run(t_, gpu_, d, stream); }

  py::object alloc_rows(uint64_t kind, int64_t n) {
    py::array_t<int32_t> out(n);
    if (!alloc_rows_raw(kind, n, out.mutable_data())) return py::none();
    return std::move(out);
  }

  void release_rows(uint64_t kind, I32Array a) { release_rows_raw(kind, a.data(), a.size()); }

  // A short Python list of rows (a chain's delta rows from a finaliser): no array.
  void release_list(uint64_t kind, const py::list& rows) {
    for (auto r : rows) release_row(kind, r.cast<int64_t>());
  }

  // The worker timeline (AHV_STORE_TRACE): (commands uint64[cap,4], engine jobs uint64[cap,4],
  // host post times uint64[cap], provisional Merkle trees uint64[cap,4], helper-wave jobs
  // uint64[cap,4]) as bytes, or None when tracing is off.
  py::object trace() const {
    if (trace_buf() == nullptr) return py::none();
    const size_t cap = static_cast<size_t>(trace_cap());
    const char* b = reinterpret_cast<const char*>(trace_buf());
    return py::make_tuple(py::bytes(b, cap * 32), py::bytes(b + cap * 32, cap * 32),
                          py::bytes(reinterpret_cast<const char*>(post_ns().data()), cap * 8),
                          py::bytes(b + cap * 64, cap * 32), py::bytes(b + cap * 96, cap * 32));
  }

  py::dict info() const {
    py::dict d;
    d["gpu"] = gpu_;
    d["device"] = device_;
    d["posted"] = posted_;
    d["ring_waits"] = ring_waits();
    d["ring_wait_us"] = static_cast<double>(ring_wait_ns()) / 1e3;
    d["launches"] = launches_;
    d["reclaims"] = reclaims();
    d["reclaim_waits"] = reclaim_waits();
    d["double_releases"] = double_releases();
    d["nslots"] = nslots_;
    d["payload_live"] = payload_live();
    d["payload_head"] = payload_head();
    d["payload_cap"] = t_.cap.B;
    d["delta_rows"] = delta_live();
    d["delta_hw"] = delta_hw();
    d["delta_cap"] = t_.cap.D;
    d["kept"] = static_cast<int64_t>(kept());  // posted results awaiting their reader
    if (gpu_) {  // worker utilisation telemetry (store_worker.hip; s_memrealtime ticks are 10 ns)
      d["worker_busy_us"] = static_cast<double>(__atomic_load_n(tail_ + 1, __ATOMIC_RELAXED)) / 100.0;
      d["worker_commands"] = __atomic_load_n(tail_ + 2, __ATOMIC_RELAXED);
      d["engine_busy_us"] = static_cast<double>(__atomic_load_n(tail_ + 3, __ATOMIC_RELAXED)) / 100.0;
      d["engine_jobs"] = __atomic_load_n(tail_ + 4, __ATOMIC_RELAXED);
    }
    return d;
  }

 private:
  Caps caps_of_partial(const py::dict& caps) const {  // growth: the arena keeps its own size
    Caps c = caps_of_nb(caps);
    c.B = t_.cap.B;
    return c;
  }
  static Caps caps_of_nb(const py::dict& caps) {
    auto cap = [&](const char* k) { return caps[k].cast<int64_t>(); };
    return Caps{cap("S"), cap("P"), cap("D"), cap("E"), cap("V"), cap("G"), cap("T"), cap("X"), 0};
  }
};

}  // namespace storebind
}  // namespace host
}  // namespace ahv
