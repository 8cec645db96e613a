// Native per-call control plane of the device-backed public API.
//
// `Hypervisor(device=...)` answers every reference call (create → join →
// activate → capture × n → saga create / add / execute → terminate, reference
// src/hypervisor/core.py:94-227) with commands to the device store.  The
// commands themselves were native already (ahv/store_host.h); what each call
// still paid was the Python around them: a handful of frames per call that
// look up rows and ids, pack argument lists, register speculation tokens and
// build the returned view objects (hypervisor/_device.py).  The functions below
// do that work in C++ against the same objects:
//
//   * they are bound as methods of the same Python classes (DeviceDeltaEngine.
//     capture, DeviceSagaOrchestrator.create_saga / add_step, ...) or called once
//     per API call from hypervisor/core.py, so the public API, the classes and
//     their attributes are unchanged — the views they return are the ordinary
//     Python objects, created here with their instance dicts filled directly;
//   * each handles the common case end to end (validate → intern → allocate row
//     → post → register the expectation → build the view) and hands anything
//     else — a pinned clock's odd values, a full table that must grow, a
//     refused speculation, an unusual argument — to the Python implementation it
//     replaces, before it has changed any state, so both paths keep one
//     semantics (the reference oracle and the device test suites run through
//     both: AHV_NATIVE_CTL=0 selects the Python path).
//
// Everything runs with the GIL held, on the caller's thread.
#include "ahv/py_store_class.h"

#include <datetime.h>
#include <time.h>

#include "ahv/semantics.h"
#include "ahv/string_pool.h"

namespace ahv {
namespace host {

bool render_delta_fields(PyObject* agent, PyObject* changes, PyObject* delta_id, PyObject* parent, PyObject* session,
                         PyObject* ts, PyObject* turn, std::string& out, size_t* null_parent_at);
PyObject* mint_uuid4(const char* prefix, size_t pl, uint64_t* hi_out, uint64_t* lo_out);

namespace {

using storebind::Store;

// ------------------------------------------------------------------ helpers

struct Own {  // owning reference
  PyObject* p = nullptr;
  Own() = default;
  explicit Own(PyObject* q) : p(q) {}
  ~Own() { Py_XDECREF(p); }
  Own(const Own&) = delete;
  Own& operator=(const Own&) = delete;
  PyObject* release() {
    PyObject* q = p;
    p = nullptr;
    return q;
  }
  explicit operator bool() const { return p != nullptr; }
};

// Interned attribute / key names.
struct Names {
#define AHV_NAMES(X)                                                                                                 \
  X(_store) X(_c) X(agents) X(_pool) X(_deferred) X(_distribute) X(verify_deferred) X(_poisoned) X(_cseq)            \
  X(_created) X(slot) X(session_id) X(creator_did) X(config) X(vfs_namespace) X(_vfs_snapshots) X(_m_state)          \
  X(_m_rows) X(_m_active) X(_m_cfg) X(_stamp) X(_owner) X(_deltas) X(_rows) X(_turn_counter) X(_sagas) X(_reg)        \
  X(delta_id) X(turn_id) X(agent_did) X(timestamp) X(changes) X(_prev) X(_dev_hash) X(_hash_override)                \
  X(_parent_override) X(_didx) X(_poff) X(_plen) X(_seq) X(_dirty) X(_pred) X(_tsu) X(_override) X(max_participants) \
  X(min_sigma_eff) X(enable_audit) X(consistency_mode) X(saga_id) X(steps) X(error) X(execute_result)                 \
  X(compensation_result) X(step_id) X(action_id) X(execute_api) X(undo_api) X(timeout_seconds) X(max_retries)        \
  X(_hint) X(append) X(capture) X(alloc) X(_tenant_v) X(_tenant) X(gc) X(policy) X(delta_retention_days) X(sso)      \
  X(delta_engine) X(saga) X(_sessions) X(_segs) X(_own) X(vouching) X(commitment) X(_closed) X(event_bus)   \
  X(_device) X(_commits)
#define AHV_DECL(n) PyObject* n = nullptr;
  AHV_NAMES(AHV_DECL)
#undef AHV_DECL
  void init() {
#define AHV_INIT(n) n = PyUnicode_InternFromString(#n);
    AHV_NAMES(AHV_INIT)
#undef AHV_INIT
  }
};
Names N;

// What the Python side hands over once (hypervisor/_device.py _install_native).
struct Ctl {
  bool ready = false;
  PyObject* GovernanceStore = nullptr;
  PyObject* DeviceSession = nullptr;
  PyObject* DeviceDelta = nullptr;
  PyObject* DeviceDeltaEngine = nullptr;
  PyObject* DeviceSagaOrchestrator = nullptr;
  PyObject* DeviceSaga = nullptr;
  PyObject* DeviceSagaStep = nullptr;
  PyObject* DeviceCommitmentEngine = nullptr;
  PyObject* CLOSED = nullptr;
  PyObject* clock_dict = nullptr;   // hypervisor._clock.__dict__ ("_override": a pinned clock)
  PyObject* py_now = nullptr;       // hypervisor._clock.now
  PyObject* py_to_us = nullptr;     // hypervisor._clock.to_us
  PyObject* mode_eventual = nullptr, *mode_strong = nullptr;
  PyObject* step_pending = nullptr, *step_executing = nullptr, *step_committed = nullptr;
  PyObject* exec_from = nullptr;    // frozenset of StepStates EXECUTING may follow
  PyObject* err_create = nullptr, *err_join = nullptr, *err_activate = nullptr, *err_transition = nullptr;
  // the Python implementations the natives replace (fallbacks)
  PyObject* fb_capture = nullptr, *fb_create_saga = nullptr, *fb_add_step = nullptr;
  int s_handshaking = 1, s_active = 2;
  int step_executing_idx = 0, step_committed_idx = 0;
  bool spec_lifecycle = true, step_speculate = true, spec_terminate = false, check_terminate = true;
  PyObject* empty_tuple = nullptr;
  PyObject* close_hv_fast = nullptr;  // _C.ctl_close_hypervisor
};
Ctl C;

inline PyObject* idict(PyObject* o) { return PyObject_GenericGetDict(o, nullptr); }  // new reference

inline PyObject* dget(PyObject* d, PyObject* k) { return PyDict_GetItemWithError(d, k); }  // borrowed

// The store's C++ object and agent interner, cached for the last store seen.
struct StoreCache {
  PyObject* obj = nullptr;  // strong ref: the address is never reused while cached
  PyObject* c = nullptr;    // its `_c` (strong)
  PyObject* pool = nullptr; // its agents interner's StringPool (strong)
  Store* s = nullptr;
  StringPool* agents = nullptr;
};
StoreCache g_store;

Store* store_of(PyObject* gs, StringPool** agents = nullptr) {
  if (Py_TYPE(gs) != reinterpret_cast<PyTypeObject*>(C.GovernanceStore)) return nullptr;
  Own d(idict(gs));
  if (!d) return nullptr;
  PyObject* c = dget(d.p, N._c);
  if (c == nullptr) return nullptr;
  if (gs == g_store.obj && c == g_store.c) {
    if (agents) *agents = g_store.agents;
    return g_store.s;
  }
  Store* s = nullptr;
  StringPool* pool = nullptr;
  PyObject* pool_obj = nullptr;
  try {
    s = py::handle(c).cast<Store*>();
    PyObject* ag = dget(d.p, N.agents);
    if (ag == nullptr) return nullptr;
    Own agd(idict(ag));
    if (!agd) return nullptr;
    pool_obj = dget(agd.p, N._pool);
    if (pool_obj == nullptr) return nullptr;
    pool = py::handle(pool_obj).cast<StringPool*>();
  } catch (...) {
    PyErr_Clear();
    return nullptr;
  }
  Py_INCREF(gs);
  Py_INCREF(c);
  Py_INCREF(pool_obj);
  Py_XDECREF(g_store.obj);
  Py_XDECREF(g_store.c);
  Py_XDECREF(g_store.pool);
  g_store = StoreCache{gs, c, pool_obj, s, pool};
  if (agents) *agents = pool;
  return s;
}

// An agent DID's dense id (GovernanceStore.agent_id); -1: not a str the fast
// path interns (the Python path handles it).
int64_t agent_id(StringPool* pool, PyObject* did) {
  if (!PyUnicode_CheckExact(did)) return -1;
  Py_ssize_t n = 0;
  const char* u = PyUnicode_AsUTF8AndSize(did, &n);
  if (u == nullptr) {
    PyErr_Clear();
    return -1;
  }
  return pool->intern(std::string_view(u, static_cast<size_t>(n)));
}

bool clock_pinned() {
  PyObject* o = PyDict_GetItem(C.clock_dict, N._override);
  return o != nullptr && o != Py_None;
}

int64_t sys_now_us() {  // time.time_ns() // 1000 (CLOCK_REALTIME)
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  return static_cast<int64_t>(t.tv_sec) * 1000000 + t.tv_nsec / 1000;
}

// hypervisor._clock.now_us(): the system clock, or to_us(pinned clock()).
bool now_us(int64_t* out) {
  if (!clock_pinned()) {
    *out = sys_now_us();
    return true;
  }
  Own ts(PyObject_CallNoArgs(C.py_now));
  if (!ts) return false;
  Own us(PyObject_CallOneArg(C.py_to_us, ts.p));
  if (!us) return false;
  *out = PyLong_AsLongLong(us.p);
  return !(*out == -1 && PyErr_Occurred());
}

// hypervisor._clock.now() and its µs: an aware UTC datetime built from the same
// CLOCK_REALTIME instant `datetime.now(timezone.utc)` reads (floored to µs).
PyObject* now_dt(int64_t* us_out) {
  if (clock_pinned()) {
    Own ts(PyObject_CallNoArgs(C.py_now));
    if (!ts) return nullptr;
    Own us(PyObject_CallOneArg(C.py_to_us, ts.p));
    if (!us) return nullptr;
    *us_out = PyLong_AsLongLong(us.p);
    if (*us_out == -1 && PyErr_Occurred()) return nullptr;
    return ts.release();
  }
  const int64_t us = sys_now_us();
  *us_out = us;
  const UtcParts t = utc_parts(us);
  return PyDateTimeAPI->DateTime_FromDateAndTime(static_cast<int>(t.year), static_cast<int>(t.month),
                                                 static_cast<int>(t.day), static_cast<int>(t.secs / 3600),
                                                 static_cast<int>((t.secs / 60) % 60), static_cast<int>(t.secs % 60),
                                                 static_cast<int>(t.micro), PyDateTime_TimeZone_UTC,
                                                 PyDateTimeAPI->DateTimeType);
}

int64_t dbits(double x) {
  int64_t v;
  std::memcpy(&v, &x, 8);
  return v;
}

// A new instance of `type` (object.__new__: no __init__ runs) and its instance
// dict (new reference) for the caller to fill.
PyObject* new_view(PyObject* type, PyObject** dict_out) {
  PyObject* o = PyBaseObject_Type.tp_new(reinterpret_cast<PyTypeObject*>(type), C.empty_tuple, nullptr);
  if (o == nullptr) return nullptr;
  PyObject* d = idict(o);
  if (d == nullptr) {
    Py_DECREF(o);
    return nullptr;
  }
  *dict_out = d;
  return o;
}

// dict[key] = value, stealing `value` (nullptr: an error is already set).
inline bool dset_steal(PyObject* d, PyObject* k, PyObject* v) {
  if (v == nullptr) return false;
  const int rc = PyDict_SetItem(d, k, v);
  Py_DECREF(v);
  return rc == 0;
}
inline bool dset(PyObject* d, PyObject* k, PyObject* v) { return PyDict_SetItem(d, k, v) == 0; }

// The expectation token (owner, make_error, arg) a speculated post carries.
PyObject* token(PyObject* owner, PyObject* make, PyObject* arg_steal) {
  if (arg_steal == nullptr) return nullptr;
  PyObject* t = PyTuple_New(3);
  if (t == nullptr) {
    Py_DECREF(arg_steal);
    return nullptr;
  }
  Py_INCREF(owner);
  Py_INCREF(make);
  PyTuple_SET_ITEM(t, 0, owner);
  PyTuple_SET_ITEM(t, 1, make);
  PyTuple_SET_ITEM(t, 2, arg_steal);
  return t;
}

// GovernanceStore.verify_deferred() (non-blocking): mismatches of speculated
// posts whose results are in go to their owners; an unowned one raises.
bool verify_deferred(PyObject* gs, Store* s) {
  Own d(idict(gs));
  if (!d) return false;
  PyObject* dl = dget(d.p, N._deferred);
  if (dl != nullptr && PyList_CheckExact(dl) && PyList_GET_SIZE(dl) > 0) {  // Python-side deferred checks
    Own r(PyObject_CallMethodNoArgs(gs, N.verify_deferred));
    return static_cast<bool>(r);
  }
  py::object bad;
  try {
    bad = s->verify_expects(false);
  } catch (py::error_already_set& e) {
    e.restore();
    return false;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return false;
  }
  if (bad.is_none()) return true;
  Own err(PyObject_CallMethodOneArg(gs, N._distribute, bad.ptr()));
  if (!err) return false;
  if (err.p != Py_None) {
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(err.p)), err.p);
    return false;
  }
  return true;
}

// DeviceSession._guard(): verify, then raise the session's speculation failure.
bool guard(PyObject* gs, Store* s, PyObject* sso_dict) {
  if (!verify_deferred(gs, s)) return false;
  PyObject* p = dget(sso_dict, N._poisoned);
  if (p != nullptr && p != Py_None) {
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(p)), p);
    return false;
  }
  return !PyErr_Occurred();
}

// The Python call a native method hands an unusual case to.
PyObject* fallback(PyObject* fn, PyObject* const* args, Py_ssize_t nargsf, PyObject* kwnames) {
  return PyObject_Vectorcall(fn, args, PyVectorcall_NARGS(nargsf), kwnames);
}

int64_t as_i64(PyObject* o, bool* ok) {
  if (!PyLong_Check(o)) {
    *ok = false;
    return 0;
  }
  int overflow = 0;
  const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
  if (overflow || (v == -1 && PyErr_Occurred())) {
    PyErr_Clear();
    *ok = false;
    return 0;
  }
  return v;
}

template <class F>
PyObject* guarded(F&& f) {  // C++ exceptions → Python exceptions
  try {
    return f();
  } catch (py::error_already_set& e) {
    e.restore();
    return nullptr;
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

// ------------------------------------------------------------------ capture

// DeviceDeltaEngine.capture(self, agent_did, changes, delta_id=None)
// (hypervisor/_device.py DeviceDeltaEngine._py_capture): render the canonical
// record, place it in the arena, post OP_DELTA_CAPTURE, predict its digest with
// SHA-NI, and return the DeviceDelta view — one native call.
PyObject* ctl_capture(PyObject*, PyObject* const* args, Py_ssize_t nargsf, PyObject* kwnames) {
  return guarded([&]() -> PyObject* {
    const Py_ssize_t n = PyVectorcall_NARGS(nargsf);
    PyObject* delta_id = Py_None;
    if (kwnames != nullptr) {
      if (n != 3 || PyTuple_GET_SIZE(kwnames) != 1 ||
          PyUnicode_Compare(PyTuple_GET_ITEM(kwnames, 0), N.delta_id) != 0)
        return fallback(C.fb_capture, args, nargsf, kwnames);
      delta_id = args[3];
    } else if (n == 4) {
      delta_id = args[3];
    } else if (n != 3) {
      return fallback(C.fb_capture, args, nargsf, kwnames);
    }
    PyObject* eng = args[0];
    PyObject* agent = args[1];
    PyObject* changes = args[2];
    Own ed(idict(eng));
    if (!ed) return nullptr;
    PyObject* gs = dget(ed.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* deltas = dget(ed.p, N._deltas);
    PyObject* rows = dget(ed.p, N._rows);
    PyObject* tc = dget(ed.p, N._turn_counter);
    PyObject* slot_o = dget(ed.p, N.slot);
    PyObject* sid = dget(ed.p, N.session_id);
    bool ok = true;
    const int64_t turn = tc ? as_i64(tc, &ok) + 1 : 0;
    const int64_t slot = slot_o ? as_i64(slot_o, &ok) : 0;
    if (s == nullptr || !ok || deltas == nullptr || !PyList_CheckExact(deltas) || rows == nullptr ||
        !PyList_CheckExact(rows) || sid == nullptr || PyErr_Occurred())
      return fallback(C.fb_capture, args, nargsf, kwnames);
    int64_t tsu = 0;
    Own ts(now_dt(&tsu));
    if (!ts) return nullptr;
    Own turn_o(PyLong_FromLongLong(turn));
    if (!turn_o) return nullptr;
    Own did;
    const int truth = PyObject_IsTrue(delta_id);
    if (truth < 0) return nullptr;
    if (truth) {
      Py_INCREF(delta_id);
      did.p = delta_id;
    } else {
      did.p = PyUnicode_FromFormat("delta:%lld", static_cast<long long>(turn));
      if (!did) return nullptr;
    }
    thread_local std::string buf;
    size_t at = 0;
    if (!render_delta_fields(agent, changes, did.p, Py_None, sid, ts.p, turn_o.p, buf, &at)) {
      if (PyErr_Occurred()) return nullptr;
      return fallback(C.fb_capture, args, nargsf, kwnames);  // types json.dumps renders: Python path
    }
    const Py_ssize_t nd = PyList_GET_SIZE(deltas);
    PyObject* prev = nd ? PyList_GET_ITEM(deltas, nd - 1) : Py_None;
    PyObject* parent = Py_None;
    Own prev_d;
    if (prev != Py_None) {
      prev_d.p = idict(prev);
      if (!prev_d) return nullptr;
      PyObject* pp = dget(prev_d.p, N._pred);
      if (pp == nullptr) return fallback(C.fb_capture, args, nargsf, kwnames);  // not a captured view
      parent = pp;
    }
    // the view first (the Python path's store.capture may need it to retry)
    PyObject* dd = nullptr;
    Own d(new_view(C.DeviceDelta, &dd));
    if (!d) return nullptr;
    Own ddict(dd);
    if (!(dset(dd, N.delta_id, did.p) && dset(dd, N.turn_id, turn_o.p) && dset(dd, N.session_id, sid) &&
          dset(dd, N.agent_did, agent) && dset(dd, N.timestamp, ts.p) && dset(dd, N.changes, changes) &&
          dset(dd, N._store, gs) && dset(dd, N._prev, prev) && dset(dd, N._dev_hash, Py_None) &&
          dset(dd, N._hash_override, Py_None) && dset(dd, N._parent_override, Py_None)))
      return nullptr;
    int64_t didx, off, len, seq;
    py::object pred;
    const py::object parent_o = py::reinterpret_borrow<py::object>(parent);
    if (s->npend(store::RK_D) >= Store::kReclaimDeltas) s->reclaim_pool(store::RK_D);
    const Placed p = s->capture_rendered(slot, turn, tsu, buf, at, Store::parent_hex(turn, parent_o));
    if (p.didx <= -2) {
      // full delta table / arena (nothing was taken): GovernanceStore.capture makes
      // room (reclaim, grow) and retries
      Own tsu_o(PyLong_FromLongLong(tsu));
      if (!tsu_o) return nullptr;
      Own r(PyObject_CallMethodObjArgs(gs, N.capture, slot_o, turn_o.p, tsu_o.p, d.p, parent, nullptr));
      if (!r) return nullptr;
      bool rok = PyTuple_Check(r.p) && PyTuple_GET_SIZE(r.p) == 5;
      didx = rok ? as_i64(PyTuple_GET_ITEM(r.p, 0), &rok) : -1;
      off = rok ? as_i64(PyTuple_GET_ITEM(r.p, 1), &rok) : -1;
      len = rok ? as_i64(PyTuple_GET_ITEM(r.p, 2), &rok) : -1;
      seq = rok ? as_i64(PyTuple_GET_ITEM(r.p, 3), &rok) : -1;
      if (!rok || didx < 0) {
        PyErr_SetString(PyExc_RuntimeError, "store capture: no delta row after making room");
        return nullptr;
      }
      pred = py::reinterpret_borrow<py::object>(PyTuple_GET_ITEM(r.p, 4));
    } else {
      didx = p.didx;
      off = p.off;
      len = p.len;
      seq = p.seq;
      pred = Store::predict(buf, at, turn, parent_o);
    }
    if (!(dset_steal(dd, N._didx, PyLong_FromLongLong(didx)) && dset_steal(dd, N._poff, PyLong_FromLongLong(off)) &&
          dset_steal(dd, N._plen, PyLong_FromLongLong(len)) && dset_steal(dd, N._seq, PyLong_FromLongLong(seq)) &&
          dset(dd, N._dirty, Py_False) && dset(dd, N._pred, pred.ptr()) &&
          dset_steal(dd, N._tsu, PyLong_FromLongLong(tsu))))
      return nullptr;
    Own di(PyLong_FromLongLong(didx));
    if (!di || PyList_Append(rows, di.p) < 0) return nullptr;
    if (PyDict_SetItem(ed.p, N._turn_counter, turn_o.p) < 0) return nullptr;
    if (PyList_Append(deltas, d.p) < 0) return nullptr;
    return d.release();
  });
}

// ------------------------------------------------------------------ sessions

// (sso, delta engine, saga orchestrator) of a new device session — DeviceSession
// (store, config, creator_did) + session_views(store, sso, saga_reg) — or None
// when the Python constructors must run (explicit id, speculation off, unusual
// config values, a full session table).
PyObject* ctl_session(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 5) {
      PyErr_SetString(PyExc_TypeError, "ctl_session(store, config, creator_did, session_id, saga_reg)");
      return nullptr;
    }
    PyObject* gs = args[0];
    PyObject* config = args[1];
    PyObject* creator = args[2];
    PyObject* reg = args[4];
    if (args[3] != Py_None || !C.spec_lifecycle) Py_RETURN_NONE;
    StringPool* pool = nullptr;
    Store* s = store_of(gs, &pool);
    if (s == nullptr) Py_RETURN_NONE;
    Own maxp(PyObject_GetAttr(config, N.max_participants));
    Own mins(PyObject_GetAttr(config, N.min_sigma_eff));
    Own aud(PyObject_GetAttr(config, N.enable_audit));
    Own mode(PyObject_GetAttr(config, N.consistency_mode));
    if (!maxp || !mins || !aud || !mode) return nullptr;
    bool ok = PyLong_CheckExact(maxp.p);
    const int64_t mp = ok ? as_i64(maxp.p, &ok) : 0;
    const bool ms_ok = PyFloat_CheckExact(mins.p) || PyLong_CheckExact(mins.p);
    const double ms = ms_ok ? PyFloat_AsDouble(mins.p) : 0.0;
    if (PyErr_Occurred()) PyErr_Clear();
    const int audit = PyObject_IsTrue(aud.p);
    if (audit < 0) return nullptr;
    int mode_code;
    if (mode.p == C.mode_eventual) mode_code = 0;
    else if (mode.p == C.mode_strong) mode_code = 1;
    else mode_code = -1;
    if (!ok || !ms_ok || mode_code < 0 || mp < INT32_MIN || mp > INT32_MAX) Py_RETURN_NONE;
    const int64_t aid = agent_id(pool, creator);
    if (aid < 0) Py_RETURN_NONE;
    int64_t now;
    if (!now_us(&now)) return nullptr;
    const int64_t slot = s->alloc_row(store::RK_S);
    if (slot < 0) Py_RETURN_NONE;  // full table: GovernanceStore.alloc grows it
    uint64_t hi = 0, lo = 0;
    static const char kPrefix[] = "session:";
    Own sid(mint_uuid4(kPrefix, sizeof kPrefix - 1, &hi, &lo));
    Own slot_o(PyLong_FromLongLong(slot));
    Own stamp_o(PyLong_FromLongLong(static_cast<int64_t>(lo)));
    Own ns(sid ? PyUnicode_FromFormat("/sessions/%U", sid.p) : nullptr);
    Own cfg(Py_BuildValue("(Ld)", static_cast<long long>(mp), ms));
    if (!sid || !slot_o || !stamp_o || !ns || !cfg) {
      s->release_row(store::RK_S, slot);
      return nullptr;
    }
    // DeviceSession
    PyObject* sd = nullptr;
    Own sso(new_view(C.DeviceSession, &sd));
    if (!sso) {
      s->release_row(store::RK_S, slot);
      return nullptr;
    }
    Own sdict(sd);
    Own zero(PyLong_FromLong(0)), minus1(PyLong_FromLong(-1)), hs(PyLong_FromLong(C.s_handshaking));
    if (!(zero && minus1 && hs && dset(sd, N._store, gs) && dset(sd, N.session_id, sid.p) &&
          dset(sd, N.creator_did, creator) && dset(sd, N.config, config) && dset(sd, N.vfs_namespace, ns.p) &&
          dset_steal(sd, N._vfs_snapshots, PyDict_New()) && dset(sd, N.slot, slot_o.p) &&
          dset(sd, N._cseq, minus1.p) && dset(sd, N._m_state, hs.p) && dset_steal(sd, N._m_rows, PyDict_New()) &&
          dset(sd, N._m_active, zero.p) && dset(sd, N._m_cfg, cfg.p) && dset(sd, N._stamp, stamp_o.p) &&
          dset(sd, N._poisoned, Py_None)))
      return nullptr;  // the view's __del__ releases the row
    // OP_SESS_CREATE, posted and verified later (status 0)
    const uint64_t a[10] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(aid), static_cast<uint64_t>(now),
                            static_cast<uint64_t>(mode_code), static_cast<uint64_t>(mp),
                            static_cast<uint64_t>(dbits(ms)), static_cast<uint64_t>(audit), hi, lo, 0};
    const uint64_t want0 = 0;
    Own tok(token(sso.p, C.err_create, (Py_INCREF(slot_o.p), slot_o.p)));
    if (!tok) return nullptr;
    s->post_expect_raw(store::OP_SESS_CREATE, a, 10, 1u, &want0, py::reinterpret_borrow<py::object>(tok.p));
    // DeviceDeltaEngine(store, slot, sid, owner=sso)
    PyObject* ed = nullptr;
    Own de(new_view(C.DeviceDeltaEngine, &ed));
    if (!de) return nullptr;
    Own edict(ed);
    if (!(dset(ed, N._store, gs) && dset(ed, N.slot, slot_o.p) && dset(ed, N.session_id, sid.p) &&
          dset(ed, N._owner, sso.p) && dset_steal(ed, N._deltas, PyList_New(0)) &&
          dset_steal(ed, N._rows, PyList_New(0)) && dset(ed, N._turn_counter, zero.p)))
      return nullptr;
    // DeviceSagaOrchestrator(store, sso, saga_reg)
    PyObject* od = nullptr;
    Own orch(new_view(C.DeviceSagaOrchestrator, &od));
    if (!orch) return nullptr;
    Own odict(od);
    if (!(dset(od, N._store, gs) && dset_steal(od, N._sagas, PyDict_New()) && dset(od, N._owner, sso.p) &&
          dset(od, N._reg, reg)))
      return nullptr;
    return PyTuple_Pack(3, sso.p, de.p, orch.p);
  });
}

// The session view's fields the join / activate fast paths read, and its store.
struct SessCtx {
  Own d;  // instance dict
  PyObject* gs = nullptr;
  Store* s = nullptr;
  StringPool* agents = nullptr;
  int64_t slot = 0, stamp = 0;
};

// false: not a plain device session of a live store (caller returns None).
bool sess_ctx(PyObject* sso, SessCtx& c) {
  if (Py_TYPE(sso) != reinterpret_cast<PyTypeObject*>(C.DeviceSession)) return false;
  c.d.p = idict(sso);
  if (!c.d) {
    PyErr_Clear();
    return false;
  }
  c.gs = dget(c.d.p, N._store);
  if (c.gs == nullptr) return false;
  c.s = store_of(c.gs, &c.agents);
  if (c.s == nullptr) return false;
  PyObject* so = dget(c.d.p, N.slot);
  PyObject* st = dget(c.d.p, N._stamp);
  PyObject* cs = dget(c.d.p, N._cseq);
  bool ok = so && st && cs;
  c.slot = ok ? as_i64(so, &ok) : 0;
  c.stamp = ok ? as_i64(st, &ok) : 0;
  const int64_t cseq = ok ? as_i64(cs, &ok) : 0;
  return ok && cseq < 0;  // a create still awaited (_created) takes the Python path
}

// The ring of a join the device will certainly admit, posted without waiting
// (DeviceSession._join_args + _join_speculated); None: outcome not known here —
// the caller awaits DeviceSession.join_gated_async.
PyObject* ctl_join(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 5) {
      PyErr_SetString(PyExc_TypeError, "ctl_join(sso, agent_did, sigma_raw, sigma_eff, trustworthy)");
      return nullptr;
    }
    SessCtx c;
    if (!sess_ctx(args[0], c)) Py_RETURN_NONE;
    if (!guard(c.gs, c.s, c.d.p)) return nullptr;
    PyObject* st = dget(c.d.p, N._m_state);
    PyObject* rows = dget(c.d.p, N._m_rows);
    PyObject* act = dget(c.d.p, N._m_active);
    PyObject* cfg = dget(c.d.p, N._m_cfg);
    if (st == nullptr || st == Py_None || rows == nullptr || !PyDict_CheckExact(rows) || act == nullptr ||
        cfg == nullptr || !PyTuple_CheckExact(cfg) || PyTuple_GET_SIZE(cfg) != 2)
      Py_RETURN_NONE;
    if (PyDict_GET_SIZE(rows) >= c.s->cap_participants()) Py_RETURN_NONE;
    const double sr = PyFloat_AsDouble(args[2]);
    if (sr == -1.0 && PyErr_Occurred()) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    const double se = PyFloat_AsDouble(args[3]);
    if (se == -1.0 && PyErr_Occurred()) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    const int trust = PyObject_IsTrue(args[4]);
    if (trust < 0) return nullptr;
    bool ok = true;
    const int64_t state = as_i64(st, &ok);
    const int64_t active = ok ? as_i64(act, &ok) : 0;
    const int64_t maxp = ok ? as_i64(PyTuple_GET_ITEM(cfg, 0), &ok) : 0;
    const double minsig = PyFloat_AsDouble(PyTuple_GET_ITEM(cfg, 1));
    if (!ok || PyErr_Occurred()) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    const int64_t aid = agent_id(c.agents, args[1]);
    if (aid < 0) Py_RETURN_NONE;
    Own aid_o(PyLong_FromLongLong(aid));
    if (!aid_o) return nullptr;
    const int dup = PyDict_Contains(rows, aid_o.p);
    if (dup < 0) return nullptr;
    int64_t now;
    if (!now_us(&now)) return nullptr;
    uint8_t ring = ring_from_sigma(se, false);
    if (!trust) ring = RING3;
    const uint8_t code = join_check(static_cast<uint8_t>(state), dup != 0, static_cast<int>(active),
                                    static_cast<int>(maxp), se, minsig, ring);
    if (code) Py_RETURN_NONE;  // refusals take the awaited path (the device's own error)
    const uint64_t a[8] = {static_cast<uint64_t>(c.slot), static_cast<uint64_t>(aid),
                           static_cast<uint64_t>(dbits(sr)), static_cast<uint64_t>(dbits(se)),
                           static_cast<uint64_t>(trust ? 1 : 0), 0, static_cast<uint64_t>(now),
                           static_cast<uint64_t>(c.stamp)};
    const uint64_t want[2] = {0, ring};
    Own tok(token(args[0], C.err_join, PyLong_FromLongLong(c.slot)));
    if (!tok) return nullptr;
    c.s->post_expect_raw(store::OP_SESS_JOIN, a, 8, 3u, want, py::reinterpret_borrow<py::object>(tok.p));
    if (PyDict_SetItem(rows, aid_o.p, Py_True) < 0) return nullptr;
    if (!dset_steal(c.d.p, N._m_active, PyLong_FromLongLong(active + 1))) return nullptr;
    return PyLong_FromLong(ring);
  });
}

// True: the activation was known to succeed and is posted (verified later);
// False: the caller awaits DeviceSession.activate_async.
PyObject* ctl_activate(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 1) {
      PyErr_SetString(PyExc_TypeError, "ctl_activate(sso)");
      return nullptr;
    }
    SessCtx c;
    if (!sess_ctx(args[0], c)) Py_RETURN_FALSE;
    if (!guard(c.gs, c.s, c.d.p)) return nullptr;
    PyObject* st = dget(c.d.p, N._m_state);
    PyObject* rows = dget(c.d.p, N._m_rows);
    bool ok = st != nullptr && st != Py_None;
    const int64_t state = ok ? as_i64(st, &ok) : -1;
    if (!ok || state != C.s_handshaking || rows == nullptr || !PyDict_CheckExact(rows) || PyDict_GET_SIZE(rows) == 0)
      Py_RETURN_FALSE;
    const uint64_t a[2] = {static_cast<uint64_t>(c.slot), static_cast<uint64_t>(c.stamp)};
    const uint64_t want0 = 0;
    Own tok(token(args[0], C.err_activate, PyLong_FromLongLong(c.slot)));
    if (!tok) return nullptr;
    c.s->post_expect_raw(store::OP_SESS_ACTIVATE, a, 2, 1u, &want0, py::reinterpret_borrow<py::object>(tok.p));
    if (!dset_steal(c.d.p, N._m_state, PyLong_FromLong(C.s_active))) return nullptr;
    Py_RETURN_TRUE;
  });
}

// DeviceSession._guard() for any view that has an owner session (orchestrators).
PyObject* ctl_guard(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 1) {
      PyErr_SetString(PyExc_TypeError, "ctl_guard(sso)");
      return nullptr;
    }
    PyObject* sso = args[0];
    if (sso == Py_None) Py_RETURN_NONE;
    Own d(idict(sso));
    if (!d) return nullptr;
    PyObject* gs = dget(d.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    if (s == nullptr) {  // closed / foreign store: the Python guard raises what it raises
      Own r(PyObject_CallMethod(sso, "_guard", nullptr));
      if (!r) return nullptr;
      Py_RETURN_NONE;
    }
    if (!guard(gs, s, d.p)) return nullptr;
    Py_RETURN_NONE;
  });
}

// ------------------------------------------------------------------ sagas

// DeviceSagaOrchestrator.create_saga(self, session_id, saga_id=None)
PyObject* ctl_create_saga(PyObject*, PyObject* const* args, Py_ssize_t nargsf, PyObject* kwnames) {
  return guarded([&]() -> PyObject* {
    const Py_ssize_t n = PyVectorcall_NARGS(nargsf);
    PyObject* saga_id = Py_None;
    if (kwnames != nullptr) {
      if (n != 2 || PyTuple_GET_SIZE(kwnames) != 1 || PyUnicode_Compare(PyTuple_GET_ITEM(kwnames, 0), N.saga_id) != 0)
        return fallback(C.fb_create_saga, args, nargsf, kwnames);
      saga_id = args[2];
    } else if (n == 3) {
      saga_id = args[2];
    } else if (n != 2) {
      return fallback(C.fb_create_saga, args, nargsf, kwnames);
    }
    Own od(idict(args[0]));
    if (!od) return nullptr;
    PyObject* gs = dget(od.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* sagas = dget(od.p, N._sagas);
    PyObject* reg = dget(od.p, N._reg);
    if (s == nullptr || sagas == nullptr || !PyDict_CheckExact(sagas) || reg == nullptr)
      return fallback(C.fb_create_saga, args, nargsf, kwnames);
    int64_t now;
    if (!now_us(&now)) return nullptr;
    Own gid;
    const int truth = PyObject_IsTrue(saga_id);
    if (truth < 0) return nullptr;
    if (truth) {
      Py_INCREF(saga_id);
      gid.p = saga_id;
    } else {
      static const char kPrefix[] = "saga:";
      gid.p = mint_uuid4(kPrefix, sizeof kPrefix - 1, nullptr, nullptr);
      if (!gid) return nullptr;
    }
    const int64_t slot = s->alloc_row(store::RK_G);
    if (slot < 0) return fallback(C.fb_create_saga, args, nargsf, kwnames);  // grows the table
    Own slot_o(PyLong_FromLongLong(slot));
    PyObject* gd = nullptr;
    Own g(slot_o ? new_view(C.DeviceSaga, &gd) : nullptr);
    if (!g) {
      s->release_row(store::RK_G, slot);
      return nullptr;
    }
    Own gdict(gd);
    if (!(dset(gd, N._store, gs) && dset(gd, N.slot, slot_o.p) && dset(gd, N.saga_id, gid.p) &&
          dset(gd, N.session_id, args[1]) && dset_steal(gd, N.steps, PyList_New(0)) && dset(gd, N.error, Py_None)))
      return nullptr;
    const uint64_t a[2] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(now)};
    s->post_raw(store::OP_SAGA_CREATE, a, 2, nullptr, 0);
    if (PyDict_SetItem(sagas, gid.p, g.p) < 0) return nullptr;
    if (reg != Py_None) {
      Own r(PyObject_CallMethodOneArg(reg, N.append, slot_o.p));
      if (!r) return nullptr;
    }
    return g.release();
  });
}

// DeviceSagaOrchestrator.add_step(self, saga_id, action_id, agent_did, execute_api,
//                                 undo_api=None, timeout_seconds=300, max_retries=0)
PyObject* ctl_add_step(PyObject*, PyObject* const* args, Py_ssize_t nargsf, PyObject* kwnames) {
  return guarded([&]() -> PyObject* {
    const Py_ssize_t n = PyVectorcall_NARGS(nargsf);
    PyObject* const* kwnames_order[3] = {&N.undo_api, &N.timeout_seconds, &N.max_retries};
    PyObject* v[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, Py_None, nullptr, nullptr};
    if (n < 5 || n > 8) return fallback(C.fb_add_step, args, nargsf, kwnames);
    for (Py_ssize_t k = 0; k < n; ++k) v[k] = args[k];
    if (kwnames != nullptr) {
      for (Py_ssize_t k = 0; k < PyTuple_GET_SIZE(kwnames); ++k) {
        PyObject* kw = PyTuple_GET_ITEM(kwnames, k);
        int at = -1;
        for (int j = 0; j < 3; ++j)
          if (PyUnicode_Compare(kw, *kwnames_order[j]) == 0) at = 5 + j;
        if (at < 0 || at < n || v[at] != (at == 5 ? Py_None : nullptr)) {
          if (PyErr_Occurred()) PyErr_Clear();
          return fallback(C.fb_add_step, args, nargsf, kwnames);
        }
        v[at] = args[n + k];
      }
    }
    Own timeout_default, retries_default;
    if (v[6] == nullptr) {
      timeout_default.p = PyLong_FromLong(300);
      v[6] = timeout_default.p;
    }
    if (v[7] == nullptr) {
      retries_default.p = PyLong_FromLong(0);
      v[7] = retries_default.p;
    }
    if (v[6] == nullptr || v[7] == nullptr) return nullptr;
    Own od(idict(v[0]));
    if (!od) return nullptr;
    PyObject* gs = dget(od.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* sagas = dget(od.p, N._sagas);
    PyObject* saga = (sagas != nullptr && PyDict_CheckExact(sagas)) ? dget(sagas, v[1]) : nullptr;
    if (PyErr_Occurred()) return nullptr;
    if (s == nullptr || saga == nullptr) return fallback(C.fb_add_step, args, nargsf, kwnames);
    Own gd(idict(saga));
    if (!gd) return nullptr;
    PyObject* gslot_o = dget(gd.p, N.slot);
    PyObject* steps = dget(gd.p, N.steps);
    bool ok = gslot_o != nullptr && steps != nullptr && PyList_CheckExact(steps);
    const int64_t gslot = ok ? as_i64(gslot_o, &ok) : 0;
    const int64_t retries = ok ? as_i64(v[7], &ok) : 0;
    const int undo = PyObject_IsTrue(v[5]);
    if (undo < 0) return nullptr;
    if (!ok) return fallback(C.fb_add_step, args, nargsf, kwnames);
    const int64_t slot = s->alloc_row(store::RK_T);
    if (slot < 0) return fallback(C.fb_add_step, args, nargsf, kwnames);  // grows the table
    Own slot_o(PyLong_FromLongLong(slot));
    static const char kPrefix[] = "step:";
    Own stid(slot_o ? mint_uuid4(kPrefix, sizeof kPrefix - 1, nullptr, nullptr) : nullptr);
    PyObject* xd = nullptr;
    Own x(stid ? new_view(C.DeviceSagaStep, &xd) : nullptr);
    if (!x) {
      s->release_row(store::RK_T, slot);
      return nullptr;
    }
    Own xdict(xd);
    if (!(dset(xd, N._store, gs) && dset(xd, N.slot, slot_o.p) && dset(xd, N.execute_result, Py_None) &&
          dset(xd, N.compensation_result, Py_None) && dset(xd, N.error, Py_None) && dset(xd, N.step_id, stid.p) &&
          dset(xd, N.action_id, v[2]) && dset(xd, N.agent_did, v[3]) && dset(xd, N.execute_api, v[4]) &&
          dset(xd, N.undo_api, v[5]) && dset(xd, N.timeout_seconds, v[6]) && dset(xd, N.max_retries, v[7])))
      return nullptr;
    const uint64_t a[4] = {static_cast<uint64_t>(gslot), static_cast<uint64_t>(slot),
                           static_cast<uint64_t>(undo ? 1 : 0), static_cast<uint64_t>(retries)};
    s->post_raw(store::OP_STEP_ADD, a, 4, nullptr, 0);
    if (!dset(xd, N._hint, C.step_pending)) return nullptr;
    if (PyList_Append(steps, x.p) < 0) return nullptr;
    return x.release();
  });
}

// DeviceSagaStep: the EXECUTING transition posted without waiting when this
// process knows the step's state allows it (can_speculate + post_transition);
// returns its sequence number, or None (the caller awaits transition_async).
PyObject* ctl_step_begin(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 2) {
      PyErr_SetString(PyExc_TypeError, "ctl_step_begin(step, attempt)");
      return nullptr;
    }
    if (!C.step_speculate) Py_RETURN_NONE;
    Own xd(idict(args[0]));
    if (!xd) return nullptr;
    PyObject* hint = dget(xd.p, N._hint);
    if (hint == nullptr || hint == Py_None) Py_RETURN_NONE;
    const int allowed = PySet_Contains(C.exec_from, hint);
    if (allowed < 0) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    if (!allowed) Py_RETURN_NONE;
    PyObject* gs = dget(xd.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* so = dget(xd.p, N.slot);
    bool ok = s != nullptr && so != nullptr;
    const int64_t slot = ok ? as_i64(so, &ok) : 0;
    const int64_t retry = ok ? as_i64(args[1], &ok) : 0;
    if (!ok) Py_RETURN_NONE;
    int64_t now;
    if (!now_us(&now)) return nullptr;
    if (!dset(xd.p, N._hint, Py_None)) return nullptr;
    const uint64_t a[4] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(C.step_executing_idx),
                           static_cast<uint64_t>(now), static_cast<uint64_t>(retry)};
    const uint64_t q = s->post_raw(store::OP_STEP_TRANSITION, a, 4, nullptr, 0);
    s->keep(q);
    return PyLong_FromUnsignedLongLong(q);
  });
}

// The executor returned: the posted EXECUTING transition is verified later and
// COMMITTED is posted the same way (both speculations owned by the session).
PyObject* ctl_step_commit(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 3) {
      PyErr_SetString(PyExc_TypeError, "ctl_step_commit(owner, step, seq)");
      return nullptr;
    }
    PyObject* owner = args[0];
    Own xd(idict(args[1]));
    if (!xd) return nullptr;
    PyObject* gs = dget(xd.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* so = dget(xd.p, N.slot);
    bool ok = s != nullptr && so != nullptr;
    const int64_t slot = ok ? as_i64(so, &ok) : 0;
    const int64_t seq = ok ? as_i64(args[2], &ok) : 0;
    if (!ok) {
      PyErr_SetString(PyExc_RuntimeError, "ctl_step_commit: not a live device step");
      return nullptr;
    }
    int64_t now;
    if (!now_us(&now)) return nullptr;
    const uint64_t want0 = 0;
    Own t1(token(owner, C.err_transition, Py_BuildValue("(LO)", static_cast<long long>(slot), C.step_executing)));
    if (!t1) return nullptr;
    s->expect_mask(static_cast<uint64_t>(seq), 1u, &want0, py::reinterpret_borrow<py::object>(t1.p));
    Own t2(token(owner, C.err_transition, Py_BuildValue("(LO)", static_cast<long long>(slot), C.step_committed)));
    if (!t2) return nullptr;
    const uint64_t a[4] = {static_cast<uint64_t>(slot), static_cast<uint64_t>(C.step_committed_idx),
                           static_cast<uint64_t>(now), ~0ull};
    s->post_expect_raw(store::OP_STEP_TRANSITION, a, 4, 1u, &want0, py::reinterpret_borrow<py::object>(t2.p));
    if (!dset(xd.p, N._hint, C.step_committed)) return nullptr;
    Py_RETURN_NONE;
  });
}

// ------------------------------------------------------------------ terminate

// The awaited device terminate up to its post (Hypervisor._terminate_device's
// "early" path): guard, GC cutoff, the chain's delta rows, the host's prediction
// of the root and of the GC count (close_prediction), then OP_SESS_CLOSE.
// Returns (seq, predicted root or None, predicted expired count, n deltas), or
// None when the Python path must decide (liability rows, no prediction,
// speculated terminates, a poisoned session) — nothing is changed then.
PyObject* ctl_close(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 4) {
      PyErr_SetString(PyExc_TypeError, "ctl_close(hv, session_id, sso, delta_engine)");
      return nullptr;
    }
    PyObject* hv = args[0];
    PyObject* sid = args[1];
    if (C.spec_terminate || !C.check_terminate) Py_RETURN_NONE;
    SessCtx c;
    if (Py_TYPE(args[3]) != reinterpret_cast<PyTypeObject*>(C.DeviceDeltaEngine)) Py_RETURN_NONE;
    if (Py_TYPE(args[2]) != reinterpret_cast<PyTypeObject*>(C.DeviceSession)) Py_RETURN_NONE;
    c.d.p = idict(args[2]);
    if (!c.d) return nullptr;
    c.gs = dget(c.d.p, N._store);
    c.s = c.gs ? store_of(c.gs) : nullptr;
    PyObject* so = dget(c.d.p, N.slot);
    bool ok = c.s != nullptr && so != nullptr;
    c.slot = ok ? as_i64(so, &ok) : 0;
    if (!ok) Py_RETURN_NONE;
    if (!guard(c.gs, c.s, c.d.p)) return nullptr;
    // liability row of (tenant, session): awaited release path in Python
    Own hd(idict(hv));
    Own gd(idict(c.gs));
    if (!hd || !gd) return nullptr;
    PyObject* tenant = dget(hd.p, N._tenant);
    PyObject* tv = dget(gd.p, N._tenant_v);
    if (tenant == nullptr || tv == nullptr || !PyDict_CheckExact(tv)) Py_RETURN_NONE;
    PyObject* per = dget(tv, tenant);
    if (PyErr_Occurred()) return nullptr;
    if (per != nullptr) {
      if (!PyDict_CheckExact(per)) Py_RETURN_NONE;
      const int has = PyDict_Contains(per, sid);
      if (has < 0) return nullptr;
      if (has) Py_RETURN_NONE;
    }
    // the prediction (close_prediction(..., check=True))
    PyObject* pois = dget(c.d.p, N._poisoned);
    PyObject* mst = dget(c.d.p, N._m_state);
    if (pois == nullptr || pois != Py_None || mst == nullptr || mst == Py_None) Py_RETURN_NONE;
    const int64_t state = as_i64(mst, &ok);
    if (!ok || (state != C.s_active && state != C.s_handshaking)) Py_RETURN_NONE;
    Own ed(idict(args[3]));
    if (!ed) return nullptr;
    PyObject* ds = dget(ed.p, N._deltas);
    PyObject* tc = dget(ed.p, N._turn_counter);
    if (ds == nullptr || !PyList_CheckExact(ds) || tc == nullptr) Py_RETURN_NONE;
    const Py_ssize_t n = PyList_GET_SIZE(ds);
    if (as_i64(tc, &ok) != n || !ok) Py_RETURN_NONE;
    Own cfg(PyObject_GetAttr(args[2], N.config));
    if (!cfg) return nullptr;
    Own aud(PyObject_GetAttr(cfg.p, N.enable_audit));
    if (!aud) return nullptr;
    const int audit = PyObject_IsTrue(aud.p);
    if (audit < 0) return nullptr;
    // GC cutoff: now - int(retention_days * 86_400_000_000)
    Own g(PyObject_GetAttr(hv, N.gc));
    Own pol(g ? PyObject_GetAttr(g.p, N.policy) : nullptr);
    Own days(pol ? PyObject_GetAttr(pol.p, N.delta_retention_days) : nullptr);
    if (!days) return nullptr;
    Own scale(PyLong_FromLongLong(86400000000LL));
    Own prod(scale ? PyNumber_Multiply(days.p, scale.p) : nullptr);
    Own span(prod ? PyNumber_Long(prod.p) : nullptr);
    if (!span) return nullptr;
    const int64_t keep_us = as_i64(span.p, &ok);
    if (!ok) Py_RETURN_NONE;
    int64_t now;
    if (!now_us(&now)) return nullptr;
    const int64_t cutoff = now - keep_us;
    std::vector<int32_t> idx(static_cast<size_t>(n));
    py::list preds(n);
    int64_t expired = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      Own dd(idict(PyList_GET_ITEM(ds, i)));
      if (!dd) return nullptr;
      PyObject* di = dget(dd.p, N._didx);
      PyObject* pr = dget(dd.p, N._pred);
      PyObject* tsu = dget(dd.p, N._tsu);
      if (di == nullptr || pr == nullptr || pr == Py_None || tsu == nullptr) Py_RETURN_NONE;
      const int64_t dix = as_i64(di, &ok);
      const int64_t t = ok ? as_i64(tsu, &ok) : 0;
      if (!ok || dix < INT32_MIN || dix > INT32_MAX) Py_RETURN_NONE;
      idx[static_cast<size_t>(i)] = static_cast<int32_t>(dix);
      if (t < cutoff) ++expired;
      Py_INCREF(pr);
      PyList_SET_ITEM(preds.ptr(), i, pr);
    }
    py::object root = py::none();
    if (audit && n) {
      root = Store::merkle_predict(preds);
      if (root.is_none()) Py_RETURN_NONE;
    }
    // committed from here on: the row leaves the mirrored states
    if (!dset(c.d.p, N._m_state, Py_None) || !dset(c.d.p, N._m_rows, Py_None)) return nullptr;
    int64_t off = 0;
    const uint8_t* inl = nullptr;
    size_t inl_bytes = 0;
    if (n <= 96) {
      inl = reinterpret_cast<const uint8_t*>(idx.data());
      inl_bytes = 4 * static_cast<size_t>(n);
    } else {
      off = c.s->stage_raw(reinterpret_cast<const uint8_t*>(idx.data()), 4 * static_cast<size_t>(n));
    }
    const uint64_t a[7] = {static_cast<uint64_t>(c.slot), static_cast<uint64_t>(n), static_cast<uint64_t>(off),
                           static_cast<uint64_t>(now), ~0ull /* v = -1 */, static_cast<uint64_t>(cutoff),
                           static_cast<uint64_t>(audit ? 1 : 0)};
    const uint64_t q = c.s->post_raw(store::OP_SESS_CLOSE, a, 7, inl, inl_bytes);
    return Py_BuildValue("(KOLn)", static_cast<unsigned long long>(q), root.ptr(), static_cast<long long>(expired), n);
  });
}

// Hypervisor._terminate_checked for an answer that agrees with the prediction:
// verify the session's speculations, take the device's root, register the
// commitment; anything else (a device error, a divergence, an event bus to
// publish to) goes to the Python implementation, which raises or publishes.
PyObject* ctl_close_finish(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 5) {
      PyErr_SetString(PyExc_TypeError, "ctl_close_finish(hv, session_id, sso, r, check)");
      return nullptr;
    }
    PyObject* hv = args[0];
    PyObject* sid = args[1];
    PyObject* sso = args[2];
    PyObject* r = args[3];
    PyObject* check = args[4];
    auto slow = [&]() -> PyObject* {
      return PyObject_CallMethod(hv, "_terminate_checked", "OOOO", sid, sso, r, check);
    };
    if (!PyTuple_CheckExact(r) || PyTuple_GET_SIZE(r) < 12 || !PyTuple_CheckExact(check) ||
        PyTuple_GET_SIZE(check) != 2)
      return slow();
    Own hd(idict(hv));
    Own sd(idict(sso));
    if (!hd || !sd) return nullptr;
    PyObject* bus = dget(hd.p, N.event_bus);
    PyObject* gs = dget(sd.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    if (s == nullptr || (bus != nullptr && bus != Py_None)) return slow();
    bool ok = true;
    const int64_t status = as_i64(PyTuple_GET_ITEM(r, 0), &ok);
    const int64_t has_root = ok ? as_i64(PyTuple_GET_ITEM(r, 1), &ok) : 0;
    const int64_t gc_n = ok ? as_i64(PyTuple_GET_ITEM(r, 11), &ok) : 0;
    const int64_t want_gc = ok ? as_i64(PyTuple_GET_ITEM(check, 1), &ok) : 0;
    if (!ok || status != 0 || gc_n != want_gc) return slow();
    if (!guard(gs, s, sd.p)) return nullptr;  // every post before the close has completed
    Own root;
    if (has_root) {
      root.p = PyUnicode_New(64, 127);
      if (!root) return nullptr;
      uint32_t w[8];
      for (int k = 0; k < 8; ++k) {
        const int64_t v = as_i64(PyTuple_GET_ITEM(r, 2 + k), &ok);
        w[k] = static_cast<uint32_t>(v);
        if (!ok || v < 0 || v > 0xffffffffLL) return slow();
      }
      host::hex_bytes(w, PyUnicode_1BYTE_DATA(root.p));
    } else {
      Py_INCREF(Py_None);
      root.p = Py_None;
    }
    Own cfg(PyObject_GetAttr(sso, N.config));
    Own aud(cfg ? PyObject_GetAttr(cfg.p, N.enable_audit) : nullptr);
    if (!aud) return nullptr;
    const int audit = PyObject_IsTrue(aud.p);
    if (audit < 0) return nullptr;
    if (audit) {
      const int same = PyObject_RichCompareBool(PyTuple_GET_ITEM(check, 0), root.p, Py_EQ);
      if (same < 0) return nullptr;
      if (!same) return slow();  // divergence: the Python path poisons the session and raises
    }
    if (root.p != Py_None && dget(hd.p, N.commitment) == nullptr) {
      // no commitment engine yet (most hypervisors never read one): the committed
      // session waits in `_commits`, which the engine absorbs when it is built
      if (PyErr_Occurred()) return nullptr;
      PyObject* pend = dget(hd.p, N._commits);
      if (pend == nullptr) {
        if (PyErr_Occurred()) return nullptr;
        if (!dset_steal(hd.p, N._commits, PyDict_New())) return nullptr;
        pend = dget(hd.p, N._commits);
      }
      if (pend == nullptr || PyDict_SetItem(pend, sid, sso) < 0) return nullptr;
    } else if (root.p != Py_None) {
      Own cm(PyObject_GetAttr(hv, N.commitment));
      if (!cm) return nullptr;
      if (Py_TYPE(cm.p) == reinterpret_cast<PyTypeObject*>(C.DeviceCommitmentEngine)) {
        Own cd(idict(cm.p));
        if (!cd) return nullptr;
        PyObject* dev = dget(cd.p, N._device);
        if (dev == nullptr || !PyDict_CheckExact(dev) || PyDict_SetItem(dev, sid, sso) < 0) {
          if (PyErr_Occurred()) return nullptr;
          Own rr(PyObject_CallMethod(cm.p, "register", "O", sso));
          if (!rr) return nullptr;
        }
      } else {
        Own rr(PyObject_CallMethod(cm.p, "register", "O", sso));
        if (!rr) return nullptr;
      }
    }
    return root.release();
  });
}

// ------------------------------------------------------------------ teardown

// close_hypervisor(hv) for a hypervisor whose sessions were all created one by
// one (no batch segments) and whose vouching engine was never built: every row
// of its views back to the store in one native pass; -1 → the Python path.
PyObject* ctl_close_hypervisor(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  return guarded([&]() -> PyObject* {
    if (PyVectorcall_NARGS(nargsf) != 1) {
      PyErr_SetString(PyExc_TypeError, "ctl_close_hypervisor(hv)");
      return nullptr;
    }
    PyObject* hv = args[0];
    Own hd(idict(hv));
    if (!hd) return nullptr;
    PyObject* gs = dget(hd.p, N._store);
    Store* s = gs ? store_of(gs) : nullptr;
    PyObject* tab = dget(hd.p, N._sessions);
    PyObject* tenant = dget(hd.p, N._tenant);
    PyObject* ve = dget(hd.p, N.vouching);
    if (s == nullptr || tab == nullptr || tenant == nullptr || ve != nullptr || PyErr_Occurred())
      return PyLong_FromLong(-1);
    {
      Own gsd(idict(gs));
      if (!gsd) return nullptr;
      PyObject* cl = dget(gsd.p, N._closed);
      if (cl != nullptr && cl != Py_False) return PyLong_FromLong(-1);  // a closed store: Python returns 0
    }
    Own segs(PyObject_GetAttr(tab, N._segs));
    Own own(segs ? PyObject_GetAttr(tab, N._own) : nullptr);
    if (!own) return nullptr;
    if (!PyList_CheckExact(segs.p) || !PyDict_CheckExact(own.p)) return PyLong_FromLong(-1);
    const Py_ssize_t ns = PyList_GET_SIZE(segs.p);
    for (Py_ssize_t i = 0; i < ns; ++i)
      if (!PyList_CheckExact(PyList_GET_ITEM(segs.p, i))) return PyLong_FromLong(-1);  // batches: Python
    std::vector<int64_t> rows[4];  // S, D, G, T
    auto slot_of = [&](PyObject* d, int64_t* out) {
      PyObject* so = dget(d, N.slot);
      bool ok = so != nullptr;
      *out = ok ? as_i64(so, &ok) : 0;
      return ok;
    };
    long count = 0;
    for (Py_ssize_t i = 0; i < ns; ++i) {
      PyObject* seg = PyList_GET_ITEM(segs.p, i);
      for (Py_ssize_t k = 0; k < PyList_GET_SIZE(seg); ++k) {
        PyObject* m = dget(own.p, PyList_GET_ITEM(seg, k));
        if (m == nullptr) {
          if (PyErr_Occurred()) return nullptr;
          continue;
        }
        ++count;
        Own sso(PyObject_GetAttr(m, N.sso));
        Own de(sso ? PyObject_GetAttr(m, N.delta_engine) : nullptr);
        Own orch(de ? PyObject_GetAttr(m, N.saga) : nullptr);
        if (!orch) return nullptr;
        // the session view
        {
          Own sd(idict(sso.p));
          if (!sd) {
            PyErr_Clear();
          } else if (dget(sd.p, N._store) == gs) {
            int64_t r;
            if (slot_of(sd.p, &r)) rows[0].push_back(r);
            if (PyObject_SetAttr(sso.p, N._store, C.CLOSED) < 0) return nullptr;
          }
        }
        // the delta chain
        if (PyObject_TypeCheck(de.p, reinterpret_cast<PyTypeObject*>(C.DeviceDeltaEngine))) {
          Own edd(idict(de.p));
          if (!edd) return nullptr;
          if (dget(edd.p, N._store) == gs) {
            PyObject* rl = dget(edd.p, N._rows);
            if (rl != nullptr && PyList_CheckExact(rl)) {
              bool ok = true;
              for (Py_ssize_t j = 0; j < PyList_GET_SIZE(rl); ++j) {
                const int64_t r = as_i64(PyList_GET_ITEM(rl, j), &ok);
                if (ok) rows[1].push_back(r);
              }
            }
            if (!dset_steal(edd.p, N._rows, PyList_New(0))) return nullptr;
            if (PyObject_SetAttr(de.p, N._store, C.CLOSED) < 0) return nullptr;
          }
          PyObject* dl = dget(edd.p, N._deltas);
          if (dl != nullptr && PyList_CheckExact(dl)) {
            for (Py_ssize_t j = 0; j < PyList_GET_SIZE(dl); ++j) {
              Own xd(idict(PyList_GET_ITEM(dl, j)));
              if (!xd || !dset(xd.p, N._store, C.CLOSED)) return nullptr;
            }
          }
        }
        // sagas and their steps
        if (PyObject_TypeCheck(orch.p, reinterpret_cast<PyTypeObject*>(C.DeviceSagaOrchestrator))) {
          Own odd(idict(orch.p));
          if (!odd) return nullptr;
          PyObject* sg = dget(odd.p, N._sagas);
          if (sg != nullptr && PyDict_CheckExact(sg)) {
            Py_ssize_t pos = 0;
            PyObject *key, *g;
            while (PyDict_Next(sg, &pos, &key, &g)) {
              Own gdd(idict(g));
              if (!gdd) return nullptr;
              if (dget(gdd.p, N._store) == gs) {
                int64_t r;
                if (slot_of(gdd.p, &r)) rows[2].push_back(r);
                if (!dset(gdd.p, N._store, C.CLOSED)) return nullptr;
              }
              PyObject* st = dget(gdd.p, N.steps);
              if (st != nullptr && PyList_CheckExact(st)) {
                for (Py_ssize_t j = 0; j < PyList_GET_SIZE(st); ++j) {
                  Own xdd(idict(PyList_GET_ITEM(st, j)));
                  if (!xdd) return nullptr;
                  if (dget(xdd.p, N._store) == gs) {
                    int64_t r;
                    if (slot_of(xdd.p, &r)) rows[3].push_back(r);
                    if (!dset(xdd.p, N._store, C.CLOSED)) return nullptr;
                  }
                }
              }
            }
          }
          if (PyObject_SetAttr(orch.p, N._store, C.CLOSED) < 0) return nullptr;
        }
      }
    }
    static const uint64_t kinds[4] = {store::RK_S, store::RK_D, store::RK_G, store::RK_T};
    for (int k = 0; k < 4; ++k)
      for (int64_t r : rows[k]) s->release_row(kinds[k], r);
    // the hypervisor's liability-session rows (release_tenant with no edges)
    Own gd(idict(gs));
    if (!gd) return nullptr;
    PyObject* tv = dget(gd.p, N._tenant_v);
    if (tv != nullptr && PyDict_CheckExact(tv)) {
      PyObject* vs = dget(tv, tenant);
      if (vs != nullptr) {
        Py_INCREF(vs);
        Own vref(vs);
        if (PyDict_DelItem(tv, tenant) < 0) return nullptr;
        if (PyDict_CheckExact(vs)) {
          Py_ssize_t pos = 0;
          PyObject *key, *val;
          bool ok = true;
          while (PyDict_Next(vs, &pos, &key, &val)) {
            const int64_t r = as_i64(val, &ok);
            if (ok) s->release_row(store::RK_V, r);
          }
        }
      }
    }
    PyObject* cm = dget(hd.p, N.commitment);
    if (cm != nullptr && PyObject_TypeCheck(cm, reinterpret_cast<PyTypeObject*>(C.DeviceCommitmentEngine))) {
      if (PyObject_SetAttr(cm, N._store, C.CLOSED) < 0) return nullptr;
    }
    if (PyObject_SetAttr(hv, N._store, C.CLOSED) < 0) return nullptr;
    return PyLong_FromLong(count);
  });
}

// ------------------------------------------------------------------ finalisers

// `__del__` of the device views (DeviceSession / DeviceDeltaEngine / DeviceSaga /
// DeviceSagaStep): detach the view (its store becomes CLOSED) and queue its row(s)
// for reclaim — a view the hypervisor's close already detached does nothing.
// Finalisers never raise (the Python versions swallow every error).
PyObject* ctl_view_del(PyObject*, PyObject* self) {
  PyObject* type = reinterpret_cast<PyObject*>(Py_TYPE(self));
  uint64_t kind;
  const bool engine = type == C.DeviceDeltaEngine;
  if (type == C.DeviceSession) kind = store::RK_S;
  else if (type == C.DeviceSaga) kind = store::RK_G;
  else if (type == C.DeviceSagaStep) kind = store::RK_T;
  else if (engine) kind = store::RK_D;
  else Py_RETURN_NONE;
  Own d(idict(self));
  if (!d) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
  PyObject* st = dget(d.p, N._store);
  if (st == nullptr || st == C.CLOSED) {
    PyErr_Clear();
    if (st == nullptr) Py_RETURN_NONE;
    if (!engine) Py_RETURN_NONE;
  }
  Py_INCREF(st);
  Own st_ref(st);
  if (PyDict_SetItem(d.p, N._store, C.CLOSED) < 0) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
  Store* s = store_of(st);
  if (engine) {
    PyObject* rows = dget(d.p, N._rows);
    if (rows == nullptr) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    Py_INCREF(rows);
    Own rows_ref(rows);
    Own empty(PyList_New(0));
    if (!empty || PyDict_SetItem(d.p, N._rows, empty.p) < 0) {
      PyErr_Clear();
      Py_RETURN_NONE;
    }
    if (st == C.CLOSED || !PyList_CheckExact(rows) || PyList_GET_SIZE(rows) == 0) Py_RETURN_NONE;
    if (s != nullptr) {
      bool ok = true;
      for (Py_ssize_t i = 0; i < PyList_GET_SIZE(rows); ++i) {
        const int64_t r = as_i64(PyList_GET_ITEM(rows, i), &ok);
        if (ok) s->release_row(kind, r);
        ok = true;
      }
    } else {  // some other store object: its own release_many
      Own r(PyObject_CallMethod(st, "release_many", "sO", "D", rows));
      PyErr_Clear();
    }
    Py_RETURN_NONE;
  }
  PyObject* so = dget(d.p, N.slot);
  bool ok = so != nullptr;
  const int64_t slot = ok ? as_i64(so, &ok) : 0;
  if (s != nullptr && ok) {
    try {
      s->release_row(kind, slot);
    } catch (...) {
    }
  } else if (so != nullptr) {
    static const char* kinds = "SGTEDV";
    const char k[2] = {kinds[kind], 0};
    Own r(PyObject_CallMethod(st, "release", "sO", k, so));
    PyErr_Clear();
  }
  PyErr_Clear();
  Py_RETURN_NONE;
}

// Hypervisor.__del__: close a device-backed hypervisor (native close when it can).
PyObject* ctl_hv_del(PyObject*, PyObject* hv) {
  Own d(idict(hv));
  if (!d) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
  PyObject* st = dget(d.p, N._store);
  if (st == nullptr || st == Py_None || st == C.CLOSED) {
    PyErr_Clear();
    Py_RETURN_NONE;
  }
  PyObject* args[1] = {hv};
  Own n(C.ready ? PyObject_Vectorcall(C.close_hv_fast, args, 1, nullptr) : nullptr);
  bool done = false;
  if (n) {
    const long v = PyLong_AsLong(n.p);
    done = v >= 0;
  }
  PyErr_Clear();
  if (!done) {
    Own r(PyObject_CallMethod(hv, "close", nullptr));
    PyErr_Clear();
  }
  Py_RETURN_NONE;
}

// ------------------------------------------------------------------ setup

PyObject* ctl_init(PyObject*, PyObject* const* args, Py_ssize_t nargsf) {
  if (PyVectorcall_NARGS(nargsf) != 1 || !PyDict_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "ctl_init(dict)");
    return nullptr;
  }
  PyObject* d = args[0];
  if (!PyDateTimeAPI) PyDateTime_IMPORT;
  if (!PyDateTimeAPI) return nullptr;
  if (N._store == nullptr) N.init();
  auto get = [&](const char* k, PyObject** slot) {
    PyObject* v = PyDict_GetItemString(d, k);
    if (v == nullptr) {
      PyErr_Format(PyExc_KeyError, "ctl_init: missing %s", k);
      return false;
    }
    Py_INCREF(v);
    Py_XSETREF(*slot, v);
    return true;
  };
  auto get_int = [&](const char* k, int* out) {
    PyObject* v = PyDict_GetItemString(d, k);
    if (v == nullptr) {
      PyErr_Format(PyExc_KeyError, "ctl_init: missing %s", k);
      return false;
    }
    *out = static_cast<int>(PyLong_AsLong(v));
    return !PyErr_Occurred();
  };
  auto get_bool = [&](const char* k, bool* out) {
    PyObject* v = PyDict_GetItemString(d, k);
    if (v == nullptr) {
      PyErr_Format(PyExc_KeyError, "ctl_init: missing %s", k);
      return false;
    }
    *out = PyObject_IsTrue(v) == 1;
    return true;
  };
  if (!(get("GovernanceStore", &C.GovernanceStore) && get("DeviceSession", &C.DeviceSession) &&
        get("DeviceDelta", &C.DeviceDelta) && get("DeviceDeltaEngine", &C.DeviceDeltaEngine) &&
        get("DeviceSagaOrchestrator", &C.DeviceSagaOrchestrator) && get("DeviceSaga", &C.DeviceSaga) &&
        get("DeviceSagaStep", &C.DeviceSagaStep) && get("DeviceCommitmentEngine", &C.DeviceCommitmentEngine) &&
        get("CLOSED", &C.CLOSED) && get("clock_dict", &C.clock_dict) && get("now", &C.py_now) &&
        get("to_us", &C.py_to_us) && get("mode_eventual", &C.mode_eventual) && get("mode_strong", &C.mode_strong) &&
        get("step_pending", &C.step_pending) && get("step_executing", &C.step_executing) &&
        get("step_committed", &C.step_committed) && get("exec_from", &C.exec_from) &&
        get("err_create", &C.err_create) && get("err_join", &C.err_join) && get("err_activate", &C.err_activate) &&
        get("err_transition", &C.err_transition) && get("fb_capture", &C.fb_capture) &&
        get("fb_create_saga", &C.fb_create_saga) && get("fb_add_step", &C.fb_add_step) &&
        get_int("s_handshaking", &C.s_handshaking) && get_int("s_active", &C.s_active) &&
        get_int("step_executing_idx", &C.step_executing_idx) &&
        get_int("step_committed_idx", &C.step_committed_idx) && get_bool("spec_lifecycle", &C.spec_lifecycle) &&
        get_bool("step_speculate", &C.step_speculate) && get_bool("spec_terminate", &C.spec_terminate) &&
        get_bool("check_terminate", &C.check_terminate)))
    return nullptr;
  if (!PyAnySet_Check(C.exec_from)) {
    PyErr_SetString(PyExc_TypeError, "ctl_init: exec_from must be a set");
    return nullptr;
  }
  if (C.empty_tuple == nullptr) C.empty_tuple = PyTuple_New(0);
  if (!get("close_hv_fast", &C.close_hv_fast)) return nullptr;
  C.ready = true;
  Py_RETURN_NONE;
}

// A builtin bound as a method: PyInstanceMethod makes `obj.method(...)` pass obj first.
PyObject* ctl_method(PyObject*, PyObject* fn) { return PyInstanceMethod_New(fn); }

PyMethodDef kMethods[] = {
    {"ctl_init", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_init)), METH_FASTCALL,
     "Hand the native control plane the classes and settings of hypervisor._device"},
    {"ctl_method", ctl_method, METH_O, "Wrap a builtin so a class attribute binds it as a method"},
    {"ctl_capture", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_capture)),
     METH_FASTCALL | METH_KEYWORDS, "DeviceDeltaEngine.capture (native)"},
    {"ctl_session", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_session)), METH_FASTCALL,
     "(sso, delta engine, saga orchestrator) of a new device session, or None"},
    {"ctl_join", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_join)), METH_FASTCALL,
     "ring of a speculated join (posted), or None"},
    {"ctl_activate", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_activate)), METH_FASTCALL,
     "True when the activation was speculated and posted"},
    {"ctl_guard", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_guard)), METH_FASTCALL,
     "DeviceSession._guard (native)"},
    {"ctl_create_saga", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_create_saga)),
     METH_FASTCALL | METH_KEYWORDS, "DeviceSagaOrchestrator.create_saga (native)"},
    {"ctl_add_step", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_add_step)),
     METH_FASTCALL | METH_KEYWORDS, "DeviceSagaOrchestrator.add_step (native)"},
    {"ctl_step_begin", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_step_begin)), METH_FASTCALL,
     "posted EXECUTING transition's sequence number, or None"},
    {"ctl_step_commit", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_step_commit)), METH_FASTCALL,
     "verify EXECUTING later, post COMMITTED speculated"},
    {"ctl_close", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_close)), METH_FASTCALL,
     "awaited terminate up to its post: (seq, root, expired, n) or None"},
    {"ctl_close_finish", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_close_finish)),
     METH_FASTCALL, "the device's root of an awaited terminate that agrees with the prediction"},
    {"ctl_close_hypervisor", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)()>(ctl_close_hypervisor)),
     METH_FASTCALL, "close_hypervisor (native); -1: the Python path"},
    {"ctl_view_del", ctl_view_del, METH_O, "__del__ of the device views (native)"},
    {"ctl_hv_del", ctl_hv_del, METH_O, "Hypervisor.__del__ (native close)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

void register_control(py::module_& m) {
  for (PyMethodDef* d = kMethods; d->ml_name != nullptr; ++d) {
    PyObject* f = PyCFunction_NewEx(d, nullptr, m.ptr());
    if (f == nullptr) throw py::error_already_set();
    if (PyModule_AddObject(m.ptr(), d->ml_name, f) < 0) {
      Py_DECREF(f);
      throw py::error_already_set();
    }
  }
}

}  // namespace host
}  // namespace ahv
