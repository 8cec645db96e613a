// Host runtime pieces of the device engine:
//   * StringPool — the DID / path / id string interner: dense int32
//     ids for device tables, a reverse table, and each string's canonical-JSON
//     escaped body stored contiguously so kernels can splice it into the audit
//     payload without re-escaping (ahv/delta_emit.h StrPool).
//   * time base helpers (N09): epoch-µs ↔ ISO text with the exact
//     datetime.isoformat() rendering used in delta hashes.
#include <Python.h>
#include <longintrepr.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ahv/delta_emit.h"
#include "ahv/semantics.h"
#include "ahv/string_pool.h"

namespace py = pybind11;

namespace ahv {
namespace host {


static py::str iso_from_us(int64_t us) {
  uint8_t buf[40];
  const uint32_t n = iso_utc(us, buf);
  return py::str(reinterpret_cast<const char*>(buf), n);
}

static py::str uuid_str(uint64_t seed, uint64_t counter, const std::string& prefix) {
  uint32_t u[4];
  uuid4_words(seed, counter, u);
  std::string s = prefix;
  for (int k = 0; k < 32; ++k) {
    if (k == 8 || k == 12 || k == 16 || k == 20) s.push_back('-');
    s.push_back(static_cast<char>(hex_nibble((u[k >> 3] >> (28 - 4 * (k & 7))) & 15u)));
  }
  return py::str(s);
}

// uuid_from_counter for n consecutive counters (the session ids a template batch
// minted on the device, formatted on demand for lazy registration).
static py::list uuids_from_counters(uint64_t seed, uint64_t base, int64_t n, const std::string& prefix) {
  if (n < 0) throw py::value_error("n must be >= 0");
  py::list out(n);
  const size_t pl = prefix.size();
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u[4];
    uuid4_words(seed, base + static_cast<uint64_t>(i), u);
    PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + 36), 127);
    if (!s) throw py::error_already_set();
    char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
    std::memcpy(o, prefix.data(), pl);
    o += pl;
    for (int k = 0, j = 0; k < 32; ++k) {
      if (k == 8 || k == 12 || k == 16 || k == 20) o[j++] = '-';
      o[j++] = static_cast<char>(hex_nibble((u[k >> 3] >> (28 - 4 * (k & 7))) & 15u));
    }
    PyList_SET_ITEM(out.ptr(), static_cast<Py_ssize_t>(i), s);
  }
  return out;
}

// ------------------------------------------------------------------ spec packing
// Hypervisor.run_pipelines with one PipelineSpec per session: flatten the specs
// into the batch kernels' columns natively (models/store_pipeline.py documents
// the columns).  Strings go through the two pools (agents: DIDs of creators and
// joins; pool: every string a record renders); each distinct config object is
// read once (None: `cfg_of(None) -> (max_participants, min_sigma_eff,
// audit|strong flags)` of the default SessionConfig).  The turn-independent part of each delta's record-size
// bound is computed here from the pool's escaped lengths (+2 quotes, 4 = null).

static std::string utf8_of(const py::handle& o) {
  Py_ssize_t n = 0;
  const char* c = PyUnicode_AsUTF8AndSize(o.ptr(), &n);
  if (c != nullptr) return std::string(c, static_cast<size_t>(n));
  PyErr_Clear();  // lone surrogates: the pools hold their surrogatepass UTF-8
  py::bytes b = py::reinterpret_steal<py::bytes>(PyUnicode_AsEncodedString(o.ptr(), "utf-8", "surrogatepass"));
  if (!b) throw py::error_already_set();
  return std::string(b);
}

template <class T>
static py::bytes as_bytes(const std::vector<T>& v) {
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(T));
}

// Borrowed items of a list / tuple (any other sequence is converted once).
struct FastSeq {
  PyObject* o;    // a new reference when the argument had to be converted, else null
  PyObject** it;
  Py_ssize_t n;
  explicit FastSeq(PyObject* x) : o(nullptr) {
    if (PyTuple_CheckExact(x)) {  // the common case: items borrowed in place, no reference taken
      it = reinterpret_cast<PyTupleObject*>(x)->ob_item;
      n = PyTuple_GET_SIZE(x);
      return;
    }
    if (PyList_CheckExact(x)) {
      it = reinterpret_cast<PyListObject*>(x)->ob_item;
      n = PyList_GET_SIZE(x);
      return;
    }
    o = PySequence_Fast(x, "expected a sequence");
    if (o == nullptr) throw py::error_already_set();
    it = PySequence_Fast_ITEMS(o);
    n = PySequence_Fast_GET_SIZE(o);
  }
  ~FastSeq() { Py_XDECREF(o); }
  FastSeq(const FastSeq&) = delete;
  FastSeq& operator=(const FastSeq&) = delete;
  PyObject* operator[](Py_ssize_t i) const {
    if (i >= n) throw py::index_error("spec tuple too short");
    return it[i];
  }
};

// Pointer-keyed open-addressing table (no allocation per insert: batches of
// distinct spec / config objects insert one entry each).
template <class V>
struct PtrTable {
  std::vector<PyObject*> key;
  std::vector<V> val;
  size_t mask = 0, used = 0;
  explicit PtrTable(size_t want) {
    size_t c = 16;
    while (c < 2 * want) c <<= 1;
    key.assign(c, nullptr);
    val.resize(c);
    mask = c - 1;
  }
  static size_t h(PyObject* o) { return (reinterpret_cast<uintptr_t>(o) >> 4) * 0x9E3779B97F4A7C15ull >> 17; }
  V* find(PyObject* o) {
    for (size_t i = h(o) & mask;; i = (i + 1) & mask) {
      if (key[i] == o) return &val[i];
      if (key[i] == nullptr) return nullptr;
    }
  }
  bool full() const { return 2 * (used + 1) > key.size(); }
  V* insert(PyObject* o, const V& v) {  // caller checks full() first
    size_t i = h(o) & mask;
    while (key[i] != nullptr && key[i] != o) i = (i + 1) & mask;
    if (key[i] == nullptr) ++used;
    key[i] = o;
    val[i] = v;
    return &val[i];
  }
};

// Attribute of a spec / config object: straight from the instance __dict__ when the
// name is there (dataclass fields), else the full attribute protocol.
static py::object getattr_(PyObject* o, const py::str& name) {
  PyObject** dp = _PyObject_GetDictPtr(o);
  if (dp != nullptr && *dp != nullptr) {
    PyObject* v = PyDict_GetItemWithError(*dp, name.ptr());  // borrowed
    if (v != nullptr) return py::reinterpret_borrow<py::object>(v);
    if (PyErr_Occurred()) throw py::error_already_set();
  }
  PyObject* r = PyObject_GetAttr(o, name.ptr());
  if (r == nullptr) throw py::error_already_set();
  return py::reinterpret_steal<py::object>(r);
}

static int truth(PyObject* o) {
  if (o == Py_True) return 1;
  if (o == Py_False || o == Py_None) return 0;
  const int v = PyObject_IsTrue(o);
  if (v < 0) throw py::error_already_set();
  return v;
}

static double as_double(PyObject* o) {
  if (PyFloat_CheckExact(o)) return PyFloat_AS_DOUBLE(o);
  const double v = PyFloat_AsDouble(o);
  if (v == -1.0 && PyErr_Occurred()) throw py::error_already_set();
  return v;
}

static int64_t as_int(PyObject* o) {
  const long long v = PyLong_AsLongLong(o);
  if (v == -1 && PyErr_Occurred()) throw py::error_already_set();
  return v;
}

// UTF-8 of a str without copying (CPython caches it in the object; ASCII strings
// return their own data).  Lone surrogates take the surrogatepass copy in `tmp`.
static std::string_view utf8_view(PyObject* o, std::string& tmp) {
  Py_ssize_t n = 0;
  const char* c = PyUnicode_AsUTF8AndSize(o, &n);
  if (c != nullptr) return std::string_view(c, static_cast<size_t>(n));
  PyErr_Clear();
  tmp = utf8_of(py::handle(o));
  return std::string_view(tmp);
}

// ConsistencyMode members are singletons: their mode is resolved once (an Enum's
// `.value` is a descriptor call) and remembered by identity (strong?)
static std::unordered_map<PyObject*, bool>& mode_members() {
  static std::unordered_map<PyObject*, bool> m;
  return m;
}

static const py::str& cfg_name(int k) {
  static const py::str names[] = {py::str("consistency_mode"), py::str("max_participants"), py::str("min_sigma_eff"),
                                  py::str("enable_audit")};
  return names[k];
}

static std::tuple<int32_t, double, uint8_t> config_row(PyObject* c) {
  static const py::str kValue("value");
  const py::str &kMode = cfg_name(0), &kMax = cfg_name(1), &kMin = cfg_name(2), &kAudit = cfg_name(3);
  auto& members = mode_members();
  py::object m = getattr_(c, kMode);
  bool strong;
  auto it = members.find(m.ptr());
  if (it != members.end()) {
    strong = it->second;
  } else {
    const bool is_str = PyUnicode_Check(m.ptr());
    py::object v = is_str ? m : getattr_(m.ptr(), kValue);
    std::string tmp;
    const std::string_view mode = utf8_view(v.ptr(), tmp);
    if (mode != "strong" && mode != "eventual")
      throw py::value_error("'" + std::string(mode) + "' is not a valid ConsistencyMode");
    strong = mode == "strong";
    if (!is_str && members.size() < 16) {
      Py_INCREF(m.ptr());  // kept alive: the cache holds the member by identity
      members.emplace(m.ptr(), strong);
    }
  }
  const int audit = truth(getattr_(c, kAudit).ptr());
  return {static_cast<int32_t>(as_int(getattr_(c, kMax).ptr())), as_double(getattr_(c, kMin).ptr()),
          static_cast<uint8_t>((audit ? 1 : 0) | (strong ? 2 : 0))};
}

// Spec packing works straight on the CPython objects: borrowed tuple items, no
// per-spec containers.  A spec object seen before in the batch (batches drawn
// from a pool of specs) copies its first occurrence's rows.
static py::dict pack_specs_serial(const py::list& specs, StringPool& agents, StringPool& pool,
                                  const py::object& cfg_of, int64_t fixed) {
  const size_t n = specs.size();
  std::vector<int32_t> creator(n), maxpart(n), join_off{0}, join_agent, delta_off{0}, d_pool, ch_off{0}, ch_rows,
      step_off{0}, s_retry;
  std::vector<double> minsig(n), join_sigma;
  std::vector<uint8_t> flags(n), s_undo, s_fail;
  std::vector<int64_t> base_caps;
  join_agent.reserve(3 * n);
  join_sigma.reserve(3 * n);
  d_pool.reserve(2 * n);
  base_caps.reserve(2 * n);
  ch_rows.reserve(16 * n);
  PtrTable<std::tuple<int32_t, double, uint8_t>> cfg_cache(std::min<size_t>(n, 65536) + 1);
  std::string tmp;
  // per call, per pool: str object → id (the same object recurs across specs — agent
  // DIDs drawn from one list, shared literals — and skips hashing its bytes)
  struct PtrCache {
    std::vector<std::pair<PyObject*, int32_t>> slot = std::vector<std::pair<PyObject*, int32_t>>(4096);
    int32_t* find(PyObject* o) {
      auto& e = slot[(reinterpret_cast<uintptr_t>(o) >> 4) & 4095];
      return e.first == o ? &e.second : nullptr;
    }
    void put(PyObject* o, int32_t id) { slot[(reinterpret_cast<uintptr_t>(o) >> 4) & 4095] = {o, id}; }
  } pc_agents, pc_pool;
  auto intern = [&](StringPool& p, PyObject* o) -> int32_t {
    PtrCache& pc = &p == &pool ? pc_pool : pc_agents;
    if (int32_t* hit = pc.find(o)) return *hit;
    if (!PyUnicode_Check(o)) throw py::type_error("spec strings must be str");
    const int32_t id = p.intern(utf8_view(o, tmp));
    pc.put(o, id);
    return id;
  };
  auto esc_of = [&](int32_t id) -> int64_t { return id < 0 ? 4 : pool.esc_len(id) + 2; };
  // first occurrence of a spec object: where its rows start in every column
  struct First {
    size_t spec, j0, d0, st0;
  };
  PtrTable<First> seen(std::min<size_t>(n, 65536));
  static const py::str kJoins("joins"), kDeltas("deltas"), kSteps("steps"), kAct("activate"), kTerm("terminate"),
      kComp("compensate"), kCfg("config"), kCreator("creator_did");
  PyObject* const* items = PySequence_Fast_ITEMS(specs.ptr());
  auto copy_range = [](auto& v, size_t a, size_t cnt) {
    v.reserve(v.size() + cnt);
    for (size_t k = 0; k < cnt; ++k) v.push_back(v[a + k]);
  };
  for (size_t i = 0; i < n; ++i) {
    PyObject* sp = items[i];
    if (!seen.full()) {  // (bounded: a batch of all-distinct specs gains nothing from the table)
      const First* hit = seen.find(sp);
      if (hit != nullptr) {
        const First& f = *hit;
        creator[i] = creator[f.spec];
        maxpart[i] = maxpart[f.spec];
        minsig[i] = minsig[f.spec];
        flags[i] = flags[f.spec];
        const size_t nj = static_cast<size_t>(join_off[f.spec + 1] - join_off[f.spec]);
        copy_range(join_agent, f.j0, nj);
        copy_range(join_sigma, f.j0, nj);
        join_off.push_back(static_cast<int32_t>(join_agent.size()));
        const size_t nd = static_cast<size_t>(delta_off[f.spec + 1] - delta_off[f.spec]);
        copy_range(d_pool, f.d0, nd);
        copy_range(base_caps, f.d0, nd);
        const int32_t cfirst = ch_off[f.d0];
        const size_t nch = static_cast<size_t>(ch_off[f.d0 + nd] - cfirst);
        const size_t c0 = ch_rows.size();
        copy_range(ch_rows, static_cast<size_t>(cfirst) * 4, nch * 4);
        for (size_t k = 0; k < nd; ++k) ch_off.push_back(static_cast<int32_t>(c0 / 4) + ch_off[f.d0 + k + 1] - cfirst);
        delta_off.push_back(static_cast<int32_t>(d_pool.size()));
        const size_t ns = static_cast<size_t>(step_off[f.spec + 1] - step_off[f.spec]);
        copy_range(s_undo, f.st0, ns);
        copy_range(s_retry, f.st0, ns);
        copy_range(s_fail, f.st0, ns);
        step_off.push_back(static_cast<int32_t>(s_undo.size()));
        continue;
      }
      seen.insert(sp, First{i, join_agent.size(), d_pool.size(), s_undo.size()});
    }
    py::object cfg = getattr_(sp, kCfg);
    const std::tuple<int32_t, double, uint8_t>* ci = cfg_cache.find(cfg.ptr());
    std::tuple<int32_t, double, uint8_t> row;
    if (ci == nullptr) {
      if (cfg.is_none()) {  // the default SessionConfig, resolved by the caller
        py::tuple t = cfg_of(cfg);
        row = std::make_tuple(t[0].cast<int32_t>(), t[1].cast<double>(), t[2].cast<uint8_t>());
      } else {
        row = config_row(cfg.ptr());
      }
      if (!cfg_cache.full()) cfg_cache.insert(cfg.ptr(), row);
      ci = &row;
    }
    maxpart[i] = std::get<0>(*ci);
    minsig[i] = std::get<1>(*ci);
    flags[i] = static_cast<uint8_t>(std::get<2>(*ci) | (truth(getattr_(sp, kAct).ptr()) ? 4 : 0) |
                                    (truth(getattr_(sp, kTerm).ptr()) ? 8 : 0) |
                                    (truth(getattr_(sp, kComp).ptr()) ? 16 : 0));
    creator[i] = intern(agents, getattr_(sp, kCreator).ptr());
    {
      py::object js = getattr_(sp, kJoins);
      FastSeq jl(js.ptr());
      for (Py_ssize_t k = 0; k < jl.n; ++k) {
        FastSeq t(jl.it[k]);
        join_agent.push_back(intern(agents, t[0]));
        join_sigma.push_back(as_double(t[1]));
      }
    }
    join_off.push_back(static_cast<int32_t>(join_agent.size()));
    {
      py::object ds = getattr_(sp, kDeltas);
      FastSeq dl(ds.ptr());
      for (Py_ssize_t k = 0; k < dl.n; ++k) {
        FastSeq t(dl.it[k]);
        const int32_t did = intern(pool, t[0]);
        d_pool.push_back(did);
        int64_t cap = fixed + esc_of(did);
        FastSeq cl(t[1]);
        for (Py_ssize_t q = 0; q < cl.n; ++q) {
          FastSeq ct(cl.it[q]);
          const int32_t path = intern(pool, ct[0]), op = intern(pool, ct[1]);
          const int32_t h = ct[2] == Py_None ? -1 : intern(pool, ct[2]);
          const int32_t prev = ct.n > 3 && ct.it[3] != Py_None ? intern(pool, ct.it[3]) : -1;
          ch_rows.push_back(path);
          ch_rows.push_back(op);
          ch_rows.push_back(h);
          ch_rows.push_back(prev);
          cap += 17 + 15 + 10 + 19 + 1 + (q ? 2 : 0) + esc_of(h) + esc_of(op) + esc_of(path) + esc_of(prev);
        }
        ch_off.push_back(static_cast<int32_t>(ch_rows.size() / 4));
        base_caps.push_back(cap);
      }
    }
    delta_off.push_back(static_cast<int32_t>(d_pool.size()));
    {
      py::object ss = getattr_(sp, kSteps);
      FastSeq sl(ss.ptr());
      for (Py_ssize_t k = 0; k < sl.n; ++k) {
        FastSeq t(sl.it[k]);
        s_undo.push_back(truth(t[3]) ? 1 : 0);
        s_retry.push_back(static_cast<int32_t>(as_int(t[4])));
        const int64_t f = as_int(t[5]);
        s_fail.push_back(static_cast<uint8_t>(f < 255 ? f : 255));
      }
    }
    step_off.push_back(static_cast<int32_t>(s_undo.size()));
  }
  py::dict out;
  out["creator"] = as_bytes(creator);
  out["maxpart"] = as_bytes(maxpart);
  out["minsig"] = as_bytes(minsig);
  out["flags"] = as_bytes(flags);
  out["join_off"] = as_bytes(join_off);
  out["join_agent"] = as_bytes(join_agent);
  out["join_sigma"] = as_bytes(join_sigma);
  out["delta_off"] = as_bytes(delta_off);
  out["d_pool"] = as_bytes(d_pool);
  out["base_caps"] = as_bytes(base_caps);
  out["ch_off"] = as_bytes(ch_off);
  out["ch_rows"] = as_bytes(ch_rows);
  out["step_off"] = as_bytes(step_off);
  out["s_undo"] = as_bytes(s_undo);
  out["s_retry"] = as_bytes(s_retry);
  out["s_fail"] = as_bytes(s_fail);
  return out;
}


// ------------------------------------------------------- parallel spec walk
// The serial walk above is bound by reading CPython objects one spec at a time
// (≈35 objects per random spec).  Here T threads walk disjoint spec ranges while
// the calling thread holds the GIL and waits: no Python code can run meanwhile,
// and the workers only READ objects through borrowed pointers — no reference
// counts, no allocation, no Python error state.  Anything off the fast shapes
// (a str that is not compact ASCII, a sequence that is not a tuple / list, an
// attribute not in the instance __dict__, a truth value that is not a bool /
// None / str, a number that is not a float or a one-digit int) marks the walk
// failed and the serial walk redoes the whole batch (same columns, its errors).
//
// Workers give strings part-local ids (first-occurrence order); the merge, back
// on the calling thread, interns each part's strings in that order — the same
// global ids the serial walk assigns — and rewrites the columns.
namespace pack {

inline bool ascii_view(PyObject* o, std::string_view& out) {
  if (!PyUnicode_CheckExact(o) || !PyUnicode_IS_COMPACT_ASCII(o)) return false;
  // PyUnicode_DATA / GET_LENGTH read the object's own fields on every version (no
  // allocation; the compact-ASCII data offset moved when 3.12 dropped wstr)
  out = std::string_view(static_cast<const char*>(PyUnicode_DATA(o)), static_cast<size_t>(PyUnicode_GET_LENGTH(o)));
  return true;
}

// Instance-__dict__ attribute (borrowed) or null.  `name` is a str whose hash the
// caller computed beforehand, so the lookup only reads.
inline PyObject* dict_attr(PyObject* o, PyObject* name) {
  PyObject** dp = _PyObject_GetDictPtr(o);
  if (dp == nullptr || *dp == nullptr || !PyDict_CheckExact(*dp)) return nullptr;
  return PyDict_GetItemWithError(*dp, name);
}

inline bool seq(PyObject* o, PyObject* const*& it, Py_ssize_t& n) {
  if (PyTuple_CheckExact(o)) {
    it = reinterpret_cast<PyTupleObject*>(o)->ob_item;
    n = PyTuple_GET_SIZE(o);
    return true;
  }
  if (PyList_CheckExact(o)) {
    it = reinterpret_cast<PyListObject*>(o)->ob_item;
    n = PyList_GET_SIZE(o);
    return true;
  }
  return false;
}

inline bool small_int(PyObject* o, int64_t& v) {
  if (!PyLong_CheckExact(o)) return false;
#if PY_VERSION_HEX >= 0x030C0000
  // 3.12 replaced ob_size / ob_digit with lv_tag; the unstable compact accessors
  // are inline reads of that layout (no allocation, no error state)
  PyLongObject* l = reinterpret_cast<PyLongObject*>(o);
  if (!PyUnstable_Long_IsCompact(l)) return false;
  v = static_cast<int64_t>(PyUnstable_Long_CompactValue(l));
  return true;
#else
  const Py_ssize_t sz = Py_SIZE(o);
  if (sz == 0) {
    v = 0;
    return true;
  }
  if (sz != 1 && sz != -1) return false;
  v = static_cast<int64_t>(reinterpret_cast<PyLongObject*>(o)->ob_digit[0]);
  if (sz < 0) v = -v;
  return true;
#endif
}

inline bool number(PyObject* o, double& v) {
  if (PyFloat_CheckExact(o)) {
    v = PyFloat_AS_DOUBLE(o);
    return true;
  }
  int64_t i;
  if (!small_int(o, i)) return false;
  v = static_cast<double>(i);
  return true;
}

inline bool truth(PyObject* o, bool& v) {
  if (o == Py_True || o == Py_False || o == Py_None) {
    v = o == Py_True;
    return true;
  }
  std::string_view s;
  if (ascii_view(o, s)) {
    v = !s.empty();
    return true;
  }
  return false;
}

// Part-local string ids by content; a direct-mapped memo skips re-hashing an
// object seen before (agent DIDs drawn from one list, shared literals).
struct LocalPool {
  std::vector<std::string_view> strs;
  std::vector<PyObject*> objs;  // a str that is not compact ASCII: encoded by the merge (GIL held)
  std::vector<int32_t> table;
  std::vector<uint64_t> hashes;
  size_t mask = 0;
  std::vector<std::pair<PyObject*, int32_t>> memo = std::vector<std::pair<PyObject*, int32_t>>(4096);
  LocalPool() : table(1024, -1), mask(1023) {}
  static uint64_t hash(std::string_view s) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ s.size();
    size_t i = 0;
    for (; i + 8 <= s.size(); i += 8) {
      uint64_t w;
      std::memcpy(&w, s.data() + i, 8);
      h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
      h ^= h >> 31;
    }
    uint64_t w = 0;
    std::memcpy(&w, s.data() + i, s.size() - i);
    h = (h ^ w) * 0x94D049BB133111EBull;
    return h ^ (h >> 29);
  }
  void grow() {
    const size_t cap = table.size() * 2;
    std::vector<int32_t> t(cap, -1);
    for (size_t id = 0; id < strs.size(); ++id) {
      if (id < objs.size() && objs[id] != nullptr) continue;  // identity-keyed: not in the content table
      size_t i = hashes[id] & (cap - 1);
      while (t[i] >= 0) i = (i + 1) & (cap - 1);
      t[i] = static_cast<int32_t>(id);
    }
    table.swap(t);
    mask = cap - 1;
  }
  // -1 if `o` is not a str (the caller fails the walk)
  int32_t get(PyObject* o) {
    auto& m = memo[(reinterpret_cast<uintptr_t>(o) >> 4) & 4095];
    if (m.first == o) return m.second;
    std::string_view s;
    if (!ascii_view(o, s)) {
      if (!PyUnicode_CheckExact(o)) return -1;
      // no UTF-8 to read without allocating: keyed by identity, encoded by the merge
      const int32_t id = static_cast<int32_t>(strs.size());
      strs.emplace_back();
      hashes.push_back(0);
      objs.resize(strs.size(), nullptr);
      objs[static_cast<size_t>(id)] = o;
      m = {o, id};
      return id;
    }
    const uint64_t h = hash(s);
    size_t i = h & mask;
    for (;; i = (i + 1) & mask) {
      const int32_t id = table[i];
      if (id < 0) break;
      if (hashes[id] == h && strs[id] == s) {
        m = {o, id};
        return id;
      }
    }
    const int32_t id = static_cast<int32_t>(strs.size());
    strs.push_back(s);
    hashes.push_back(h);
    if (!objs.empty()) objs.push_back(nullptr);
    table[i] = id;
    if (2 * strs.size() > table.size()) grow();
    m = {o, id};
    return id;
  }
};

struct Names {
  PyObject *joins, *deltas, *steps, *act, *term, *comp, *cfg, *creator;
  PyObject *mode, *maxp, *mins, *audit;
  const std::vector<std::pair<PyObject*, bool>>* members;  // resolved ConsistencyMode members
};

struct Part {
  size_t lo = 0, hi = 0;
  bool ok = true;
  LocalPool agents, pool;
  std::vector<PyObject*> cfg;
  std::vector<std::tuple<int32_t, double, uint8_t>> cfg_row;  // valid where cfg_ok
  std::vector<uint8_t> cfg_ok;
  std::vector<int32_t> creator, njoin, join_agent, ndelta, d_pool, nch, ch_rows, nstep, s_retry;
  std::vector<double> join_sigma;
  std::vector<uint8_t> bits, s_undo, s_fail;

  int bad_line = 0;
  bool fail(int line) {
    bad_line = line;
    return false;
  }
  bool walk_one(PyObject* sp, const Names& k) {
    PyObject* c = dict_attr(sp, k.cfg);
    if (c == nullptr) return fail(__LINE__);
    cfg.push_back(c);
    config(c, k);
    bool a, t, m;
    PyObject *pa = dict_attr(sp, k.act), *pt = dict_attr(sp, k.term), *pm = dict_attr(sp, k.comp);
    if (!pa || !pt || !pm || !truth(pa, a) || !truth(pt, t) || !truth(pm, m)) return fail(__LINE__);
    bits.push_back(static_cast<uint8_t>((a ? 4 : 0) | (t ? 8 : 0) | (m ? 16 : 0)));
    PyObject* cr = dict_attr(sp, k.creator);
    if (cr == nullptr) return fail(__LINE__);
    const int32_t cid = agents.get(cr);
    if (cid < 0) return fail(__LINE__);
    creator.push_back(cid);
    PyObject* const* it;
    Py_ssize_t n;
    PyObject* js = dict_attr(sp, k.joins);
    if (js == nullptr || !seq(js, it, n)) return fail(__LINE__);
    njoin.push_back(static_cast<int32_t>(n));
    for (Py_ssize_t q = 0; q < n; ++q) {
      PyObject* const* jt;
      Py_ssize_t jn;
      if (!seq(it[q], jt, jn) || jn < 2) return fail(__LINE__);
      const int32_t id = agents.get(jt[0]);
      double sg;
      if (id < 0 || !number(jt[1], sg)) return fail(__LINE__);
      join_agent.push_back(id);
      join_sigma.push_back(sg);
    }
    PyObject* ds = dict_attr(sp, k.deltas);
    if (ds == nullptr || !seq(ds, it, n)) return fail(__LINE__);
    ndelta.push_back(static_cast<int32_t>(n));
    for (Py_ssize_t q = 0; q < n; ++q) {
      PyObject* const* dt;
      Py_ssize_t dn;
      if (!seq(it[q], dt, dn) || dn < 2) return fail(__LINE__);
      const int32_t did = pool.get(dt[0]);
      if (did < 0) return fail(__LINE__);
      d_pool.push_back(did);
      PyObject* const* ct;
      Py_ssize_t cn;
      if (!seq(dt[1], ct, cn)) return fail(__LINE__);
      nch.push_back(static_cast<int32_t>(cn));
      for (Py_ssize_t r = 0; r < cn; ++r) {
        PyObject* const* x;
        Py_ssize_t xn;
        if (!seq(ct[r], x, xn) || xn < 3) return fail(__LINE__);
        const int32_t path = pool.get(x[0]), op = pool.get(x[1]);
        const int32_t h = x[2] == Py_None ? -1 : pool.get(x[2]);
        const int32_t prev = xn > 3 && x[3] != Py_None ? pool.get(x[3]) : -1;
        if (path < 0 || op < 0 || (h < 0 && x[2] != Py_None) || (prev < 0 && xn > 3 && x[3] != Py_None)) return fail(__LINE__);
        ch_rows.push_back(path);
        ch_rows.push_back(op);
        ch_rows.push_back(h);
        ch_rows.push_back(prev);
      }
    }
    PyObject* ss = dict_attr(sp, k.steps);
    if (ss == nullptr || !seq(ss, it, n)) return fail(__LINE__);
    nstep.push_back(static_cast<int32_t>(n));
    for (Py_ssize_t q = 0; q < n; ++q) {
      PyObject* const* st;
      Py_ssize_t sn;
      if (!seq(it[q], st, sn) || sn < 6) return fail(__LINE__);
      bool undo;
      int64_t retry, nfail;
      if (!truth(st[3], undo) || !small_int(st[4], retry) || !small_int(st[5], nfail)) return fail(__LINE__);
      s_undo.push_back(undo ? 1 : 0);
      s_retry.push_back(static_cast<int32_t>(retry));
      s_fail.push_back(static_cast<uint8_t>(nfail < 255 ? nfail : 255));
    }
    return true;
  }

  // A SessionConfig's row when every field is on the fast shapes and its mode
  // member was resolved before the walk; else the merge resolves it (GIL held).
  void config(PyObject* c, const Names& k) {
    cfg_row.emplace_back();
    cfg_ok.push_back(0);
    if (c == Py_None) return;
    PyObject *m = dict_attr(c, k.mode), *mx = dict_attr(c, k.maxp), *mn = dict_attr(c, k.mins),
             *au = dict_attr(c, k.audit);
    if (!m || !mx || !mn || !au) return;
    int64_t maxp;
    double mins;
    bool audit;
    if (!small_int(mx, maxp) || !number(mn, mins) || !truth(au, audit)) return;
    for (const auto& e : *k.members)
      if (e.first == m) {
        cfg_row.back() = std::make_tuple(static_cast<int32_t>(maxp), mins,
                                         static_cast<uint8_t>((audit ? 1 : 0) | (e.second ? 2 : 0)));
        cfg_ok.back() = 1;
        return;
      }
  }

  double ms = 0;
  void walk(PyObject* const* items, const Names& k) {
    const auto t0 = std::chrono::steady_clock::now();
    walk_(items, k);
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  void walk_(PyObject* const* items, const Names& k) {
    const size_t m = hi - lo;
    cfg.reserve(m);
    bits.reserve(m);
    creator.reserve(m);
    for (size_t i = lo; i < hi && ok; ++i) ok = walk_one(items[i], k);
  }
};

}  // namespace pack

static int pack_threads_default() {
  static const int v = [] {
    const char* e = std::getenv("AHV_PACK_THREADS");
    if (e != nullptr) return std::atoi(e);
    // a GPU box grants one process about 16 CPUs (20k random specs: 16.9 ms serial,
    // 7.1 ms on 8 threads, 6.1 ms on 16; MI355X box)
    const unsigned h = std::thread::hardware_concurrency();
    return static_cast<int>(h == 0 ? 1 : h < 16 ? h : 16);
  }();
  return v;
}

// The GIL-free walk reads instance dicts through _PyObject_GetDictPtr.  Up to 3.10
// that only returns the slot; from 3.11 objects keep "managed" inline values and the
// call MATERIALISES a dict (allocates and stores into the object) — never allowed
// off the GIL thread.  So the parallel walk exists only where it is read-only.
#if PY_VERSION_HEX < 0x030B0000
#define AHV_PARALLEL_SPEC_WALK 1
#else
#define AHV_PARALLEL_SPEC_WALK 0
#endif

static const char* g_last_walk = "none";  // "serial" / "parallel" / "parallel->serial" (tests, profiling)

// threads: < 0 → AHV_PACK_THREADS or min(16, cores) for batches of ≥ 4,096 specs;
// 0 / 1 → the serial walk (always, on Python ≥ 3.11).
static py::dict pack_specs(const py::list& specs, StringPool& agents, StringPool& pool, const py::object& cfg_of,
                           int64_t fixed, int threads) {
  const size_t n = specs.size();
  int T = threads;
  if (T < 0) T = n >= 4096 ? pack_threads_default() : 1;
  if (T > 64) T = 64;
  if (!AHV_PARALLEL_SPEC_WALK || T <= 1 || n < static_cast<size_t>(2 * T)) {
    g_last_walk = "serial";
    return pack_specs_serial(specs, agents, pool, cfg_of, fixed);
  }
  g_last_walk = "parallel";
  static const py::str kJoins("joins"), kDeltas("deltas"), kSteps("steps"), kAct("activate"), kTerm("terminate"),
      kComp("compensate"), kCfg("config"), kCreator("creator_did");
  for (const py::str* nm : {&kJoins, &kDeltas, &kSteps, &kAct, &kTerm, &kComp, &kCfg, &kCreator, &cfg_name(0),
                            &cfg_name(1), &cfg_name(2), &cfg_name(3)})
    if (PyObject_Hash(nm->ptr()) == -1) throw py::error_already_set();  // cached: the workers' lookups only read
  PyObject* const* items = PySequence_Fast_ITEMS(specs.ptr());
  {
    // resolve the first spec's consistency mode member here, so the workers find it
    PyObject* c0 = pack::dict_attr(items[0], kCfg.ptr());
    if (c0 != nullptr && c0 != Py_None) {
      try {
        config_row(c0);
      } catch (py::error_already_set&) {
        // reported by the merge / serial walk, which reads the same object
        PyErr_Clear();
      }
    }
  }
  std::vector<std::pair<PyObject*, bool>> members(mode_members().begin(), mode_members().end());
  const pack::Names names{kJoins.ptr(), kDeltas.ptr(), kSteps.ptr(), kAct.ptr(), kTerm.ptr(), kComp.ptr(),
                          kCfg.ptr(), kCreator.ptr(), cfg_name(0).ptr(), cfg_name(1).ptr(), cfg_name(2).ptr(),
                          cfg_name(3).ptr(), &members};
  std::vector<pack::Part> parts(static_cast<size_t>(T));
  for (int t = 0; t < T; ++t) {
    parts[t].lo = n * static_cast<size_t>(t) / static_cast<size_t>(T);
    parts[t].hi = n * static_cast<size_t>(t + 1) / static_cast<size_t>(T);
  }
  const auto tw0 = std::chrono::steady_clock::now();
  {
    // the GIL stays held by this thread: nothing else touches the objects meanwhile
    std::vector<std::thread> pool_threads;
    pool_threads.reserve(static_cast<size_t>(T - 1));
    for (int t = 1; t < T; ++t)
      pool_threads.emplace_back([&parts, items, &names, t] {
        try {
          parts[t].walk(items, names);
        } catch (...) {
          parts[t].ok = false;
        }
      });
    try {
      parts[0].walk(items, names);
    } catch (...) {
      parts[0].ok = false;
    }
    for (auto& th : pool_threads) th.join();
  }
  const auto tw1 = std::chrono::steady_clock::now();
  for (const auto& p : parts)
    if (!p.ok) {
      if (std::getenv("AHV_PACK_DEBUG")) std::fprintf(stderr, "[pack] serial walk: part fell back at line %d\n", p.bad_line);
      g_last_walk = "parallel->serial";
      return pack_specs_serial(specs, agents, pool, cfg_of, fixed);
    }
  // ---- merge: (1) with the GIL, intern each part's strings in first-occurrence
  // order (the serial walk's global ids) and resolve the configs the workers could
  // not; (2) the workers write their ranges of the columns, ids remapped, at offsets
  // from a prefix sum over the parts.
  const size_t P = parts.size();
  std::vector<size_t> jb(P + 1, 0), db(P + 1, 0), cb(P + 1, 0), sb(P + 1, 0);
  for (size_t t = 0; t < P; ++t) {
    jb[t + 1] = jb[t] + parts[t].join_agent.size();
    db[t + 1] = db[t] + parts[t].d_pool.size();
    cb[t + 1] = cb[t] + parts[t].ch_rows.size() / 4;
    sb[t + 1] = sb[t] + parts[t].s_undo.size();
  }
  std::vector<int32_t> creator(n), maxpart(n), join_off(n + 1), join_agent(jb[P]), delta_off(n + 1), d_pool(db[P]),
      ch_off(db[P] + 1), ch_rows(4 * cb[P]), step_off(n + 1), s_retry(sb[P]);
  std::vector<double> minsig(n), join_sigma(jb[P]);
  std::vector<uint8_t> flags(n), s_undo(sb[P]), s_fail(sb[P]);
  std::vector<int64_t> base_caps(db[P]);
  join_off[0] = delta_off[0] = ch_off[0] = step_off[0] = 0;
  std::vector<std::vector<int32_t>> amap(P), pmap(P);
  std::vector<std::vector<int64_t>> pesc(P);
  {
    PtrTable<std::tuple<int32_t, double, uint8_t>> cfg_cache(std::min<size_t>(n, 65536) + 1);
    std::string tmp;
    auto local = [&tmp](const pack::LocalPool& lp, size_t l) -> std::string_view {
      if (l < lp.objs.size() && lp.objs[l] != nullptr) return utf8_view(lp.objs[l], tmp);
      return lp.strs[l];
    };
    for (size_t t = 0; t < P; ++t) {
      pack::Part& p = parts[t];
      amap[t].resize(p.agents.strs.size());
      for (size_t l = 0; l < amap[t].size(); ++l) amap[t][l] = agents.intern(local(p.agents, l));
      pmap[t].resize(p.pool.strs.size());
      pesc[t].resize(pmap[t].size());
      for (size_t l = 0; l < pmap[t].size(); ++l) {
        pmap[t][l] = pool.intern(local(p.pool, l));
        pesc[t][l] = pool.esc_len(pmap[t][l]) + 2;
      }
      for (size_t r = 0; r < p.cfg.size(); ++r) {
        if (p.cfg_ok[r]) continue;
        PyObject* cfg = p.cfg[r];
        const std::tuple<int32_t, double, uint8_t>* ci = cfg_cache.find(cfg);
        if (ci == nullptr) {
          std::tuple<int32_t, double, uint8_t> row;
          if (cfg == Py_None) {
            py::tuple tt = cfg_of(py::none());
            row = std::make_tuple(tt[0].cast<int32_t>(), tt[1].cast<double>(), tt[2].cast<uint8_t>());
          } else {
            row = config_row(cfg);
          }
          if (!cfg_cache.full()) ci = cfg_cache.insert(cfg, row);
          p.cfg_row[r] = row;
        } else {
          p.cfg_row[r] = *ci;
        }
        p.cfg_ok[r] = 1;
      }
    }
  }
  auto fill = [&](size_t t) {
    const pack::Part& p = parts[t];
    const std::vector<int32_t>& am = amap[t];
    const std::vector<int32_t>& pm = pmap[t];
    const std::vector<int64_t>& pe = pesc[t];
    auto Pm = [&pm](int32_t l) { return l < 0 ? -1 : pm[static_cast<size_t>(l)]; };
    auto E = [&pe](int32_t l) -> int64_t { return l < 0 ? 4 : pe[static_cast<size_t>(l)]; };
    size_t jk = 0, dk = 0, ck = 0, sk = 0;
    size_t jo = jb[t], dd = db[t], co = cb[t], so = sb[t];
    for (size_t i = p.lo, r = 0; i < p.hi; ++i, ++r) {
      const auto& ci = p.cfg_row[r];
      maxpart[i] = std::get<0>(ci);
      minsig[i] = std::get<1>(ci);
      flags[i] = static_cast<uint8_t>(std::get<2>(ci) | p.bits[r]);
      creator[i] = am[static_cast<size_t>(p.creator[r])];
      for (int32_t q = 0; q < p.njoin[r]; ++q, ++jk, ++jo) {
        join_agent[jo] = am[static_cast<size_t>(p.join_agent[jk])];
        join_sigma[jo] = p.join_sigma[jk];
      }
      join_off[i + 1] = static_cast<int32_t>(jo);
      for (int32_t q = 0; q < p.ndelta[r]; ++q, ++dk, ++dd) {
        const int32_t ld = p.d_pool[dk];
        d_pool[dd] = Pm(ld);
        int64_t cap = fixed + E(ld);
        for (int32_t c = 0; c < p.nch[dk]; ++c, ck += 4, ++co) {
          const int32_t path = p.ch_rows[ck], op = p.ch_rows[ck + 1], h = p.ch_rows[ck + 2], prev = p.ch_rows[ck + 3];
          ch_rows[4 * co] = Pm(path);
          ch_rows[4 * co + 1] = Pm(op);
          ch_rows[4 * co + 2] = Pm(h);
          ch_rows[4 * co + 3] = Pm(prev);
          cap += 17 + 15 + 10 + 19 + 1 + (c ? 2 : 0) + E(h) + E(op) + E(path) + E(prev);
        }
        ch_off[dd + 1] = static_cast<int32_t>(co);
        base_caps[dd] = cap;
      }
      delta_off[i + 1] = static_cast<int32_t>(dd);
      for (int32_t q = 0; q < p.nstep[r]; ++q, ++sk, ++so) {
        s_undo[so] = p.s_undo[sk];
        s_retry[so] = p.s_retry[sk];
        s_fail[so] = p.s_fail[sk];
      }
      step_off[i + 1] = static_cast<int32_t>(so);
    }
  };
  {
    std::vector<std::thread> fill_threads;
    fill_threads.reserve(P - 1);
    for (size_t t = 1; t < P; ++t) fill_threads.emplace_back(fill, t);
    fill(0);
    for (auto& th : fill_threads) th.join();
  }
  if (std::getenv("AHV_PACK_DEBUG")) {
    const auto tw2 = std::chrono::steady_clock::now();
    for (const auto& p : parts) std::fprintf(stderr, "[pack]   part %zu..%zu %.2f ms, %zu+%zu strings\n", p.lo, p.hi, p.ms,
                                             p.agents.strs.size(), p.pool.strs.size());
    std::fprintf(stderr, "[pack] T=%d walk %.2f ms merge %.2f ms\n", T,
                 std::chrono::duration<double, std::milli>(tw1 - tw0).count(),
                 std::chrono::duration<double, std::milli>(tw2 - tw1).count());
  }
  py::dict out;
  out["creator"] = as_bytes(creator);
  out["maxpart"] = as_bytes(maxpart);
  out["minsig"] = as_bytes(minsig);
  out["flags"] = as_bytes(flags);
  out["join_off"] = as_bytes(join_off);
  out["join_agent"] = as_bytes(join_agent);
  out["join_sigma"] = as_bytes(join_sigma);
  out["delta_off"] = as_bytes(delta_off);
  out["d_pool"] = as_bytes(d_pool);
  out["base_caps"] = as_bytes(base_caps);
  out["ch_off"] = as_bytes(ch_off);
  out["ch_rows"] = as_bytes(ch_rows);
  out["step_off"] = as_bytes(step_off);
  out["s_undo"] = as_bytes(s_undo);
  out["s_retry"] = as_bytes(s_retry);
  out["s_fail"] = as_bytes(s_fail);
  return out;
}

// The changes fragment of a template delta (ahv/delta_emit.h emit_changes_fragment)
// rendered from the pool's escaped strings: `changes` = [[path, op, content_hash,
// previous_hash], ...] pool ids (-1 = null).  The device copies these bytes.
static py::bytes render_fragment(const StringPool& pool, const std::vector<std::array<int32_t, 4>>& changes,
                                 uint32_t turn, bool has_parent) {
  std::vector<ChangeIds> ch;
  for (const auto& c : changes) {
    for (int32_t id : c)
      if (id >= static_cast<int32_t>(pool.size())) throw py::index_error("string id out of range");
    ch.push_back(ChangeIds{c[0], c[1], c[2], c[3]});
  }
  const StrPool sp = pool.str_pool();
  std::vector<uint8_t> out;
  ByteSink sink{&out};
  emit_changes_fragment(sink, sp, ch.data(), static_cast<uint32_t>(ch.size()), -1, turn, has_parent);
  return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
}

// ------------------------------------------------------------------ record head fragments
// The batched store pipeline's records all begin `{"agent_did": <did>, "changes":
// [...], "delta_id": "delta:` — bytes fixed by the delta's agent and change list
// (canonical JSON, sorted keys).  A batch's deltas draw those from far fewer
// distinct (agent, changes) pairs than it has deltas, so each distinct head is
// rendered once here with the device's own emitters (ahv/delta_emit.h), and the
// render kernel copies it into each record with 16-byte stores before emitting the
// per-record rest (turn, parent hole, session id, timestamp).  Every record is
// still written and hashed in full.
//
// frag_pack(pool, d_pool, ch_off, ch_rows) -> {"dfrag": int32[nd] bytes, "fbytes":
// bytes (entries 16-aligned, zero-padded), "foff": int64[F], "flen": int32[F]}
static py::dict frag_pack(const StringPool& pool, const py::bytes& d_pool_b, const py::bytes& ch_off_b,
                          const py::bytes& ch_rows_b) {
  std::string_view dpv = d_pool_b, cov = ch_off_b, crv = ch_rows_b;
  const size_t nd = dpv.size() / 4;
  if (cov.size() / 4 != nd + 1) throw py::value_error("frag_pack: ch_off must have nd + 1 entries");
  const int32_t* dp = reinterpret_cast<const int32_t*>(dpv.data());
  const int32_t* co = reinterpret_cast<const int32_t*>(cov.data());
  const int32_t* cr = reinterpret_cast<const int32_t*>(crv.data());
  const size_t nrows = crv.size() / 16;
  const int32_t np = static_cast<int32_t>(pool.size());
  std::string dfrag(4 * nd, '\0');
  int32_t* df = reinterpret_cast<int32_t*>(dfrag.data());
  std::vector<uint8_t> bytes;
  std::vector<int64_t> foff;
  std::vector<int32_t> flen;
  std::unordered_map<std::string, int32_t> seen;
  seen.reserve(1024);
  std::string key;
  const StrPool sp = pool.str_pool();
  std::vector<ChangeIds> ch;
  {
    py::gil_scoped_release nogil;
    for (size_t g = 0; g < nd; ++g) {
      const int32_t lo = co[g], hi = co[g + 1];
      if (lo < 0 || hi < lo || static_cast<size_t>(hi) > nrows) throw std::out_of_range("frag_pack: change range");
      key.assign(reinterpret_cast<const char*>(dp + g), 4);
      key.append(reinterpret_cast<const char*>(cr + 4 * lo), 16 * static_cast<size_t>(hi - lo));
      auto it = seen.find(key);
      if (it != seen.end()) {
        df[g] = it->second;
        continue;
      }
      const int32_t f = static_cast<int32_t>(foff.size());
      seen.emplace(key, f);
      df[g] = f;
      if (dp[g] >= np) throw std::out_of_range("frag_pack: agent string id");
      ch.clear();
      for (int32_t c = lo; c < hi; ++c) {
        const int32_t* r = cr + 4 * c;
        for (int k = 0; k < 4; ++k)
          if (r[k] >= np) throw std::out_of_range("frag_pack: change string id");
        ch.push_back(ChangeIds{r[0], r[1], r[2], r[3]});
      }
      foff.push_back(static_cast<int64_t>(bytes.size()));
      const size_t b0 = bytes.size();
      ByteSink sink{&bytes};
      emit_lit(sink, canon::K_OPEN_AGENT);
      emit_pool_str(sink, sp, dp[g]);
      emit_lit(sink, canon::K_CHANGES);
      for (size_t c = 0; c < ch.size(); ++c) {
        if (c) emit_lit(sink, canon::K_CH_SEP);
        emit_lit(sink, canon::K_CH_OPEN);
        emit_pool_str(sink, sp, ch[c].content_hash);
        emit_lit(sink, canon::K_CH_OP);
        emit_pool_str(sink, sp, ch[c].op);
        emit_lit(sink, canon::K_CH_PATH);
        emit_pool_str(sink, sp, ch[c].path);
        emit_lit(sink, canon::K_CH_PREV);
        emit_pool_str(sink, sp, ch[c].previous_hash);
        emit_lit(sink, canon::K_CH_CLOSE);
      }
      emit_lit(sink, canon::K_DELTA_ID);
      emit_lit(sink, canon::K_DELTA_PFX);
      flen.push_back(static_cast<int32_t>(bytes.size() - b0));
      bytes.resize((bytes.size() + 15) & ~size_t(15), 0);  // the next entry starts 16-aligned
    }
  }
  bytes.resize(bytes.size() + 16, 0);  // a tail read of the last entry stays in bounds
  py::dict out;
  out["dfrag"] = py::bytes(dfrag);
  out["fbytes"] = py::bytes(reinterpret_cast<const char*>(bytes.data()), bytes.size());
  out["foff"] = py::bytes(reinterpret_cast<const char*>(foff.data()), 8 * foff.size());
  out["flen"] = py::bytes(reinterpret_cast<const char*>(flen.data()), 4 * flen.size());
  return out;
}

// ------------------------------------------------------------------ attribution packing
// CausalAttributor.attribute_batch: the K21 columns of many failure cases, read
// natively from their dicts.  Per case the agents are listed in the iteration
// order of set(agent_actions) — the order the scalar engine ranks ties in — and
// each node's (agent column, success, root cause, ω) is taken exactly as
// build_causal_dag / raw_scores read it.

static py::tuple pack_attribution(const py::list& cases) {
  std::vector<int32_t> node_off{0}, agent_off{0}, agent_of;
  std::vector<uint8_t> succ, root;
  std::vector<double> omega;
  py::list agents_per_case(cases.size());
  static const py::str kAA("agent_actions"), kFS("failure_step_id"), kFA("failure_agent_did"), kRW("risk_weights"),
      kSucc("success"), kStep("step_id"), kAct("action_id");
  size_t ci = 0;
  for (py::handle c : cases) {
    py::dict cd = py::reinterpret_borrow<py::dict>(c);
    py::dict aa = py::reinterpret_borrow<py::dict>(cd[kAA]);
    py::object fstep = cd[kFS], fagent = cd[kFA];
    py::object rwo = cd.contains(kRW) ? py::object(cd[kRW]) : py::object(py::none());
    const bool has_rw = !rwo.is_none() && PyObject_IsTrue(rwo.ptr());
    // set(agent_actions.keys()) exactly: a set built from the dict itself is presized
    // and iterates in a different order than one built from the keys view
    py::object kview = aa.attr("keys")();
    py::set keys = py::reinterpret_steal<py::set>(PySet_New(kview.ptr()));
    if (!keys) throw py::error_already_set();
    py::list agents;
    std::unordered_map<PyObject*, int32_t> col;
    int32_t j = 0;
    for (py::handle k : keys) {  // set iteration order
      agents.append(k);
      col.emplace(k.ptr(), j++);
    }
    for (auto kv : aa) {
      py::handle agent = kv.first;
      auto it = col.find(agent.ptr());
      int32_t aj;
      if (it != col.end()) {
        aj = it->second;
      } else {  // equal key, different object: fall back to equality
        aj = -1;
        int32_t q = 0;
        for (py::handle k : agents) {
          if (k.equal(agent)) { aj = q; break; }
          ++q;
        }
      }
      const bool me = agent.equal(fagent);
      for (py::handle a : kv.second) {
        py::dict ad = py::reinterpret_borrow<py::dict>(a);
        agent_of.push_back(aj);
        py::object s = ad.contains(kSucc) ? py::object(ad[kSucc]) : py::object(py::bool_(true));
        const int t = PyObject_IsTrue(s.ptr());
        if (t < 0) throw py::error_already_set();
        succ.push_back(t ? 1 : 0);
        root.push_back(me && ad.contains(kStep) && py::object(ad[kStep]).equal(fstep) ? 1 : 0);
        double w = 0.5;
        if (has_rw) {
          py::object aid = ad.contains(kAct) ? py::object(ad[kAct]) : py::object(py::str(""));
          PyObject* v = PyDict_Check(rwo.ptr()) ? PyDict_GetItemWithError(rwo.ptr(), aid.ptr()) : nullptr;
          if (v == nullptr && PyErr_Occurred()) throw py::error_already_set();
          if (v != nullptr) w = py::reinterpret_borrow<py::object>(v).cast<double>();
          else if (!PyDict_Check(rwo.ptr())) w = py::float_(rwo.attr("get")(aid, 0.5)).cast<double>();
        }
        omega.push_back(w);
      }
    }
    node_off.push_back(static_cast<int32_t>(agent_of.size()));
    agent_off.push_back(agent_off.back() + static_cast<int32_t>(py::len(agents)));
    agents_per_case[ci++] = agents;
  }
  return py::make_tuple(as_bytes(node_off), as_bytes(agent_off), as_bytes(agent_of), as_bytes(succ), as_bytes(root),
                        as_bytes(omega), agents_per_case);
}

// Python's round(x, n) (correctly rounded decimal, half-even on the exact binary
// value) for many values at once: printf's %.*f rounds the exact value in the
// default rounding mode, and strtod reads the decimal back.
static py::list round_many(const std::vector<double>& xs, int n) {
  py::list out(xs.size());
  char buf[512];
  for (size_t i = 0; i < xs.size(); ++i) {
    const double x = xs[i];
    if (!std::isfinite(x) || std::fabs(x) >= 1e300) {
      out[i] = py::float_(x);
      continue;
    }
    std::snprintf(buf, sizeof buf, "%.*f", n, x);
    double y = std::strtod(buf, nullptr);
    if (y == 0.0) y = std::copysign(0.0, x);  // round(-0.00001, 4) is -0.0
    out[i] = py::float_(y);
  }
  return out;
}

void register_runtime(py::module_& m) {
  py::class_<StringPool>(m, "StringPool", "Host string interner feeding the device string pool")
      .def(py::init<>())
      .def("intern", static_cast<int32_t (StringPool::*)(const std::string&)>(&StringPool::intern))
      .def("intern_many", &StringPool::intern_many)
      .def("lookup", &StringPool::lookup)
      // bytes (UTF-8, lone surrogates in surrogatepass form): the Python wrapper decodes
      .def("str", [](const StringPool& p, int32_t id) { return py::bytes(p.str(id)); })
      .def("escaped", &StringPool::escaped)
      .def("bytes_view", &StringPool::bytes_view)
      .def("offsets_view", &StringPool::offsets_view)
      .def("lengths_view", &StringPool::lengths_view)
      .def_property_readonly("nbytes", &StringPool::nbytes)
      .def("__len__", &StringPool::size);
  m.def("pack_attribution", &pack_attribution, py::arg("cases"),
        "K21 columns + per-case agent lists (set order) of CausalAttributor.attribute_batch cases");
  m.def("round_many", &round_many, py::arg("xs"), py::arg("ndigits"), "[round(x, ndigits) for x in xs]");
  // The store's join decision (OP_SESS_JOIN: K01 ring gate + join_check) from the
  // same semantics.h predicates, for hosts that know the session row's state.
  m.def(
      "join_predict",
      [](int state, bool duplicate, int active, int max_participants, double sigma_eff, double min_sigma,
         bool trustworthy) {
        uint8_t ring = ring_from_sigma(sigma_eff, false);
        if (!trustworthy) ring = RING3;
        const uint8_t code = join_check(static_cast<uint8_t>(state), duplicate, active, max_participants, sigma_eff,
                                        min_sigma, ring);
        return py::make_tuple(static_cast<int>(code), static_cast<int>(ring));
      },
      py::arg("state"), py::arg("duplicate"), py::arg("active"), py::arg("max_participants"), py::arg("sigma_eff"),
      py::arg("min_sigma"), py::arg("trustworthy"), "(JoinCode, ring) the device join would produce");
  m.def("render_fragment", &render_fragment, py::arg("pool"), py::arg("changes"), py::arg("turn"),
        py::arg("has_parent"));
  m.def("frag_pack", &frag_pack, py::arg("pool"), py::arg("d_pool"), py::arg("ch_off"), py::arg("ch_rows"),
        "Distinct record heads ({\"agent_did\" ... \"delta:) of a batch's deltas, rendered once each");
  m.def("pack_specs", &pack_specs, py::arg("specs"), py::arg("agents"), py::arg("pool"), py::arg("cfg_of"),
        py::arg("fixed"), py::arg("threads") = -1,
        "Flatten PipelineSpecs into the batch kernels' columns (models/store_pipeline.py); threads: < 0 auto "
        "(AHV_PACK_THREADS), 1 serial");
  m.def("pack_walk_info", [] {
    return py::make_tuple(static_cast<bool>(AHV_PARALLEL_SPEC_WALK), std::string(g_last_walk));
  }, "(parallel walk compiled in for this Python, the last pack_specs call's walk)");
  m.def("iso_from_us", &iso_from_us, "datetime.isoformat() text of an epoch-µs UTC instant");
  m.def("uuids_from_counters", &uuids_from_counters, py::arg("seed"), py::arg("base"), py::arg("n"),
        py::arg("prefix") = std::string(), "uuid_from_counter(seed, base + i, prefix) for i < n");
  m.def("uuid_from_counter", &uuid_str, py::arg("seed"), py::arg("counter"), py::arg("prefix") = std::string(),
        "uuid4 string minted by the device id generator for (seed, counter)");
}

}  // namespace host
}  // namespace ahv
