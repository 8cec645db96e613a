// Host (scalar API path) audit primitives exposed to Python.
//
// These replace the reference's pure-Python hot spots:
//   * json.dumps(sort_keys) + hashlib over the SemanticDelta payload
//     (reference audit/delta.py:41-64)             -> delta_hash()
//   * level-wise hex-concatenation Merkle tree
//     (reference audit/delta.py:117-134)           -> merkle_root()
//   * sha256(content).hexdigest() for VFS edits
//     (reference session/sso.py:214-216)           -> sha256_hex()
//   * uuid4-based ids (3 per pipeline)             -> uuid4() / hex_id()
// The SHA-256 core is the shared host/device header ahv/sha256.h, so the scalar
// path and the batched gfx950 kernels hash with the same code.
#include <Python.h>
#include <datetime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "ahv/canon_json.h"
#include "ahv/host_sha.h"
#include "ahv/sha256.h"

namespace py = pybind11;

namespace ahv {
namespace host {

// ---------------------------------------------------------------- utilities

static inline void hex_of(const uint32_t d[8], char out[64]) {
  static const char* digits = "0123456789abcdef";
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = digits[(d[i] >> (28 - 4 * j)) & 15u];
}

static inline PyObject* hex_pystr(const uint32_t d[8]) {
  PyObject* s = PyUnicode_New(64, 127);
  if (!s) return nullptr;
  hex_of(d, reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s)));
  return s;
}

// Append the json.dumps(ensure_ascii=True) rendering of a Python str.
static void append_json_str(std::string& out, PyObject* s) {
  const Py_ssize_t n = PyUnicode_GET_LENGTH(s);
  out.push_back('"');
  if (PyUnicode_IS_ASCII(s)) {
    const char* p = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(s));
    Py_ssize_t run = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      const uint32_t c = static_cast<uint8_t>(p[i]);
      if (canon::json_plain(c)) { ++run; continue; }
      out.append(p + i - run, static_cast<size_t>(run));
      run = 0;
      switch (c) {
        case '"': out.append("\\\""); break;
        case '\\': out.append("\\\\"); break;
        case '\n': out.append("\\n"); break;
        case '\r': out.append("\\r"); break;
        case '\t': out.append("\\t"); break;
        case '\b': out.append("\\b"); break;
        case '\f': out.append("\\f"); break;
        default: {
          char buf[8];
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          out.append(buf, 6);
        }
      }
    }
    out.append(p + n - run, static_cast<size_t>(run));
  } else {
    const int kind = PyUnicode_KIND(s);
    const void* data = PyUnicode_DATA(s);
    for (Py_ssize_t i = 0; i < n; ++i) {
      const Py_UCS4 c = PyUnicode_READ(kind, data, i);
      if (canon::json_plain(c)) { out.push_back(static_cast<char>(c)); continue; }
      char buf[16];
      switch (c) {
        case '"': out.append("\\\""); break;
        case '\\': out.append("\\\\"); break;
        case '\n': out.append("\\n"); break;
        case '\r': out.append("\\r"); break;
        case '\t': out.append("\\t"); break;
        case '\b': out.append("\\b"); break;
        case '\f': out.append("\\f"); break;
        default:
          if (c > 0xffff) {  // UTF-16 surrogate pair, as CPython's encoder does
            const uint32_t v = c - 0x10000;
            std::snprintf(buf, sizeof buf, "\\u%04x\\u%04x", 0xd800 | ((v >> 10) & 0x3ff),
                          0xdc00 | (v & 0x3ff));
            out.append(buf, 12);
          } else {
            std::snprintf(buf, sizeof buf, "\\u%04x", static_cast<unsigned>(c));
            out.append(buf, 6);
          }
      }
    }
  }
  out.push_back('"');
}

// str -> json string, None -> null; anything else is unsupported here (the
// Python caller then falls back to json.dumps for exact parity on exotic types).
static bool append_json_opt_str(std::string& out, PyObject* v) {
  if (v == Py_None) { out.append(canon::K_NULL); return true; }
  if (PyUnicode_Check(v)) { append_json_str(out, v); return true; }
  return false;
}

struct Names {
  PyObject *delta_id, *turn_id, *session_id, *agent_did, *timestamp, *changes, *parent_hash;
  PyObject *path, *operation, *content_hash, *previous_hash, *isoformat, *delta_hash;
};
static Names* g_names = nullptr;

static Names* names() {
  if (!g_names) {
    g_names = new Names{
        PyUnicode_InternFromString("delta_id"),     PyUnicode_InternFromString("turn_id"),
        PyUnicode_InternFromString("session_id"),   PyUnicode_InternFromString("agent_did"),
        PyUnicode_InternFromString("timestamp"),    PyUnicode_InternFromString("changes"),
        PyUnicode_InternFromString("parent_hash"),  PyUnicode_InternFromString("path"),
        PyUnicode_InternFromString("operation"),    PyUnicode_InternFromString("content_hash"),
        PyUnicode_InternFromString("previous_hash"), PyUnicode_InternFromString("isoformat"),
        PyUnicode_InternFromString("delta_hash")};
  }
  return g_names;
}

struct Ref {  // minimal owning PyObject* holder
  PyObject* p;
  explicit Ref(PyObject* q) : p(q) {}
  ~Ref() { Py_XDECREF(p); }
  Ref(const Ref&) = delete;
  Ref& operator=(const Ref&) = delete;
};

// datetime.isoformat() for exact `datetime` objects whose tzinfo is the
// timezone.utc singleton; returns -1 for anything else (caller falls back to
// calling isoformat()).
static int utc_isoformat(PyObject* dt, char* out) {
  if (!PyDateTimeAPI) PyDateTime_IMPORT;
  if (!PyDateTimeAPI || !PyDateTime_CheckExact(dt)) return -1;
  if (PyDateTime_DATE_GET_TZINFO(dt) != PyDateTime_TimeZone_UTC) return -1;
  const int us = PyDateTime_DATE_GET_MICROSECOND(dt);
  int n = std::snprintf(out, 40, "%04d-%02d-%02dT%02d:%02d:%02d", PyDateTime_GET_YEAR(dt),
                        PyDateTime_GET_MONTH(dt), PyDateTime_GET_DAY(dt),
                        PyDateTime_DATE_GET_HOUR(dt), PyDateTime_DATE_GET_MINUTE(dt),
                        PyDateTime_DATE_GET_SECOND(dt));
  if (us) n += std::snprintf(out + n, 40 - n, ".%06d", us);
  std::memcpy(out + n, "+00:00", 6);
  return n + 6;
}

// Render the canonical payload of a SemanticDelta-like object.  Returns false
// (without a Python error set) when a field has a type json.dumps would render
// differently than this fast path; raises on attribute errors.
//
// With `null_parent_at` set, `parent_hash` is not read: the payload is rendered
// with a `null` parent and the byte offset of that `null` is stored, so the
// device store can splice the chain head's digest in (csrc/host/py_store.cpp).
bool render_delta_fields(PyObject* agent, PyObject* changes, PyObject* delta_id, PyObject* parent, PyObject* session,
                         PyObject* ts, PyObject* turn, std::string& out, size_t* null_parent_at);

bool render_delta(PyObject* d, std::string& out, size_t* null_parent_at = nullptr) {
  Names* nm = names();
  Ref agent(PyObject_GetAttr(d, nm->agent_did));
  Ref changes(PyObject_GetAttr(d, nm->changes));
  Ref delta_id(PyObject_GetAttr(d, nm->delta_id));
  Ref parent(null_parent_at ? (Py_INCREF(Py_None), Py_None) : PyObject_GetAttr(d, nm->parent_hash));
  Ref session(PyObject_GetAttr(d, nm->session_id));
  Ref ts(PyObject_GetAttr(d, nm->timestamp));
  Ref turn(PyObject_GetAttr(d, nm->turn_id));
  if (!agent.p || !changes.p || !delta_id.p || !parent.p || !session.p || !ts.p || !turn.p)
    throw py::error_already_set();
  return render_delta_fields(agent.p, changes.p, delta_id.p, parent.p, session.p, ts.p, turn.p, out, null_parent_at);
}

// The same rendering from the field values themselves (the native control plane
// renders a capture before its delta object exists: no attribute lookups).
bool render_delta_fields(PyObject* agent_p, PyObject* changes_p, PyObject* delta_id_p, PyObject* parent_p,
                         PyObject* session_p, PyObject* ts_p, PyObject* turn_p, std::string& out,
                         size_t* null_parent_at) {
  Names* nm = names();
  struct Field {
    PyObject* p;
  } agent{agent_p}, changes{changes_p}, delta_id{delta_id_p}, parent{parent_p}, session{session_p}, ts{ts_p},
      turn{turn_p};
  if (!PyLong_CheckExact(turn.p)) return false;
  char isobuf[40];
  int isolen = utc_isoformat(ts.p, isobuf);
  Ref iso(nullptr);
  if (isolen < 0) {
    iso.p = PyObject_CallMethodNoArgs(ts.p, nm->isoformat);
    if (!iso.p) throw py::error_already_set();
    if (!PyUnicode_Check(iso.p)) return false;
  }

  out.clear();
  out.reserve(320);
  out.append(canon::K_OPEN_AGENT);
  if (!append_json_opt_str(out, agent.p)) return false;
  out.append(canon::K_CHANGES);
  Ref seq(PySequence_Fast(changes.p, "changes must be a sequence"));
  if (!seq.p) throw py::error_already_set();
  const Py_ssize_t nc = PySequence_Fast_GET_SIZE(seq.p);
  PyObject** items = PySequence_Fast_ITEMS(seq.p);
  for (Py_ssize_t i = 0; i < nc; ++i) {
    if (i) out.append(canon::K_CH_SEP);
    PyObject* c = items[i];
    Ref ch(PyObject_GetAttr(c, nm->content_hash));
    Ref op(PyObject_GetAttr(c, nm->operation));
    Ref path(PyObject_GetAttr(c, nm->path));
    Ref prev(PyObject_GetAttr(c, nm->previous_hash));
    if (!ch.p || !op.p || !path.p || !prev.p) throw py::error_already_set();
    out.append(canon::K_CH_OPEN);
    if (!append_json_opt_str(out, ch.p)) return false;
    out.append(canon::K_CH_OP);
    if (!append_json_opt_str(out, op.p)) return false;
    out.append(canon::K_CH_PATH);
    if (!append_json_opt_str(out, path.p)) return false;
    out.append(canon::K_CH_PREV);
    if (!append_json_opt_str(out, prev.p)) return false;
    out.append(canon::K_CH_CLOSE);
  }
  out.append(canon::K_DELTA_ID);
  if (!append_json_opt_str(out, delta_id.p)) return false;
  out.append(canon::K_PARENT);
  if (null_parent_at) *null_parent_at = out.size();
  if (!append_json_opt_str(out, parent.p)) return false;
  out.append(canon::K_SESSION);
  if (!append_json_opt_str(out, session.p)) return false;
  out.append(canon::K_TS);
  if (isolen >= 0) {
    out.push_back('"');
    out.append(isobuf, static_cast<size_t>(isolen));
    out.push_back('"');
  } else {
    append_json_str(out, iso.p);
  }
  out.append(canon::K_TURN);
  int overflow = 0;
  const long long t = PyLong_AsLongLongAndOverflow(turn.p, &overflow);
  if (overflow) return false;
  out.append(std::to_string(t));
  out.append(canon::K_CLOSE);
  return true;
}

// ------------------------------------------------------------ Python API

// delta_payload(delta) -> bytes | None  (None = use the json.dumps fallback)
static py::object delta_payload(py::handle d) {
  std::string buf;
  if (!render_delta(d.ptr(), buf)) return py::none();
  return py::reinterpret_steal<py::object>(
      PyBytes_FromStringAndSize(buf.data(), static_cast<Py_ssize_t>(buf.size())));
}

// delta_hash(delta) -> str | None  (hex digest of the canonical payload)
static py::object delta_hash(py::handle d) {
  thread_local std::string buf;
  if (!render_delta(d.ptr(), buf)) return py::none();
  uint32_t h[8];
  sha256_bytes(reinterpret_cast<const uint8_t*>(buf.data()), buf.size(), h);
  return py::reinterpret_steal<py::object>(hex_pystr(h));
}

// Parse a 64-char lowercase/uppercase hex string into 8 words; false if not hex.
static bool parse_hex64(PyObject* s, uint32_t out[8]) {
  if (!PyUnicode_Check(s) || !PyUnicode_IS_ASCII(s) || PyUnicode_GET_LENGTH(s) != 64) return false;
  const uint8_t* p = PyUnicode_1BYTE_DATA(s);
  for (int i = 0; i < 8; ++i) {
    uint32_t v = 0;
    for (int j = 0; j < 8; ++j) {
      const uint8_t c = p[8 * i + j];
      uint32_t n;
      if (c >= '0' && c <= '9') n = c - '0';
      else if (c >= 'a' && c <= 'f') n = c - 'a' + 10;
      else return false;  // uppercase would hash to different ASCII: take slow path
      v = (v << 4) | n;
    }
    out[i] = v;
  }
  return true;
}

// merkle_root(hashes: list[str]) -> str | None
// Exact reference semantics: sha256(f"{left}{right}".encode()), odd node
// duplicated.  Canonical 64-hex leaves use the word-level node hash; any other
// leaf strings (tampered state) go through the byte-level path.
static py::object merkle_root(py::handle seq_h) {
  Ref seq(PySequence_Fast(seq_h.ptr(), "hashes must be a sequence"));
  if (!seq.p) throw py::error_already_set();
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq.p);
  if (n == 0) return py::none();
  PyObject** items = PySequence_Fast_ITEMS(seq.p);
  if (n == 1) return py::reinterpret_borrow<py::object>(items[0]);

  std::vector<uint32_t> level(static_cast<size_t>(n) * 8);
  bool canonical = true;
  for (Py_ssize_t i = 0; i < n && canonical; ++i) canonical = parse_hex64(items[i], &level[8 * i]);
  if (canonical) {
    size_t m = static_cast<size_t>(n);
    while (m > 1) {
      const size_t half = (m + 1) / 2;
      for (size_t i = 0; i < half; ++i) {
        const uint32_t* l = &level[16 * i];
        const uint32_t* r = (2 * i + 1 < m) ? &level[16 * i + 8] : l;
        uint32_t o[8];
        merkle_node_host(l, r, o);
        std::memcpy(&level[8 * i], o, sizeof o);
      }
      m = half;
    }
    return py::reinterpret_steal<py::object>(hex_pystr(level.data()));
  }
  // Byte-level path over arbitrary strings.
  std::vector<std::string> cur;
  cur.reserve(static_cast<size_t>(n));
  for (Py_ssize_t i = 0; i < n; ++i) {
    Py_ssize_t len = 0;
    const char* u = PyUnicode_AsUTF8AndSize(items[i], &len);
    if (!u) throw py::error_already_set();
    cur.emplace_back(u, static_cast<size_t>(len));
  }
  while (cur.size() > 1) {
    std::vector<std::string> next;
    for (size_t i = 0; i < cur.size(); i += 2) {
      const std::string& l = cur[i];
      const std::string& r = (i + 1 < cur.size()) ? cur[i + 1] : l;
      std::string cat = l + r;
      uint32_t h[8];
      sha256_bytes(reinterpret_cast<const uint8_t*>(cat.data()), cat.size(), h);
      char hex[64];
      hex_of(h, hex);
      next.emplace_back(hex, 64);
    }
    cur.swap(next);
  }
  return py::str(cur[0]);
}

// sha256_hex(str | bytes) -> str   (str is UTF-8 encoded, like str.encode())
// merkle_root_words(ptr, n) -> hex: the reference tree over n digests held as
// 8 native u32 words each (a CPU int32 [n, 8] tensor's data), with SHA-NI —
// the host oracle for the device K09 kernels on long chains.
static py::str merkle_root_words(uintptr_t ptr, int64_t n) {
  if (n <= 0) throw py::value_error("no leaves");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(ptr);
  std::vector<uint32_t> level(src, src + static_cast<size_t>(n) * 8);
  size_t m = static_cast<size_t>(n);
  {
    py::gil_scoped_release nogil;
    while (m > 1) {
      const size_t half = (m + 1) / 2;
      for (size_t i = 0; i < half; ++i) {
        const uint32_t* l = &level[16 * i];
        const uint32_t* r = (2 * i + 1 < m) ? &level[16 * i + 8] : l;
        uint32_t o[8];
        merkle_node_host(l, r, o);
        std::memcpy(&level[8 * i], o, sizeof o);
      }
      m = half;
    }
  }
  return py::reinterpret_steal<py::str>(hex_pystr(level.data()));
}

static py::object sha256_hex(py::handle v) {
  const char* p = nullptr;
  Py_ssize_t len = 0;
  if (PyUnicode_Check(v.ptr())) {
    p = PyUnicode_AsUTF8AndSize(v.ptr(), &len);
    if (!p) throw py::error_already_set();
  } else if (PyBytes_Check(v.ptr())) {
    p = PyBytes_AS_STRING(v.ptr());
    len = PyBytes_GET_SIZE(v.ptr());
  } else {
    throw py::type_error("sha256_hex expects str or bytes");
  }
  uint32_t h[8];
  sha256_bytes(reinterpret_cast<const uint8_t*>(p), static_cast<size_t>(len), h);
  return py::reinterpret_steal<py::object>(hex_pystr(h));
}

// ------------------------------------------------------------------ ids

// xoshiro256** seeded from the OS entropy source; one generator per thread.
struct IdRng {
  uint64_t s[4];
  IdRng() {
    std::random_device rd;
    for (auto& x : s) x = (uint64_t(rd()) << 32) ^ rd();
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
};
static thread_local IdRng g_rng;

static void put_hex(char* dst, uint64_t v, int nchars) {
  static const char* digits = "0123456789abcdef";
  for (int i = nchars - 1; i >= 0; --i) { dst[i] = digits[v & 15u]; v >>= 4; }
}

// uuid4(prefix="") -> prefix + canonical RFC-4122 version-4 uuid string
static py::object uuid4(const std::string& prefix) {
  uint64_t hi = g_rng.next(), lo = g_rng.next();
  hi = (hi & 0xffffffffffff0fffull) | 0x0000000000004000ull;  // version 4
  lo = (lo & 0x3fffffffffffffffull) | 0x8000000000000000ull;  // RFC variant
  const size_t pl = prefix.size();
  PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + 36), 127);
  if (!s) throw py::error_already_set();
  char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
  std::memcpy(o, prefix.data(), pl);
  o += pl;
  put_hex(o, hi >> 32, 8); o[8] = '-';
  put_hex(o + 9, (hi >> 16) & 0xffff, 4); o[13] = '-';
  put_hex(o + 14, hi & 0xffff, 4); o[18] = '-';
  put_hex(o + 19, lo >> 48, 4); o[23] = '-';
  put_hex(o + 24, lo & 0xffffffffffffull, 12);
  return py::reinterpret_steal<py::object>(s);
}

// prefix + a fresh uuid4 as a new str reference (nullptr on allocation failure),
// and the uuid's two halves: the native control plane's id minting (py_control.cpp).
PyObject* mint_uuid4(const char* prefix, size_t pl, uint64_t* hi_out, uint64_t* lo_out) {
  uint64_t hi = g_rng.next(), lo = g_rng.next();
  hi = (hi & 0xffffffffffff0fffull) | 0x0000000000004000ull;
  lo = (lo & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + 36), 127);
  if (!s) return nullptr;
  char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
  std::memcpy(o, prefix, pl);
  o += pl;
  put_hex(o, hi >> 32, 8); o[8] = '-';
  put_hex(o + 9, (hi >> 16) & 0xffff, 4); o[13] = '-';
  put_hex(o + 14, hi & 0xffff, 4); o[18] = '-';
  put_hex(o + 19, lo >> 48, 4); o[23] = '-';
  put_hex(o + 24, lo & 0xffffffffffffull, 12);
  if (hi_out) *hi_out = hi;
  if (lo_out) *lo_out = lo;
  return s;
}

// uuid4_id(prefix="") -> (prefix + uuid4 string, hi, lo): the uuid's two 64-bit
// halves as signed int64 (the store's session id words), no re-parse of the string.
static py::tuple uuid4_id(const std::string& prefix) {
  uint64_t hi = g_rng.next(), lo = g_rng.next();
  hi = (hi & 0xffffffffffff0fffull) | 0x0000000000004000ull;
  lo = (lo & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  const size_t pl = prefix.size();
  PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + 36), 127);
  if (!s) throw py::error_already_set();
  char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
  std::memcpy(o, prefix.data(), pl);
  o += pl;
  put_hex(o, hi >> 32, 8); o[8] = '-';
  put_hex(o + 9, (hi >> 16) & 0xffff, 4); o[13] = '-';
  put_hex(o + 14, hi & 0xffff, 4); o[18] = '-';
  put_hex(o + 19, lo >> 48, 4); o[23] = '-';
  put_hex(o + 24, lo & 0xffffffffffffull, 12);
  return py::make_tuple(py::reinterpret_steal<py::object>(s), static_cast<int64_t>(hi), static_cast<int64_t>(lo));
}

// uuid4_many(n, prefix) -> ([prefix + uuid4] * n, bytes of n×4 native u32 words):
// the words are the uuid's 32 hex digits as four big-endian 8-digit numbers
// (the layout of the store's s_uuid rows and of the device renderer).
static py::tuple uuid4_many(int64_t n, const std::string& prefix) {
  if (n < 0) throw py::value_error("n must be >= 0");
  py::list ids(n);
  std::string words(static_cast<size_t>(n) * 16, '\0');
  uint32_t* w = reinterpret_cast<uint32_t*>(words.data());
  const size_t pl = prefix.size();
  for (int64_t i = 0; i < n; ++i) {
    uint64_t hi = g_rng.next(), lo = g_rng.next();
    hi = (hi & 0xffffffffffff0fffull) | 0x0000000000004000ull;
    lo = (lo & 0x3fffffffffffffffull) | 0x8000000000000000ull;
    PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + 36), 127);
    if (!s) throw py::error_already_set();
    char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
    std::memcpy(o, prefix.data(), pl);
    o += pl;
    put_hex(o, hi >> 32, 8); o[8] = '-';
    put_hex(o + 9, (hi >> 16) & 0xffff, 4); o[13] = '-';
    put_hex(o + 14, hi & 0xffff, 4); o[18] = '-';
    put_hex(o + 19, lo >> 48, 4); o[23] = '-';
    put_hex(o + 24, lo & 0xffffffffffffull, 12);
    PyList_SET_ITEM(ids.ptr(), static_cast<Py_ssize_t>(i), s);
    w[4 * i + 0] = static_cast<uint32_t>(hi >> 32);
    w[4 * i + 1] = static_cast<uint32_t>(hi);
    w[4 * i + 2] = static_cast<uint32_t>(lo >> 32);
    w[4 * i + 3] = static_cast<uint32_t>(lo);
  }
  return py::make_tuple(ids, py::bytes(words));
}

// hex_id(prefix, nchars) -> prefix + nchars random lowercase hex digits
// (the reference's f"{prefix}{uuid.uuid4().hex[:n]}" id pattern).
static py::object hex_id(const std::string& prefix, int nchars) {
  if (nchars < 0 || nchars > 32) throw py::value_error("nchars must be in [0, 32]");
  const size_t pl = prefix.size();
  PyObject* s = PyUnicode_New(static_cast<Py_ssize_t>(pl + nchars), 127);
  if (!s) throw py::error_already_set();
  char* o = reinterpret_cast<char*>(PyUnicode_1BYTE_DATA(s));
  std::memcpy(o, prefix.data(), pl);
  const uint64_t a = g_rng.next(), b = g_rng.next();
  if (nchars <= 16) {
    put_hex(o + pl, a >> (64 - 4 * nchars), nchars);
  } else {
    put_hex(o + pl, a, 16);
    put_hex(o + pl + 16, b >> (64 - 4 * (nchars - 16)), nchars - 16);
  }
  return py::reinterpret_steal<py::object>(s);
}

// verify_chain_records(blob, rec_off, rec_len, hole, digest, sess_off, root, commit_n, threads)
//   -> (bad_chain bytes[N], bad_root bytes[N])
// K10 + K09 over audit records held in host memory (checkpoint restore, before
// they are written back): session i owns records [sess_off[i], sess_off[i+1]) in
// chain order.  A chain is good when every record hashes to its digest and
// record k > 0 quotes record k-1's digest at its parent hole (record 0: no hole);
// a committed session (commit_n > 0) needs root == the Merkle root of its first
// commit_n digests.  Sessions are split over `threads` host threads (SHA-NI).
static py::tuple verify_chain_records(py::buffer blob, py::array_t<int64_t, py::array::c_style | py::array::forcecast> off,
                                      py::array_t<int64_t, py::array::c_style | py::array::forcecast> len,
                                      py::array_t<int32_t, py::array::c_style | py::array::forcecast> hole,
                                      py::array_t<uint32_t, py::array::c_style | py::array::forcecast> dig,
                                      py::array_t<int64_t, py::array::c_style | py::array::forcecast> soff,
                                      py::array_t<uint32_t, py::array::c_style | py::array::forcecast> root,
                                      py::array_t<int32_t, py::array::c_style | py::array::forcecast> commit_n,
                                      int threads) {
  const py::buffer_info bi = blob.request();
  const uint8_t* b = static_cast<const uint8_t*>(bi.ptr);
  const int64_t bn = static_cast<int64_t>(bi.size * bi.itemsize);
  const int64_t nrec = off.size();
  const int64_t ns = soff.size() - 1;
  if (len.size() != nrec || hole.size() != nrec || dig.size() != 8 * nrec || ns < 0 || root.size() != 8 * ns ||
      commit_n.size() != ns)
    throw py::value_error("verify_chain_records: inconsistent array sizes");
  const int64_t* po = off.data();
  const int64_t* pl = len.data();
  const int32_t* ph = hole.data();
  const uint32_t* pd = dig.data();
  const int64_t* so = soff.data();
  const uint32_t* pr = root.data();
  const int32_t* pc = commit_n.data();
  if (ns > 0 && (so[0] < 0 || so[ns] > nrec)) throw py::value_error("verify_chain_records: session offsets out of range");
  for (int64_t i = 0; i < ns; ++i)
    if (so[i + 1] < so[i]) throw py::value_error("verify_chain_records: session offsets decrease");
  std::string bad_chain(static_cast<size_t>(ns), '\0'), bad_root(static_cast<size_t>(ns), '\0');
  auto work = [&](int64_t s0, int64_t s1) {
    std::vector<uint32_t> level;
    for (int64_t s = s0; s < s1; ++s) {
      bool ok = true;
      for (int64_t r = so[s]; r < so[s + 1] && ok; ++r) {
        const int64_t k = r - so[s];
        if (po[r] < 0 || pl[r] < 0 || po[r] + pl[r] > bn) { ok = false; break; }
        const uint8_t* rec = b + po[r];
        uint32_t h[8];
        sha256_bytes(rec, static_cast<size_t>(pl[r]), h);
        ok = std::memcmp(h, pd + 8 * r, 32) == 0;
        if (!ok) break;
        if (k == 0) {
          ok = ph[r] < 0;
        } else {
          const int64_t at = ph[r];
          if (at < 0 || at + 66 > pl[r]) { ok = false; break; }
          uint8_t q[64];
          hex_bytes(pd + 8 * (r - 1), q);
          ok = rec[at] == '"' && rec[at + 65] == '"' && std::memcmp(rec + at + 1, q, 64) == 0;
        }
      }
      bad_chain[static_cast<size_t>(s)] = ok ? 0 : 1;
      const int64_t m0 = pc[s];
      if (m0 > 0) {
        if (m0 > so[s + 1] - so[s]) { bad_root[static_cast<size_t>(s)] = 1; continue; }
        level.assign(pd + 8 * so[s], pd + 8 * (so[s] + m0));
        size_t m = static_cast<size_t>(m0);
        while (m > 1) {
          const size_t half = (m + 1) / 2;
          for (size_t i = 0; i < half; ++i) {
            const uint32_t* l = &level[16 * i];
            const uint32_t* rr = (2 * i + 1 < m) ? &level[16 * i + 8] : l;
            uint32_t o[8];
            merkle_node_host(l, rr, o);
            std::memcpy(&level[8 * i], o, sizeof o);
          }
          m = half;
        }
        bad_root[static_cast<size_t>(s)] = std::memcmp(level.data(), pr + 8 * s, 32) == 0 ? 0 : 1;
      }
    }
  };
  {
    py::gil_scoped_release nogil;
    const int nt = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(threads, (ns + 1023) / 1024)));
    std::vector<std::thread> pool;
    const int64_t per = (ns + nt - 1) / std::max(nt, 1);
    for (int t = 1; t < nt; ++t) {
      const int64_t a = std::min(ns, t * per), z = std::min(ns, (t + 1) * per);
      if (a < z) pool.emplace_back(work, a, z);
    }
    work(0, std::min(ns, per));
    for (auto& th : pool) th.join();
  }
  return py::make_tuple(py::bytes(bad_chain), py::bytes(bad_root));
}

void register_audit(py::module_& m) {
  m.def("verify_chain_records", &verify_chain_records, py::arg("blob"), py::arg("rec_off"), py::arg("rec_len"),
        py::arg("hole"), py::arg("digest"), py::arg("sess_off"), py::arg("root"), py::arg("commit_n"),
        py::arg("threads") = 8, "K10 chains + K09 roots over host-held audit records (checkpoint restore)");
  m.def("delta_payload", &delta_payload, "Canonical JSON payload bytes of a SemanticDelta");
  m.def("delta_hash", &delta_hash, "SHA-256 hex of the canonical SemanticDelta payload");
  m.def("merkle_root", &merkle_root, "Merkle root over hex leaf hashes (reference semantics)");
  m.def("merkle_root_words", &merkle_root_words, py::arg("ptr"), py::arg("n"),
        "Merkle root over n digests given as native u32 words (host SHA-NI oracle)");
  m.def("sha256_hex", &sha256_hex, "SHA-256 hex digest of str (UTF-8) or bytes");
  m.def("uuid4", &uuid4, py::arg("prefix") = std::string(), "prefix + random uuid4 string");
  m.def("uuid4_id", &uuid4_id, py::arg("prefix") = std::string(),
        "(prefix + random uuid4 string, hi, lo) with the halves as signed int64");
  m.def("hex_id", &hex_id, py::arg("prefix"), py::arg("nchars"), "prefix + random hex digits");
  m.def("uuid4_many", &uuid4_many, py::arg("n"), py::arg("prefix") = std::string(),
        "n uuid4 strings and their 4 u32 words each");
}

}  // namespace host
}  // namespace ahv
