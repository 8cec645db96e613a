// Host runtime pieces of the device engine:
//   * StringPool — the DID / path / id string interner: dense int32
//     ids for device tables, a reverse table, and each string's canonical-JSON
//     escaped body stored contiguously so kernels can splice it into the audit
//     payload without re-escaping (ahv/delta_emit.h StrPool).
//   * time base helpers (N09): epoch-µs ↔ ISO text with the exact
//     datetime.isoformat() rendering used in delta hashes.
#include <Python.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "ahv/delta_emit.h"
#include "ahv/semantics.h"

namespace py = pybind11;

namespace ahv {
namespace host {

// json.dumps(ensure_ascii=True) body (no quotes) of a UTF-8 string.
static void escape_json_utf8(const std::string& in, std::vector<uint8_t>& out) {
  auto put = [&](const char* s, size_t n) { out.insert(out.end(), s, s + n); };
  size_t i = 0;
  const size_t n = in.size();
  while (i < n) {
    uint32_t c = static_cast<uint8_t>(in[i]);
    size_t adv = 1;
    if (c >= 0x80) {  // decode UTF-8 (input is produced by CPython, so well-formed)
      if ((c & 0xe0) == 0xc0) { c = ((c & 0x1f) << 6) | (in[i + 1] & 0x3f); adv = 2; }
      else if ((c & 0xf0) == 0xe0) { c = ((c & 0x0f) << 12) | ((in[i + 1] & 0x3f) << 6) | (in[i + 2] & 0x3f); adv = 3; }
      else { c = ((c & 0x07) << 18) | ((in[i + 1] & 0x3f) << 12) | ((in[i + 2] & 0x3f) << 6) | (in[i + 3] & 0x3f); adv = 4; }
    }
    i += adv;
    if (canon::json_plain(c)) { out.push_back(static_cast<uint8_t>(c)); continue; }
    char buf[16];
    switch (c) {
      case '"': put("\\\"", 2); break;
      case '\\': put("\\\\", 2); break;
      case '\n': put("\\n", 2); break;
      case '\r': put("\\r", 2); break;
      case '\t': put("\\t", 2); break;
      case '\b': put("\\b", 2); break;
      case '\f': put("\\f", 2); break;
      default:
        if (c > 0xffff) {
          const uint32_t v = c - 0x10000;
          std::snprintf(buf, sizeof buf, "\\u%04x\\u%04x", 0xd800 | ((v >> 10) & 0x3ff), 0xdc00 | (v & 0x3ff));
          put(buf, 12);
        } else {
          std::snprintf(buf, sizeof buf, "\\u%04x", c);
          put(buf, 6);
        }
    }
  }
}

class StringPool {
 public:
  int32_t intern(const std::string& s) {
    auto it = ids_.find(s);
    if (it != ids_.end()) return it->second;
    const int32_t id = static_cast<int32_t>(raw_.size());
    ids_.emplace(s, id);
    raw_.push_back(s);
    // every string starts 16-byte aligned so kernels read it with 16-byte loads
    bytes_.resize((bytes_.size() + 15) & ~size_t(15), 0);
    offsets_.push_back(static_cast<int64_t>(bytes_.size()));
    const size_t before = bytes_.size();
    escape_json_utf8(s, bytes_);
    lengths_.push_back(static_cast<int32_t>(bytes_.size() - before));
    // keep the pool a multiple of 16 bytes: kernels read whole 16-byte chunks
    bytes_.resize((bytes_.size() + 15) & ~size_t(15), 0);
    return id;
  }

  std::vector<int32_t> intern_many(const std::vector<std::string>& v) {
    std::vector<int32_t> out;
    out.reserve(v.size());
    for (const auto& s : v) out.push_back(intern(s));
    return out;
  }

  int32_t lookup(const std::string& s) const {
    auto it = ids_.find(s);
    return it == ids_.end() ? -1 : it->second;
  }

  const std::string& str(int32_t id) const {
    if (id < 0 || static_cast<size_t>(id) >= raw_.size()) throw py::index_error("string id out of range");
    return raw_[static_cast<size_t>(id)];
  }

  size_t size() const { return raw_.size(); }
  size_t nbytes() const { return bytes_.size(); }

  py::bytes escaped(int32_t id) const {
    str(id);
    return py::bytes(reinterpret_cast<const char*>(bytes_.data()) + offsets_[id], lengths_[id]);
  }

  // Zero-copy views (valid until the next intern call).
  py::memoryview bytes_view() const {
    return py::memoryview::from_memory(bytes_.data(), static_cast<py::ssize_t>(bytes_.size()));
  }
  py::memoryview offsets_view() const {
    return py::memoryview::from_memory(offsets_.data(), static_cast<py::ssize_t>(offsets_.size() * 8));
  }
  py::memoryview lengths_view() const {
    return py::memoryview::from_memory(lengths_.data(), static_cast<py::ssize_t>(lengths_.size() * 4));
  }

 private:
  std::unordered_map<std::string, int32_t> ids_;
  std::vector<std::string> raw_;
  std::vector<uint8_t> bytes_;
  std::vector<int64_t> offsets_;
  std::vector<int32_t> lengths_;
};

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

void register_runtime(py::module_& m) {
  py::class_<StringPool>(m, "StringPool", "Host string interner feeding the device string pool")
      .def(py::init<>())
      .def("intern", &StringPool::intern)
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
  m.def("iso_from_us", &iso_from_us, "datetime.isoformat() text of an epoch-µs UTC instant");
  m.def("uuid_from_counter", &uuid_str, py::arg("seed"), py::arg("counter"), py::arg("prefix") = std::string(),
        "uuid4 string minted by the device id generator for (seed, counter)");
}

}  // namespace host
}  // namespace ahv
