// Host string interner shared by the runtime bindings and the native control
// plane: dense int32 ids for device tables, a reverse table, and
// each string's canonical-JSON escaped body stored contiguously so kernels can
// splice it into audit payloads without re-escaping (ahv/delta_emit.h StrPool).
#pragma once

#include <pybind11/pybind11.h>

#include <cstdio>
#include <deque>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "ahv/canon_json.h"
#include "ahv/delta_emit.h"

namespace ahv {
namespace host {

// json.dumps(ensure_ascii=True) body (no quotes) of a UTF-8 string.
inline void escape_json_utf8(const std::string& in, std::vector<uint8_t>& out) {
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
  int32_t intern(const std::string& s) { return intern(std::string_view(s)); }

  // Lookup without building a std::string (keys are views of the stable raw_
  // entries: a deque never moves its elements).
  int32_t intern(std::string_view s) {
    auto it = ids_.find(s);
    if (it != ids_.end()) return it->second;
    const int32_t id = static_cast<int32_t>(raw_.size());
    raw_.emplace_back(s);
    ids_.emplace(std::string_view(raw_.back()), id);
    // every string starts 16-byte aligned so kernels read it with 16-byte loads
    bytes_.resize((bytes_.size() + 15) & ~size_t(15), 0);
    offsets_.push_back(static_cast<int64_t>(bytes_.size()));
    const size_t before = bytes_.size();
    escape_json_utf8(raw_.back(), bytes_);
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
    auto it = ids_.find(std::string_view(s));
    return it == ids_.end() ? -1 : it->second;
  }

  const std::string& str(int32_t id) const {
    if (id < 0 || static_cast<size_t>(id) >= raw_.size()) throw pybind11::index_error("string id out of range");
    return raw_[static_cast<size_t>(id)];
  }

  int32_t esc_len(int32_t id) const { return lengths_[static_cast<size_t>(id)]; }
  size_t size() const { return raw_.size(); }
  // The pool as the emitters read it (host memory; valid until the next intern).
  StrPool str_pool() const { return StrPool{bytes_.data(), offsets_.data(), lengths_.data()}; }
  size_t nbytes() const { return bytes_.size(); }

  pybind11::bytes escaped(int32_t id) const {
    str(id);
    return pybind11::bytes(reinterpret_cast<const char*>(bytes_.data()) + offsets_[id], lengths_[id]);
  }

  // Zero-copy views (valid until the next intern call).
  pybind11::memoryview bytes_view() const {
    return pybind11::memoryview::from_memory(bytes_.data(), static_cast<pybind11::ssize_t>(bytes_.size()));
  }
  pybind11::memoryview offsets_view() const {
    return pybind11::memoryview::from_memory(offsets_.data(), static_cast<pybind11::ssize_t>(offsets_.size() * 8));
  }
  pybind11::memoryview lengths_view() const {
    return pybind11::memoryview::from_memory(lengths_.data(), static_cast<pybind11::ssize_t>(lengths_.size() * 4));
  }

 private:
  std::unordered_map<std::string_view, int32_t> ids_;
  std::deque<std::string> raw_;
  std::vector<uint8_t> bytes_;
  std::vector<int64_t> offsets_;
  std::vector<int32_t> lengths_;
};

}  // namespace host
}  // namespace ahv
