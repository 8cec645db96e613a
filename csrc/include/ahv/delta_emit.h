// Canonical SemanticDelta payload emission into a hashing "sink".
//
// One emitter, two sinks:
//   * HostSink        — streams bytes into SHA-256 (host twin / CPU tests);
//   * WordWindowSink  — (ahv/wave_sink.h) assembles a window of each lane's
//     message in LDS, a 32-bit word at a time, and compresses it on the device.
//
// Emitter contract: before writing a segment the emitter calls `s.seg(len)`
// with the segment's exact byte length; a false answer means the sink skipped
// the segment (its bytes are outside the current window) and nothing is written.
// Bytes are handed over in big-endian chunks: `put4(v)` = 4 bytes, `put(v, n)`
// = the top n ∈ [0, 4] bytes of v (the rest of v zero; n may differ per lane).
//
// Byte-exact with json.dumps(sort_keys=True) of the reference payload
// (audit/delta.py:43-63); pool strings are stored pre-escaped (JSON body without
// quotes) by the host interner (agent_hypervisor_amd/utils/interner.py).
#pragma once

#include <vector>

#include "ahv/canon_json.h"
#include "ahv/sha256.h"

namespace ahv {

// Interned string pool: id -> JSON-escaped bytes (no surrounding quotes).
struct StrPool {
  const uint8_t* bytes;
  const int64_t* off;
  const int32_t* len;
};

// civil-from-days (proleptic Gregorian), days since 1970-01-01.
AHV_HD void civil_from_days(int64_t z, int32_t& y, uint32_t& m, uint32_t& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const uint32_t doe = static_cast<uint32_t>(z - era * 146097);
  const uint32_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const uint32_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const uint32_t mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = static_cast<int32_t>(yoe) + static_cast<int32_t>(era) * 400 + (m <= 2 ? 1 : 0);
}

// Broken-down UTC instant.
struct UtcParts {
  uint32_t year, month, day, secs, micro;
};

AHV_HD UtcParts utc_parts(int64_t us) {
  int64_t days = us / 86400000000LL;
  int64_t rem = us - days * 86400000000LL;
  if (rem < 0) { rem += 86400000000LL; --days; }
  int32_t y; uint32_t mo, d;
  civil_from_days(days, y, mo, d);
  return UtcParts{static_cast<uint32_t>(y), mo, d, static_cast<uint32_t>(rem / 1000000),
                  static_cast<uint32_t>(rem % 1000000)};
}

// Host helper: datetime.isoformat() text of an epoch-µs UTC instant.
AHV_HD uint32_t iso_utc(int64_t us, uint8_t* out) {
  const UtcParts t = utc_parts(us);
  uint32_t n = 0;
  auto d2 = [&](uint32_t v) { out[n++] = '0' + v / 10; out[n++] = '0' + v % 10; };
  d2((t.year / 100) % 100); d2(t.year % 100);
  out[n++] = '-'; d2(t.month); out[n++] = '-'; d2(t.day);
  out[n++] = 'T'; d2(t.secs / 3600); out[n++] = ':'; d2((t.secs / 60) % 60); out[n++] = ':'; d2(t.secs % 60);
  if (t.micro) { out[n++] = '.'; d2(t.micro / 10000); d2((t.micro / 100) % 100); d2(t.micro % 100); }
  out[n++] = '+'; out[n++] = '0'; out[n++] = '0'; out[n++] = ':'; out[n++] = '0'; out[n++] = '0';
  return n;
}

// ---------------------------------------------------------------- host sink

struct HostSink {
  Sha256Stream h;
  uint32_t scratch[8][8];
  AHV_HD bool seg(uint32_t) { return true; }
  AHV_HD void put4(uint32_t v) {
    for (int j = 0; j < 4; ++j) h.put(static_cast<uint8_t>(v >> (24 - 8 * j)));
  }
  AHV_HD void put(uint32_t v, uint32_t n) {
    for (uint32_t j = 0; j < n; ++j) h.put(static_cast<uint8_t>(v >> (24 - 8 * j)));
  }
  AHV_HD bool any(bool b) const { return b; }
  template <class T>
  AHV_HD void launder(T&) const {}
  template <class Emit>
  AHV_HD void hash(Emit&& emit, uint32_t out[8]) {
    h.init();
    emit(*this);
    h.final(out);
  }
  // The host streams every byte; the midstate modes only change the device's
  // work, never the digest, so the host twin ignores them.
  template <class Emit, class Mid>
  AHV_HD void hash_mid(Emit&& emit, uint32_t out[8], Mid&, int) {
    hash(emit, out);
  }
  // Resume from a midstate taken after `base_bytes` (multiple of 64) that the
  // emitter does not replay (see WordWindowSink::hash_from).
  template <class Emit>
  AHV_HD void hash_from(Emit&& emit, const uint32_t st_in[8], uint32_t base_bytes, uint32_t out[8]) {
    h.init();
    for (int k = 0; k < 8; ++k) h.st[k] = st_in[k];
    h.total = base_bytes;
    emit(*this);
    h.final(out);
  }
  AHV_HD void stash(int j, const uint32_t d[8]) {
    for (int k = 0; k < 8; ++k) scratch[j][k] = d[k];
  }
  AHV_HD void load(int j, uint32_t d[8]) const {
    for (int k = 0; k < 8; ++k) d[k] = scratch[j][k];
  }
  AHV_HD void node(const uint32_t l[8], const uint32_t r[8], uint32_t out[8]) const {
    uint32_t t[8];  // out may alias l or r
    merkle_node(l, r, t);
    for (int k = 0; k < 8; ++k) out[k] = t[k];
  }
};

// Merkle root of `n` leaves read by `leaf(i, out)`, with the reference's level-wise
// odd-node duplication (audit/delta.py:117-134), computed as a binary counter:
// after k leaves the sink's scratch slot L holds the subtree of level L for every
// set bit L of k, so only ⌊log2 n⌋+1 digests are ever stored.  At the end the
// partial subtrees are folded from the lowest level up; a subtree that is short
// of its left neighbour's level is first self-paired (H(x, x)) once per missing
// level, which is exactly what the level-wise algorithm does to the last node of
// every odd level.
template <class Sink, class Leaf>
AHV_HD void merkle_root_counter(Sink& s, uint32_t n, Leaf&& leaf, uint32_t root[8]) {
  for (uint32_t k = 0; k < n; ++k) {
    uint32_t carry[8];
    leaf(k, carry);
    uint32_t lvl = 0;
    while ((k >> lvl) & 1u) {
      uint32_t left[8];
      s.load(static_cast<int>(lvl), left);
      s.node(left, carry, carry);
      ++lvl;
    }
    s.stash(static_cast<int>(lvl), carry);
  }
  uint32_t lvl = 0;
  while (!((n >> lvl) & 1u)) ++lvl;
  s.load(static_cast<int>(lvl), root);
  uint32_t cur = lvl;
  for (uint32_t L = lvl + 1; (n >> L) != 0; ++L) {
    if (!((n >> L) & 1u)) continue;
    for (; cur < L; ++cur) s.node(root, root, root);
    uint32_t left[8];
    s.load(static_cast<int>(L), left);
    s.node(left, root, root);
    cur = L + 1;
  }
}

// Level-wise Merkle root of `n` leaves read by `leaf(i, out)` (reference
// audit/delta.py:117-134: odd node duplicated), with every interior node hashed
// at ONE call site: level 1 reads the leaves, later levels work in place on the
// sink's scratch slots (node j overwrites slot j after reading 2j and 2j+1).
// Needs ⌈n/2⌉ scratch slots.
template <class Sink, class Leaf>
AHV_HD void merkle_root_levels(Sink& s, uint32_t n, Leaf&& leaf, uint32_t root[8]) {
  if (n == 1) {
    leaf(0, root);
    return;
  }
  uint32_t m = n;
  bool from_leaves = true;
  while (m > 1) {
    const uint32_t half = (m + 1) >> 1;
#pragma nounroll
    for (uint32_t j = 0; j < half; ++j) {
      const uint32_t ri = 2 * j + 1 < m ? 2 * j + 1 : 2 * j;
      uint32_t l[8], r[8], o[8];
      if (from_leaves) {
        leaf(2 * j, l);
        leaf(ri, r);
      } else {
        s.load(static_cast<int>(2 * j), l);
        s.load(static_cast<int>(ri), r);
      }
      s.node(l, r, o);
      s.stash(static_cast<int>(j), o);
    }
    m = half;
    from_leaves = false;
  }
  s.load(0, root);
}

// Level-wise Merkle root over `m` (≤ 8) digests stashed in the sink's scratch
// slots 0..m-1 (reference audit/delta.py:117-134: odd node duplicated).
template <class Sink>
AHV_HD void merkle_root_stashed(Sink& s, int m, uint32_t root[8]) {
  while (m > 1) {
    const int half = (m + 1) >> 1;
    for (int j = 0; j < half; ++j) {
      uint32_t l[8], r[8], o[8];
      s.load(2 * j, l);
      s.load((2 * j + 1 < m) ? 2 * j + 1 : 2 * j, r);
      s.node(l, r, o);
      s.stash(j, o);
    }
    m = half;
  }
  s.load(0, root);
}

// ------------------------------------------------------------ emission API

// Byte i of a literal as the top byte of a word (0 past the end).
template <size_t N>
AHV_HD constexpr uint32_t lit_byte(const char (&lit)[N], size_t i) {
  return i < N - 1 ? static_cast<uint32_t>(static_cast<uint8_t>(lit[i])) : 0u;
}

// A compile-time literal as whole big-endian words plus a tail chunk (after
// inlining every word is an immediate).
template <class Sink, size_t N>
AHV_HD void emit_lit(Sink& s, const char (&lit)[N]) {
  constexpr uint32_t n = static_cast<uint32_t>(N - 1);
  // A short literal is cheaper to emit than to test against the window (its
  // out-of-window words land in the trash row); longer ones are skipped whole.
  if (n > 8 && !s.seg(n)) return;
#pragma unroll
  for (uint32_t i = 0; i + 4 <= n; i += 4)
    s.put4(lit_byte(lit, i) << 24 | lit_byte(lit, i + 1) << 16 | lit_byte(lit, i + 2) << 8 | lit_byte(lit, i + 3));
  constexpr uint32_t t = n & 3u;
  if (t) {
    const uint32_t i = n & ~3u;
    s.put(lit_byte(lit, i) << 24 | lit_byte(lit, i + 1) << 16 | lit_byte(lit, i + 2) << 8, t);
  }
}

// One ASCII byte (a segment of its own).
template <class Sink>
AHV_HD void emit_char(Sink& s, uint32_t c) {
  if (s.seg(1)) s.put(c << 24, 1);
}

// A resolved pool string: 16-byte aligned pointer + length (-1 = null).
struct StrRef {
  const uint8_t* p;
  int32_t n;
};

AHV_HD StrRef pool_ref(const StrPool& pool, int32_t id) {
  if (id < 0) return StrRef{nullptr, -1};
  return StrRef{pool.bytes + pool.off[id], pool.len[id]};
}

struct alignas(16) U4 {
  uint32_t a, b, c, d;
};

AHV_HD uint32_t bswap_word(uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(0u, w, 0x00010203u);
#else
  return bswap32(w);
#endif
}

// Top `cnt` bytes (clamped to [0, 4]) of a little-endian memory word, in memory order.
template <class Sink>
AHV_HD void emit_word_le(Sink& s, uint32_t w, int32_t cnt) {
  const uint32_t m = cnt <= 0 ? 0u : (cnt >= 4 ? 4u : static_cast<uint32_t>(cnt));
  const uint32_t keep = m >= 4u ? 0xffffffffu : ~(0xffffffffu >> (8u * m));
  s.put(bswap_word(w) & keep, m);
}

// Quoted string body from 16-byte aligned storage, 16 bytes per load; the byte
// count may differ per lane (lanes past their end hand over zero bytes).
template <class Sink>
AHV_HD void emit_str_ref(Sink& s, StrRef r) {
  if (r.n < 0) {
    emit_lit(s, canon::K_NULL);
    return;
  }
  const uint32_t n = static_cast<uint32_t>(r.n);
  if (!s.seg(n + 2)) return;
  s.put(0x22u << 24, 1);
  const U4* q = reinterpret_cast<const U4*>(r.p);
  const uint32_t full = n / 16;
  // whole 16-byte chunks as four 4-byte puts (one v_alignbit each in the sink);
  // four named words, no indexing into the chunk (a runtime index would put it
  // in scratch memory on the device)
  for (uint32_t c = 0; c < full; ++c) {
    const U4 cur = q[c];
    s.put4(bswap_word(cur.a));
    s.put4(bswap_word(cur.b));
    s.put4(bswap_word(cur.c));
    s.put4(bswap_word(cur.d));
  }
  if (n & 15u) {
    const U4 cur = q[full];
    const int32_t left = static_cast<int32_t>(n & 15u);
    emit_word_le(s, cur.a, left);
    emit_word_le(s, cur.b, left - 4);
    emit_word_le(s, cur.c, left - 8);
    emit_word_le(s, cur.d, left - 12);
  }
  s.put(0x22u << 24, 1);
}

// Raw bytes [p, p+n) (already JSON text) as one segment, read as aligned 32-bit
// words and funnel-shifted to the span's byte offset.  Never reads past the word
// holding the span's last byte.
template <class Sink>
AHV_HD void emit_span(Sink& s, const uint8_t* p, uint32_t n) {
  if (!s.seg(n) || n == 0) return;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
  const uint32_t sh = static_cast<uint32_t>(a & 3u) * 8u;
  const uint32_t words = (n + (sh >> 3) + 3u) >> 2;  // aligned words touched
  auto funnel = [sh](uint32_t lo, uint32_t hi) -> uint32_t {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
#endif
  };
  uint32_t cur = w[0];
  const uint32_t full = n >> 2;
  // whole 4-byte chunks: the cheap funnel put (one v_alignbit in the sink)
  for (uint32_t k = 0; k < full; ++k) {
    const uint32_t nxt = k + 1 < words ? w[k + 1] : 0u;
    s.put4(bswap_word(funnel(cur, nxt)));
    cur = nxt;
  }
  if (n & 3u) {
    const uint32_t nxt = full + 1 < words ? w[full + 1] : 0u;
    s.put(bswap_word(funnel(cur, nxt)), n & 3u);
  }
}

// emit_span with loads issued `P` words ahead: for long spans read from HBM by a
// lane whose neighbours read unrelated addresses (chain re-hash of arena
// payloads), P independent loads are in flight before the first is consumed
// instead of one dependent load per 4 bytes.  Same bytes, same sink calls.
template <int P, class Sink>
AHV_HD void emit_span_prefetch(Sink& s, const uint8_t* p, uint32_t n) {
  if (!s.seg(n) || n == 0) return;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~static_cast<uintptr_t>(3));
  const uint32_t sh = static_cast<uint32_t>(a & 3u) * 8u;
  const uint32_t words = (n + (sh >> 3) + 3u) >> 2;
  auto funnel = [sh](uint32_t lo, uint32_t hi) -> uint32_t {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return sh ? (lo >> sh) | (hi << (32u - sh)) : lo;
#endif
  };
  uint32_t cur = w[0];
  const uint32_t full = n >> 2;
  uint32_t k = 0;
  for (; k + P <= full; k += P) {
    uint32_t nx[P];
#pragma unroll
    for (int j = 0; j < P; ++j) nx[j] = k + 1 + j < words ? w[k + 1 + j] : 0u;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      s.put4(bswap_word(funnel(cur, nx[j])));
      cur = nx[j];
    }
  }
  for (; k < full; ++k) {
    const uint32_t nxt = k + 1 < words ? w[k + 1] : 0u;
    s.put4(bswap_word(funnel(cur, nxt)));
    cur = nxt;
  }
  if (n & 3u) {
    const uint32_t nxt = full + 1 < words ? w[full + 1] : 0u;
    s.put(bswap_word(funnel(cur, nxt)), n & 3u);
  }
}

// Pool string id as a JSON value: "…" or null.
template <class Sink>
AHV_HD void emit_pool_str(Sink& s, const StrPool& pool, int32_t id) {
  emit_str_ref(s, pool_ref(pool, id));
}

// Decimal digits, most significant first (no local digit array: an array indexed
// by a runtime position would live in scratch memory on the device).
template <class Sink>
AHV_HD void emit_uint(Sink& s, uint64_t v) {
  // turn numbers and counts: one or two digits in one put, 32-bit arithmetic (the
  // general form divides 64-bit values by a variable power of ten, a long
  // instruction sequence on the device, twice per rendered record)
  if (v < 100u) {
    const uint32_t x = static_cast<uint32_t>(v);
    if (x < 10u) {
      if (s.seg(1)) s.put(('0' + x) << 24, 1);
    } else if (s.seg(2)) {
      const uint32_t t = x / 10u;
      s.put((('0' + t) << 24) | (('0' + x - 10u * t) << 16), 2);
    }
    return;
  }
  if (!s.seg(canon::dec_digits(v))) return;
  uint64_t p = 1;
  while (v / p >= 10) p *= 10;
  for (; p; p /= 10) s.put(static_cast<uint32_t>('0' + (v / p) % 10) << 24, 1);
}

// "<64 hex>" of a digest: 16 SWAR hex words between the quotes.
template <class Sink>
AHV_HD void emit_hex_digest_quoted(Sink& s, const uint32_t d[8]) {
  if (!s.seg(66)) return;
  s.put(0x22u << 24, 1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t hi, lo;
    word_to_hex_words(d[i], hi, lo);
    s.put4(hi);
    s.put4(lo);
  }
  s.put(0x22u << 24, 1);
}

// "session:xxxxxxxx-xxxx-xxxx-xxxx-xxxxxxxxxxxx" from 4 big-endian uuid words.
template <class Sink>
AHV_HD void emit_session_uuid_quoted(Sink& s, const uint32_t u[4]) {
  if (!s.seg(46)) return;
  s.put4(0x22736573u);  // "ses
  s.put4(0x73696f6eu);  // sion
  s.put(0x3a000000u, 1);  // :
  uint32_t hi, lo;
  word_to_hex_words(u[0], hi, lo);
  s.put4(hi);
  s.put4(lo);
  s.put(0x2d000000u, 1);
  word_to_hex_words(u[1], hi, lo);
  s.put4(hi);
  s.put(0x2d000000u, 1);
  s.put4(lo);
  s.put(0x2d000000u, 1);
  word_to_hex_words(u[2], hi, lo);
  s.put4(hi);
  s.put(0x2d000000u, 1);
  s.put4(lo);
  word_to_hex_words(u[3], hi, lo);
  s.put4(hi);
  s.put4(lo);
  s.put(0x22000000u, 1);
}

// Two decimal digits of v < 100 as the top half of a word.
AHV_HD uint32_t dig2(uint32_t v) { return (('0' + v / 10) << 24) | (('0' + v % 10) << 16); }

// datetime.isoformat() text, quoted, straight into the sink.
template <class Sink>
AHV_HD void emit_iso_quoted(Sink& s, int64_t us) {
  const UtcParts t = utc_parts(us);
  if (!s.seg(t.micro ? 34u : 27u)) return;
  // "YYYY-MM-DDTHH:MM:SS
  s.put(0x22000000u | (dig2((t.year / 100) % 100) >> 8), 3);
  s.put(dig2(t.year % 100) | 0x2d00u | ((t.month / 10) + '0'), 4);
  s.put((('0' + t.month % 10) << 24) | 0x2d0000u | (dig2(t.day) >> 16), 4);
  s.put(0x54000000u | (dig2(t.secs / 3600) >> 8) | 0x3au, 4);
  s.put(dig2((t.secs / 60) % 60) | 0x3a00u | ('0' + (t.secs % 60) / 10), 4);
  s.put(static_cast<uint32_t>('0' + t.secs % 10) << 24, 1);
  if (t.micro) {
    s.put(0x2e000000u | (dig2(t.micro / 10000) >> 8) | ('0' + (t.micro / 1000) % 10), 4);
    s.put((('0' + (t.micro / 100) % 10) << 24) | (dig2(t.micro % 100) >> 8), 3);
  }
  s.put4(0x2b30303au);  // +00:
  s.put(0x30302200u, 3);  // 00"
}

// One change object {"content_hash", "operation", "path", "previous_hash"}.
struct ChangeIds {
  int32_t path, op, content_hash, previous_hash;  // pool ids, -1 = null
};

// Session identity: either a pool string (API-created sessions) or a device
// uuid4 (engine-minted sessions).
struct SessionIdent {
  int32_t str_id;    // >= 0: pool string id of the full session id
  uint32_t uuid[4];  // else: 4 uuid words, rendered as "session:<uuid>"
};

// A digest passed by value (no pointers to register arrays: those would force
// the array into scratch memory on the device).
struct Digest {
  uint32_t v[8];
};

// The full canonical payload of one delta.
// The part of a delta record between the agent DID value and the parent digest:
// `, "changes": [...], "delta_id": "…", "parent_hash": ` — plus `null` for a
// record without parent.  It does not depend on the session: a template batch
// renders it once per delta on the host (render_fragment) and the device copies
// it (emit_frag) instead of assembling the change objects per session and pass.
template <class Sink>
AHV_HD void emit_changes_fragment(Sink& s, const StrPool& pool, const ChangeIds* ch, uint32_t nch,
                                  int32_t delta_id_str, uint32_t turn, bool has_parent) {
  emit_lit(s, canon::K_CHANGES);
  for (uint32_t c = 0; c < nch; ++c) {
    if (c) emit_lit(s, canon::K_CH_SEP);
    emit_lit(s, canon::K_CH_OPEN);
    emit_pool_str(s, pool, ch[c].content_hash);
    emit_lit(s, canon::K_CH_OP);
    emit_pool_str(s, pool, ch[c].op);
    emit_lit(s, canon::K_CH_PATH);
    emit_pool_str(s, pool, ch[c].path);
    emit_lit(s, canon::K_CH_PREV);
    emit_pool_str(s, pool, ch[c].previous_hash);
    emit_lit(s, canon::K_CH_CLOSE);
  }
  emit_lit(s, canon::K_DELTA_ID);
  if (delta_id_str >= 0) {
    emit_pool_str(s, pool, delta_id_str);
  } else {
    emit_lit(s, canon::K_DELTA_PFX);
    emit_uint(s, turn);
    emit_char(s, 0x22u);
  }
  emit_lit(s, canon::K_PARENT);
  if (!has_parent) emit_lit(s, canon::K_NULL);
}

// A pre-rendered fragment: `n` bytes as big-endian words (first byte in the top
// byte).  Its address and length are the same for every lane of the batch, so on
// the device the words come through the scalar cache (constant address space:
// s_load, no per-lane vector load and no dependent string-pool lookups).
AHV_HD uint32_t frag_word(const uint32_t* w, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) uint32_t* cword;  // NOLINT: address-space cast
  return ((cword)w)[k];
#else
  return w[k];
#endif
}

template <class Sink>
AHV_HD void emit_frag(Sink& s, const uint32_t* w, uint32_t n) {
  if (!s.seg(n)) return;
  const uint32_t full = n >> 2;
  for (uint32_t k = 0; k < full; ++k) s.put4(frag_word(w, k));
  if (n & 3u) s.put(frag_word(w, full), n & 3u);
}

// Canonical JSON payload of one delta (reference audit/delta.py:41-64).  With
// `frag` (n `frag_n` bytes) the changes fragment is copied instead of rendered.
template <class Sink>
AHV_HD void emit_delta_payload(Sink& s, const StrPool& pool, StrRef agent, const ChangeIds* ch,
                               uint32_t nch, int32_t delta_id_str, uint32_t turn, bool has_parent,
                               Digest parent, SessionIdent sid, int64_t ts_us, const uint32_t* frag = nullptr,
                               uint32_t frag_n = 0) {
  // The device sink calls this once per window pass; laundering the per-lane
  // inputs stops the compiler from hoisting every derived hex word (parent
  // digest, uuid) out of the pass loop and keeping them all live in VGPRs.
  // (turn and the timestamp are wave-uniform: their digits live in SGPRs.)
  s.launder(agent.n);
#pragma unroll
  for (int k = 0; k < 8; ++k) s.launder(parent.v[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) s.launder(sid.uuid[k]);
  emit_lit(s, canon::K_OPEN_AGENT);
  emit_str_ref(s, agent);
  if (frag) emit_frag(s, frag, frag_n);
  else emit_changes_fragment(s, pool, ch, nch, delta_id_str, turn, has_parent);
  if (has_parent) emit_hex_digest_quoted(s, parent.v);
  emit_lit(s, canon::K_SESSION);
  if (sid.str_id >= 0) emit_pool_str(s, pool, sid.str_id);
  else emit_session_uuid_quoted(s, sid.uuid);
  emit_lit(s, canon::K_TS);
  emit_iso_quoted(s, ts_us);
  emit_lit(s, canon::K_TURN);
  emit_uint(s, turn);
  emit_lit(s, canon::K_CLOSE);
}

// Byte collector (host): what an emitter produces, as bytes.
struct ByteSink {
  std::vector<uint8_t>* out;
  bool seg(uint32_t) { return true; }
  void put4(uint32_t v) {
    for (int j = 0; j < 4; ++j) out->push_back(static_cast<uint8_t>(v >> (24 - 8 * j)));
  }
  void put(uint32_t v, uint32_t n) {
    for (uint32_t j = 0; j < n; ++j) out->push_back(static_cast<uint8_t>(v >> (24 - 8 * j)));
  }
  bool any(bool b) const { return b; }
  template <class T>
  void launder(T&) const {}
};

// Midstate reuse across the deltas of one session.  The payload's first 64 bytes
// are `{"agent_did": "<did>", "changes": [{"content_hash": ` (47 + |did| bytes) or,
// with no changes, `{"agent_did": "<did>", "changes": [], "delta_id": "delta:`
// (52 + |did|) cut at 64 — fixed text plus the agent DID — whenever the escaped
// DID is ≥ kMidstateMinDid bytes, so every delta of the session shares its first
// SHA-256 block.  (At 16 bytes, byte 63 would be the first byte of the first
// content hash value, '"' or 'n', which may differ between deltas.)  Mode 1 hashes
// normally and captures the state after block 0 in `mid`; mode 2 resumes from
// `mid` at byte 64 (one compression and part of the emission saved per delta).
constexpr int32_t kMidstateMinDid = 17;
enum MidMode : int { MID_OFF = 0, MID_CAPTURE = 1, MID_RESUME = 2 };

template <class Sink>
AHV_HD void emit_delta_and_hash(Sink& s, const StrPool& pool, StrRef agent, const ChangeIds* ch,
                                uint32_t nch, int32_t delta_id_str, uint32_t turn,
                                bool has_parent, const Digest parent, const SessionIdent sid, int64_t ts_us,
                                uint32_t out[8], Digest& mid, int mid_mode) {
  s.hash_mid([=](Sink& k) {
    emit_delta_payload(k, pool, agent, ch, nch, delta_id_str, turn, has_parent, parent, sid, ts_us);
  }, out, mid, mid_mode);
}

}  // namespace ahv
