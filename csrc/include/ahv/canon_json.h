// Canonical JSON rendering of the SemanticDelta hash payload.
//
// The reference hashes `json.dumps(payload, sort_keys=True)` (audit/delta.py:43-63):
// ", " / ": " separators, ensure_ascii escaping, `null` for None.  The key order
// after sorting is fixed:
//   {"agent_did", "changes":[{"content_hash","operation","path","previous_hash"}],
//    "delta_id", "parent_hash", "session_id", "timestamp", "turn_id"}
// This header holds the byte-exact template pieces shared by the host renderer
// (csrc/host/py_audit.cpp) and the device renderer (csrc/hip/audit_kernels.hip).
#pragma once

#include "ahv/hd.h"

namespace ahv {
namespace canon {

// Template literals, in emission order.  `K_*` pieces are emitted verbatim.
constexpr char K_OPEN_AGENT[] = "{\"agent_did\": ";            // then <json str>
constexpr char K_CHANGES[] = ", \"changes\": [";                 // then change objects
constexpr char K_CH_OPEN[] = "{\"content_hash\": ";              // then <json str|null>
constexpr char K_CH_OP[] = ", \"operation\": ";                  // then <json str>
constexpr char K_CH_PATH[] = ", \"path\": ";                     // then <json str>
constexpr char K_CH_PREV[] = ", \"previous_hash\": ";            // then <json str|null>
constexpr char K_CH_CLOSE[] = "}";
constexpr char K_CH_SEP[] = ", ";
constexpr char K_DELTA_ID[] = "], \"delta_id\": ";               // then <json str>
constexpr char K_DELTA_PFX[] = "\"delta:";                        // then <int> "
constexpr char K_PARENT[] = ", \"parent_hash\": ";               // then null | "<64 hex>"
constexpr char K_SESSION[] = ", \"session_id\": ";               // then <json str>
constexpr char K_TS[] = ", \"timestamp\": ";                     // then <json str>
constexpr char K_TURN[] = ", \"turn_id\": ";                     // then <int>
constexpr char K_CLOSE[] = "}";
constexpr char K_NULL[] = "null";

template <size_t N>
constexpr uint32_t lit_len(const char (&)[N]) { return static_cast<uint32_t>(N - 1); }

// Is `c` emitted unescaped by json.dumps(ensure_ascii=True)?  The encoder's
// ESCAPE_ASCII class is ([\\"]|[^\ -~]), so printable ASCII except '"' and '\\'.
AHV_HD bool json_plain(uint32_t c) { return c >= 0x20u && c <= 0x7eu && c != 0x22u && c != 0x5cu; }

// Number of decimal digits of a non-negative value.
AHV_HD uint32_t dec_digits(uint64_t v) {
  uint32_t n = 1;
  while (v >= 10u) { v /= 10u; ++n; }
  return n;
}

}  // namespace canon
}  // namespace ahv
