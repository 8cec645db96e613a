// Shared definitions of the batched governance pipeline — the device form of the
// reference benchmark's `full_governance_pipeline` (benchmarks/bench_hypervisor.py:
// 217-239) — whose per-session body is `template_session` in ahv/store_template.h
// (it writes the device store's rows; there is no separate pipeline table).
#pragma once

#include "ahv/delta_emit.h"
#include "ahv/events.h"
#include "ahv/semantics.h"

namespace ahv {

constexpr int kMaxParticipants = 16;   // participant rows a pipeline session writes at most
constexpr int kMaxDeltasPipeline = 8;  // ⌈8/2⌉ Merkle scratch slots fit the LDS window
constexpr int kMaxChanges = 4;

// Per-session counters reduced into the batch statistics (collective X04):
// sessions, ok, participants, deltas, commitments, archived.
constexpr int kPipeStats = 6;
struct PipeCounters {
  uint32_t v[kPipeStats];
};

}  // namespace ahv
