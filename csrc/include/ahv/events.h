// Device event ring buffer: kernels append compact event records
// with one atomic per wave; the host drains them into HypervisorEventBus
// objects (agent_hypervisor_amd/runtime/events.py).  Codes are the positions of
// hypervisor.observability.event_bus.EventType (EVENT_CODE), checked by a test.
#pragma once

#include "ahv/hd.h"

namespace ahv {

enum EventCode : uint8_t {
  EV_SESSION_CREATED = 0,
  EV_SESSION_JOINED = 1,
  EV_SESSION_ACTIVATED = 2,
  EV_SESSION_TERMINATED = 3,
  EV_SESSION_ARCHIVED = 4,
  EV_RING_ASSIGNED = 5,
  EV_SAGA_CREATED = 16,
  EV_SAGA_STEP_COMMITTED = 18,
  EV_AUDIT_DELTA_CAPTURED = 35,
  EV_AUDIT_COMMITTED = 36,
  EV_AUDIT_GC_COLLECTED = 37,
};

// Structure-of-arrays records split into kStatSpread segments of
// `capacity / kStatSpread` records; workgroup b appends to segment
// b % kStatSpread through cursor[segment] (one hot address per segment instead
// of one for the whole grid).  A cursor counts every append ever reserved in its
// segment; records past the segment's end are dropped (cursor > segment size).
struct EventRing {
  uint8_t* type;
  int32_t* slot;    // session table row
  int32_t* agent;   // agent id (-1 = none); DIDs resolve through the agent table
  int64_t* ts_us;
  int32_t* aux;     // e.g. ring for RING_ASSIGNED, delta index for DELTA_CAPTURED
  unsigned long long* cursor;  // [kStatSpread]
  int64_t capacity;            // total records (multiple of kStatSpread)
};

AHV_HD int64_t event_segment_size(const EventRing& r) { return r.capacity / kStatSpread; }

struct EventRec {
  uint8_t type;
  int32_t agent;
  int64_t ts;
  int32_t aux;
};

// `at` is the position within segment `seg`.
AHV_HD void event_store(const EventRing& r, int seg, unsigned long long pos, int32_t slot, const EventRec& e) {
  const int64_t segsz = event_segment_size(r);
  if (pos >= static_cast<unsigned long long>(segsz)) return;
  const int64_t at = seg * segsz + static_cast<int64_t>(pos);
  r.type[at] = e.type;
  r.slot[at] = slot;
  r.agent[at] = e.agent;
  r.ts_us[at] = e.ts;
  r.aux[at] = e.aux;
}

}  // namespace ahv
