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

// Structure-of-arrays ring of `capacity` records; `cursor` counts every append
// ever reserved (records past capacity are dropped and show up as cursor > cap).
struct EventRing {
  uint8_t* type;
  int32_t* slot;    // session table row
  int32_t* agent;   // agent id (-1 = none); DIDs resolve through the agent table
  int64_t* ts_us;
  int32_t* aux;     // e.g. ring for RING_ASSIGNED, delta index for DELTA_CAPTURED
  unsigned long long* cursor;
  int64_t capacity;
};

struct EventRec {
  uint8_t type;
  int32_t agent;
  int64_t ts;
  int32_t aux;
};

AHV_HD inline void event_store(const EventRing& r, unsigned long long at, int32_t slot, const EventRec& e) {
  if (at >= static_cast<unsigned long long>(r.capacity)) return;
  r.type[at] = e.type;
  r.slot[at] = slot;
  r.agent[at] = e.agent;
  r.ts_us[at] = e.ts;
  r.aux[at] = e.aux;
}

}  // namespace ahv
