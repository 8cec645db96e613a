"""Device event ring buffer.

The batched pipeline kernel (``store_template_kernel``) appends compact lifecycle records — one 64-bit
atomic per wave reserves the wave's slots — into SoA tensors owned here.  The
host drains them on its own cadence into :class:`HypervisorEventBus` events
(the same event types the scalar facade publishes), so kernels can emit events
without a host round trip per session.

The ring is split into 64 segments (one per workgroup residue, so appends
contend on 64 cursors instead of one); records past a segment's end are
dropped (counted by :attr:`DeviceEventRing.dropped`).  Size the ring for one
drain interval (≈8 records per session, plus slack for segment imbalance).
"""

from __future__ import annotations

from typing import Optional

import torch

from agent_hypervisor_amd.utils.stats import SPREAD
from hypervisor import _clock
from hypervisor.observability.event_bus import EVENT_FROM_CODE, HypervisorEvent

u8, i32, i64 = torch.uint8, torch.int32, torch.int64


class DeviceEventRing:
    def __init__(self, capacity: int, device) -> None:
        dev = torch.device(device)
        capacity = -(-int(capacity) // SPREAD) * SPREAD  # whole segments
        self.capacity = capacity
        self.segment = capacity // SPREAD
        self.device = dev
        self.type = torch.zeros(capacity, dtype=u8, device=dev)
        self.slot = torch.zeros(capacity, dtype=i32, device=dev)
        self.agent = torch.zeros(capacity, dtype=i32, device=dev)
        self.ts_us = torch.zeros(capacity, dtype=i64, device=dev)
        self.aux = torch.zeros(capacity, dtype=i32, device=dev)
        self.cursor = torch.zeros(SPREAD, dtype=i64, device=dev)  # read as unsigned 64-bit by kernels
        self.total_dropped = 0

    def kernel_args(self) -> tuple[dict, dict]:
        """(scalars, tensors) entries for a pipeline launch."""
        return ({"ev_capacity": self.capacity},
                {"ev_type": self.type, "ev_slot": self.slot, "ev_agent": self.agent, "ev_ts_us": self.ts_us,
                 "ev_aux": self.aux, "ev_cursor": self.cursor})

    def _counts(self) -> list[int]:
        return [int(c) for c in self.cursor.cpu().tolist()]

    @property
    def pending(self) -> int:
        return sum(min(c, self.segment) for c in self._counts())

    @property
    def dropped(self) -> int:
        return sum(max(0, c - self.segment) for c in self._counts())

    def snapshot(self) -> dict[str, torch.Tensor]:
        """Host copies of the pending records, segment by segment (does not reset)."""
        counts = self._counts()
        idx = torch.cat([torch.arange(min(c, self.segment)) + g * self.segment for g, c in enumerate(counts)])
        idx = idx.to(self.type.device)
        return {k: getattr(self, k).index_select(0, idx).cpu() for k in ("type", "slot", "agent", "ts_us", "aux")}

    def reset(self) -> None:
        self.total_dropped += self.dropped
        self.cursor.zero_()

    def drain(self, engine, bus=None, limit: Optional[int] = None) -> list[HypervisorEvent]:
        """Convert pending records to events (published on ``bus`` if given) and
        reset the ring.  Events are ordered by (timestamp, slot, emission order)."""
        snap = self.snapshot()
        self.reset()
        n = snap["type"].numel()
        if n == 0:
            return []
        order = sorted(range(n), key=lambda j: (int(snap["ts_us"][j]), int(snap["slot"][j]), j))
        if limit is not None:
            order = order[:limit]
        t = engine.sessions
        sid_cache: dict[int, str] = {}
        out = []
        for j in order:
            slot = int(snap["slot"][j])
            sid = sid_cache.get(slot)
            if sid is None:
                w = t.sess_uuid[slot].cpu().tolist()
                h = "".join(f"{x & 0xFFFFFFFF:08x}" for x in w)
                sid = sid_cache[slot] = f"session:{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"
            a = int(snap["agent"][j])  # store agent id (participant rows)
            did = engine.store.did(a) if a >= 0 else None
            et = EVENT_FROM_CODE[int(snap["type"][j])]
            payload = {"ring": int(snap["aux"][j])} if et.value == "ring.assigned" else {}
            ev = HypervisorEvent(event_type=et, timestamp=_clock.from_us(int(snap["ts_us"][j])), session_id=sid,
                                 agent_did=did, payload=payload)
            out.append(ev)
            if bus is not None:
                bus.emit(ev)
        return out
