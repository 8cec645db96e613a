"""Structured, append-only hypervisor event bus with pub/sub.

Parity target: reference ``observability/event_bus.py:18-219``: 40 dotted event
types in 8 categories, frozen :class:`HypervisorEvent` records (16-hex ids),
indexes by type / session / agent, type-specific subscribers notified before
wildcard (``None``) subscribers, ``query(..., limit)`` keeping the *last*
``limit`` matches.

Difference: the reference never emitted anything (Q03).  Here
:class:`hypervisor.core.Hypervisor` emits session, ring, audit, liability and
saga events when constructed with an ``event_bus`` (the REST server passes its
bus), so ``GET /api/v1/events`` reflects real activity.  The device engine has a
ring-buffer twin (``agent_hypervisor_amd.runtime.event_ring``) that
kernels append to and the host drains into this bus.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Any, Callable, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now


class EventType(str, Enum):
    # session lifecycle
    SESSION_CREATED = "session.created"
    SESSION_JOINED = "session.joined"
    SESSION_ACTIVATED = "session.activated"
    SESSION_TERMINATED = "session.terminated"
    SESSION_ARCHIVED = "session.archived"
    # rings
    RING_ASSIGNED = "ring.assigned"
    RING_ELEVATED = "ring.elevated"
    RING_DEMOTED = "ring.demoted"
    RING_ELEVATION_EXPIRED = "ring.elevation_expired"
    RING_BREACH_DETECTED = "ring.breach_detected"
    # liability
    VOUCH_CREATED = "liability.vouch_created"
    VOUCH_RELEASED = "liability.vouch_released"
    SLASH_EXECUTED = "liability.slash_executed"
    FAULT_ATTRIBUTED = "liability.fault_attributed"
    QUARANTINE_ENTERED = "liability.quarantine_entered"
    QUARANTINE_RELEASED = "liability.quarantine_released"
    # saga
    SAGA_CREATED = "saga.created"
    SAGA_STEP_STARTED = "saga.step_started"
    SAGA_STEP_COMMITTED = "saga.step_committed"
    SAGA_STEP_FAILED = "saga.step_failed"
    SAGA_COMPENSATING = "saga.compensating"
    SAGA_COMPLETED = "saga.completed"
    SAGA_ESCALATED = "saga.escalated"
    SAGA_FANOUT_STARTED = "saga.fanout_started"
    SAGA_FANOUT_RESOLVED = "saga.fanout_resolved"
    SAGA_CHECKPOINT_SAVED = "saga.checkpoint_saved"
    # vfs
    VFS_WRITE = "vfs.write"
    VFS_DELETE = "vfs.delete"
    VFS_SNAPSHOT = "vfs.snapshot"
    VFS_RESTORE = "vfs.restore"
    VFS_CONFLICT = "vfs.conflict"
    # security
    RATE_LIMITED = "security.rate_limited"
    AGENT_KILLED = "security.agent_killed"
    SAGA_HANDOFF = "security.saga_handoff"
    IDENTITY_VERIFIED = "security.identity_verified"
    # audit
    AUDIT_DELTA_CAPTURED = "audit.delta_captured"
    AUDIT_COMMITTED = "audit.committed"
    AUDIT_GC_COLLECTED = "audit.gc_collected"
    # verification
    BEHAVIOR_DRIFT = "verification.behavior_drift"
    HISTORY_VERIFIED = "verification.history_verified"


EVENT_CODE = {t: i for i, t in enumerate(EventType)}
EVENT_FROM_CODE = {i: t for t, i in EVENT_CODE.items()}


@dataclass(frozen=True)
class HypervisorEvent:
    event_id: str = field(default_factory=lambda: _C.hex_id("", 16))
    event_type: EventType = EventType.SESSION_CREATED
    timestamp: datetime = field(default_factory=_now)
    session_id: Optional[str] = None
    agent_did: Optional[str] = None
    causal_trace_id: Optional[str] = None
    parent_event_id: Optional[str] = None
    payload: dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict[str, Any]:
        return {
            "event_id": self.event_id,
            "event_type": self.event_type.value,
            "timestamp": self.timestamp.isoformat(),
            "session_id": self.session_id,
            "agent_did": self.agent_did,
            "causal_trace_id": self.causal_trace_id,
            "parent_event_id": self.parent_event_id,
            "payload": self.payload,
        }


EventHandler = Callable[[HypervisorEvent], None]


class HypervisorEventBus:
    def __init__(self) -> None:
        self._events: list[HypervisorEvent] = []
        self._subscribers: dict[Optional[EventType], list[EventHandler]] = {}
        self._by_type: dict[EventType, list[HypervisorEvent]] = {}
        self._by_session: dict[str, list[HypervisorEvent]] = {}
        self._by_agent: dict[str, list[HypervisorEvent]] = {}

    def emit(self, event: HypervisorEvent) -> None:
        self._events.append(event)
        self._by_type.setdefault(event.event_type, []).append(event)
        if event.session_id:
            self._by_session.setdefault(event.session_id, []).append(event)
        if event.agent_did:
            self._by_agent.setdefault(event.agent_did, []).append(event)
        for h in self._subscribers.get(event.event_type, ()):
            h(event)
        for h in self._subscribers.get(None, ()):
            h(event)

    def publish(
        self,
        event_type: EventType,
        session_id: Optional[str] = None,
        agent_did: Optional[str] = None,
        **payload: Any,
    ) -> HypervisorEvent:
        """Convenience: build and emit an event."""
        ev = HypervisorEvent(event_type=event_type, session_id=session_id, agent_did=agent_did, payload=payload)
        self.emit(ev)
        return ev

    def subscribe(self, event_type: Optional[EventType] = None, handler: Optional[EventHandler] = None) -> None:
        if handler:
            self._subscribers.setdefault(event_type, []).append(handler)

    def query_by_type(self, event_type: EventType) -> list[HypervisorEvent]:
        return list(self._by_type.get(event_type, ()))

    def query_by_session(self, session_id: str) -> list[HypervisorEvent]:
        return list(self._by_session.get(session_id, ()))

    def query_by_agent(self, agent_did: str) -> list[HypervisorEvent]:
        return list(self._by_agent.get(agent_did, ()))

    def query_by_time_range(self, start: datetime, end: Optional[datetime] = None) -> list[HypervisorEvent]:
        end = end if end is not None else _now()
        return [e for e in self._events if start <= e.timestamp <= end]

    def query(
        self,
        event_type: Optional[EventType] = None,
        session_id: Optional[str] = None,
        agent_did: Optional[str] = None,
        limit: Optional[int] = None,
    ) -> list[HypervisorEvent]:
        out = self._events
        if event_type is not None:
            out = [e for e in out if e.event_type == event_type]
        if session_id is not None:
            out = [e for e in out if e.session_id == session_id]
        if agent_did is not None:
            out = [e for e in out if e.agent_did == agent_did]
        if limit is not None:
            out = out[-limit:]
        return list(out) if out is self._events else out

    @property
    def event_count(self) -> int:
        return len(self._events)

    @property
    def all_events(self) -> list[HypervisorEvent]:
        return list(self._events)

    def type_counts(self) -> dict[str, int]:
        return {t.value: len(v) for t, v in self._by_type.items()}

    def clear(self) -> None:
        self._events.clear()
        self._by_type.clear()
        self._by_session.clear()
        self._by_agent.clear()
