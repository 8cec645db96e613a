"""Quarantine: read-only isolation of a liable agent before termination.

Parity target: reference ``liability/quarantine.py:18-177``.

* A second quarantine of the same (agent, session) escalates the live record:
  ``details += "; escalated: …"`` and forensic data is merged.
* Duration is ``duration_seconds or 300`` — ``None`` does **not** mean
  indefinite (preserved).
* Expiry is wall-clock; :meth:`QuarantineManager.tick` auto-releases (device twin:
  expiry kernel K18).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime, timedelta
from enum import Enum
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now
from hypervisor._devsel import device_variant


class QuarantineReason(str, Enum):
    BEHAVIORAL_DRIFT = "behavioral_drift"
    LIABILITY_VIOLATION = "liability_violation"
    RING_BREACH = "ring_breach"
    RATE_LIMIT_EXCEEDED = "rate_limit_exceeded"
    MANUAL = "manual"
    CASCADE_SLASH = "cascade_slash"


@dataclass
class QuarantineRecord:
    quarantine_id: str = field(default_factory=lambda: _C.hex_id("quar:", 8))
    agent_did: str = ""
    session_id: str = ""
    reason: QuarantineReason = QuarantineReason.MANUAL
    details: str = ""
    entered_at: datetime = field(default_factory=_now)
    expires_at: Optional[datetime] = None
    released_at: Optional[datetime] = None
    is_active: bool = True
    forensic_data: dict = field(default_factory=dict)

    @property
    def is_expired(self) -> bool:
        return self.expires_at is not None and _now() > self.expires_at

    @property
    def duration_seconds(self) -> float:
        return ((self.released_at or _now()) - self.entered_at).total_seconds()


class QuarantineManager:
    DEFAULT_QUARANTINE_SECONDS = 300

    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceQuarantineManager (batched kernel path)."""
        return device_variant(cls, QuarantineManager, "DeviceQuarantineManager", device)

    def __init__(self, device=None) -> None:
        self._quarantines: dict[str, QuarantineRecord] = {}

    def quarantine(
        self,
        agent_did: str,
        session_id: str,
        reason: QuarantineReason,
        details: str = "",
        duration_seconds: Optional[int] = None,
        forensic_data: Optional[dict] = None,
    ) -> QuarantineRecord:
        live = self.get_active_quarantine(agent_did, session_id)
        if live is not None:
            live.details += f"; escalated: {details}"
            if forensic_data:
                live.forensic_data.update(forensic_data)
            return live
        secs = duration_seconds or self.DEFAULT_QUARANTINE_SECONDS
        t = _now()
        rec = QuarantineRecord(
            agent_did=agent_did,
            session_id=session_id,
            reason=reason,
            details=details,
            entered_at=t,
            expires_at=t + timedelta(seconds=secs) if secs else None,
            forensic_data=forensic_data or {},
        )
        self._quarantines[rec.quarantine_id] = rec
        return rec

    def quarantine_batch(self, requests) -> list[QuarantineRecord]:
        """``quarantine`` over ``(agent_did, session_id, reason[, details,
        duration_seconds, forensic_data])`` tuples in order."""
        return [self.quarantine(*q) for q in requests]

    def release(self, agent_did: str, session_id: str) -> Optional[QuarantineRecord]:
        rec = self.get_active_quarantine(agent_did, session_id)
        if rec is not None:
            rec.is_active = False
            rec.released_at = _now()
        return rec

    def is_quarantined(self, agent_did: str, session_id: str) -> bool:
        return self.get_active_quarantine(agent_did, session_id) is not None

    def get_active_quarantine(self, agent_did: str, session_id: str) -> Optional[QuarantineRecord]:
        for r in self._quarantines.values():
            if r.agent_did == agent_did and r.session_id == session_id and r.is_active and not r.is_expired:
                return r
        return None

    def tick(self) -> list[QuarantineRecord]:
        out = []
        for r in self._quarantines.values():
            if r.is_active and r.is_expired:
                r.is_active = False
                r.released_at = _now()
                out.append(r)
        return out

    def get_history(
        self, agent_did: Optional[str] = None, session_id: Optional[str] = None
    ) -> list[QuarantineRecord]:
        return [
            r
            for r in self._quarantines.values()
            if (not agent_did or r.agent_did == agent_did) and (not session_id or r.session_id == session_id)
        ]

    @property
    def active_quarantines(self) -> list[QuarantineRecord]:
        return [r for r in self._quarantines.values() if r.is_active and not r.is_expired]

    @property
    def quarantine_count(self) -> int:
        return len(self.active_quarantines)
