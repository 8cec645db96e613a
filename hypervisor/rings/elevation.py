"""Time-bounded ring elevation ("sudo with a TTL") and spawn inheritance.

Parity target: reference ``rings/elevation.py:19-211``.

* Elevation must target a strictly more privileged ring; Ring 0 is never granted
  here (it needs the SRE-witness protocol).
* One active elevation per (agent, session).
* TTL 0 → ``DEFAULT_TTL`` (300 s); clamped to ``MAX_ELEVATION_TTL`` (3600 s).
* Expiry is wall-clock; :meth:`RingElevationManager.tick` deactivates and returns
  the expired grants (device twin: expiry kernel K18).
* Spawned children get at most ``min(parent + 1, 3)``.

Active grants are indexed by (agent, session) so lookups are O(1) rather than a
scan over every grant ever made.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime, timedelta
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now
from hypervisor._devsel import device_variant
from hypervisor.models import ExecutionRing


def _elev_id() -> str:
    return _C.hex_id("elev:", 8)


@dataclass
class RingElevation:
    elevation_id: str = field(default_factory=_elev_id)
    agent_did: str = ""
    session_id: str = ""
    original_ring: ExecutionRing = ExecutionRing.RING_3_SANDBOX
    elevated_ring: ExecutionRing = ExecutionRing.RING_2_STANDARD
    granted_at: datetime = field(default_factory=_now)
    expires_at: datetime = field(default_factory=_now)
    attestation: Optional[str] = None
    reason: str = ""
    is_active: bool = True

    @property
    def is_expired(self) -> bool:
        return _now() > self.expires_at

    @property
    def remaining_seconds(self) -> float:
        return max(0.0, (self.expires_at - _now()).total_seconds())


class RingElevationError(Exception):
    """Invalid elevation request or unknown elevation id."""


def _child_ring(parent: ExecutionRing) -> ExecutionRing:
    return ExecutionRing(min(parent.value + 1, ExecutionRing.RING_3_SANDBOX.value))


class RingElevationManager:
    MAX_ELEVATION_TTL = 3600
    DEFAULT_TTL = 300

    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceRingElevationManager (batched kernel path)."""
        return device_variant(cls, RingElevationManager, "DeviceRingElevationManager", device)

    def __init__(self, device=None) -> None:
        self._elevations: dict[str, RingElevation] = {}
        self._by_key: dict[tuple[str, str], list[str]] = {}
        self._parent_map: dict[str, str] = {}
        self._children: dict[str, list[str]] = {}

    def request_elevation(
        self,
        agent_did: str,
        session_id: str,
        current_ring: ExecutionRing,
        target_ring: ExecutionRing,
        ttl_seconds: int = 0,
        attestation: Optional[str] = None,
        reason: str = "",
    ) -> RingElevation:
        if target_ring.value >= current_ring.value:
            raise RingElevationError(
                f"Target ring {target_ring.value} is not more privileged "
                f"than current ring {current_ring.value}"
            )
        if target_ring == ExecutionRing.RING_0_ROOT:
            raise RingElevationError(
                "Ring 0 elevation not available via elevation manager — requires SRE Witness protocol"
            )
        live = self.get_active_elevation(agent_did, session_id)
        if live is not None:
            raise RingElevationError(
                f"Agent {agent_did} already has active elevation to ring {live.elevated_ring.value}"
            )
        ttl = ttl_seconds if ttl_seconds > 0 else self.DEFAULT_TTL
        ttl = min(ttl, self.MAX_ELEVATION_TTL)
        t = _now()
        e = RingElevation(
            agent_did=agent_did,
            session_id=session_id,
            original_ring=current_ring,
            elevated_ring=target_ring,
            granted_at=t,
            expires_at=t + timedelta(seconds=ttl),
            attestation=attestation,
            reason=reason,
        )
        self._elevations[e.elevation_id] = e
        self._by_key.setdefault((agent_did, session_id), []).append(e.elevation_id)
        return e

    def request_elevation_batch(self, requests) -> list:
        """``request_elevation`` over argument tuples in order → each
        RingElevation, or the RingElevationError it raised."""
        out: list = []
        for q in requests:
            try:
                out.append(self.request_elevation(*q))
            except RingElevationError as e:
                out.append(e)
        return out

    def get_active_elevation(self, agent_did: str, session_id: str) -> Optional[RingElevation]:
        for eid in self._by_key.get((agent_did, session_id), ()):
            e = self._elevations[eid]
            if e.is_active and not e.is_expired:
                return e
        return None

    def get_effective_ring(self, agent_did: str, session_id: str, base_ring: ExecutionRing) -> ExecutionRing:
        e = self.get_active_elevation(agent_did, session_id)
        return e.elevated_ring if e is not None else base_ring

    def revoke_elevation(self, elevation_id: str) -> None:
        e = self._elevations.get(elevation_id)
        if e is None:
            raise RingElevationError(f"Elevation {elevation_id} not found")
        e.is_active = False

    def tick(self) -> list[RingElevation]:
        expired = [e for e in self._elevations.values() if e.is_active and e.is_expired]
        for e in expired:
            e.is_active = False
        return expired

    # -- spawn inheritance ---------------------------------------------------
    def register_child(self, parent_did: str, child_did: str, parent_ring: ExecutionRing) -> ExecutionRing:
        self._parent_map[child_did] = parent_did
        self._children.setdefault(parent_did, []).append(child_did)
        return _child_ring(parent_ring)

    def get_parent(self, child_did: str) -> Optional[str]:
        return self._parent_map.get(child_did)

    def get_children(self, parent_did: str) -> list[str]:
        return list(self._children.get(parent_did, ()))

    def get_max_child_ring(self, parent_ring: ExecutionRing) -> ExecutionRing:
        return _child_ring(parent_ring)

    @property
    def active_elevations(self) -> list[RingElevation]:
        return [e for e in self._elevations.values() if e.is_active and not e.is_expired]

    @property
    def elevation_count(self) -> int:
        return len(self._elevations)
