"""Ring breach detector: sliding-window anomaly score with a circuit breaker.

Parity target: reference ``rings/breach_detector.py:20-218``.

Per ``agent:session`` profile: a window (deque, maxlen 1000) of
(timestamp, agent ring, called ring).  Each call prunes entries older than
``window_seconds``.  While a tripped breaker is cooling down (30 s) no events are
produced.  With ≥ 5 windowed calls the anomaly rate is the fraction of calls into
rings more privileged than the agent's *current* ring; ≥0.9 CRITICAL, ≥0.7 HIGH,
≥0.5 MEDIUM, ≥0.3 LOW.  HIGH/CRITICAL trip the breaker.

Batched twin: kernel K16 (``breach_window``) keeps the same window as a ring
buffer of (ts_us, called_ring) per profile; see ``ops/security_ops.py``.
"""

from __future__ import annotations

from collections import defaultdict, deque
from dataclasses import dataclass, field
from datetime import datetime, timedelta
from enum import Enum
from typing import Optional

from hypervisor._clock import now as _now
from hypervisor._devsel import device_variant
from hypervisor.models import ExecutionRing


class BreachSeverity(str, Enum):
    NONE = "none"
    LOW = "low"
    MEDIUM = "medium"
    HIGH = "high"
    CRITICAL = "critical"


@dataclass
class BreachEvent:
    agent_did: str
    session_id: str
    severity: BreachSeverity
    anomaly_score: float
    call_count_window: int
    expected_rate: float
    actual_rate: float
    timestamp: datetime = field(default_factory=_now)
    details: str = ""


@dataclass
class AgentCallProfile:
    agent_did: str
    session_id: str
    calls: deque = field(default_factory=lambda: deque(maxlen=1000))
    total_calls: int = 0
    ring_call_counts: dict = field(default_factory=lambda: defaultdict(int))
    breaker_tripped: bool = False
    breaker_tripped_at: Optional[datetime] = None


def classify_rate(rate: float) -> BreachSeverity:
    """Severity band of an anomaly rate (shared with the K16 kernel codes)."""
    d = RingBreachDetector
    if rate >= d.CRITICAL_THRESHOLD:
        return BreachSeverity.CRITICAL
    if rate >= d.HIGH_THRESHOLD:
        return BreachSeverity.HIGH
    if rate >= d.MEDIUM_THRESHOLD:
        return BreachSeverity.MEDIUM
    if rate >= d.LOW_THRESHOLD:
        return BreachSeverity.LOW
    return BreachSeverity.NONE


class RingBreachDetector:
    WINDOW_SECONDS = 60
    LOW_THRESHOLD = 0.3
    MEDIUM_THRESHOLD = 0.5
    HIGH_THRESHOLD = 0.7
    CRITICAL_THRESHOLD = 0.9
    CIRCUIT_BREAKER_COOLDOWN = 30
    MIN_CALLS = 5

    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceRingBreachDetector (batched kernel path)."""
        return device_variant(cls, RingBreachDetector, "DeviceRingBreachDetector", device)

    def __init__(self, window_seconds: int = 0, device=None) -> None:
        self._profiles: dict[str, AgentCallProfile] = {}
        self._breach_history: list[BreachEvent] = []
        self.window_seconds = window_seconds or self.WINDOW_SECONDS

    def _cooling(self, p: AgentCallProfile, t: datetime) -> bool:
        return (
            p.breaker_tripped
            and p.breaker_tripped_at is not None
            and t < p.breaker_tripped_at + timedelta(seconds=self.CIRCUIT_BREAKER_COOLDOWN)
        )

    def record_call(
        self,
        agent_did: str,
        session_id: str,
        agent_ring: ExecutionRing,
        called_ring: ExecutionRing,
    ) -> Optional[BreachEvent]:
        key = f"{agent_did}:{session_id}"
        p = self._profiles.get(key)
        if p is None:
            p = self._profiles[key] = AgentCallProfile(agent_did=agent_did, session_id=session_id)
        t = _now()
        p.calls.append((t, agent_ring, called_ring))
        p.total_calls += 1
        p.ring_call_counts[called_ring.value] += 1
        horizon = t - timedelta(seconds=self.window_seconds)
        calls = p.calls
        while calls and calls[0][0] < horizon:
            calls.popleft()
        if self._cooling(p, t):
            return None
        return self._analyze(p, agent_ring, t)

    def _analyze(self, profile: AgentCallProfile, agent_ring: ExecutionRing, now: datetime) -> Optional[BreachEvent]:
        total = len(profile.calls)
        if total < self.MIN_CALLS:
            return None
        mine = agent_ring.value
        hits = sum(1 for _, _, called in profile.calls if called.value < mine)
        rate = hits / total
        sev = classify_rate(rate)
        if sev is BreachSeverity.NONE:
            return None
        if sev is BreachSeverity.HIGH or sev is BreachSeverity.CRITICAL:
            profile.breaker_tripped = True
            profile.breaker_tripped_at = now
        ev = BreachEvent(
            agent_did=profile.agent_did,
            session_id=profile.session_id,
            severity=sev,
            anomaly_score=rate,
            call_count_window=total,
            expected_rate=0.0,
            actual_rate=rate,
            details=f"{hits}/{total} calls to more-privileged rings in {self.window_seconds}s window",
        )
        self._breach_history.append(ev)
        return ev

    def record_calls_batch(self, calls, now=None) -> list[Optional[BreachEvent]]:
        """``record_call`` over ``(agent_did, session_id, agent_ring, called_ring)``
        tuples in order (the device variant runs them as one K16 launch)."""
        return [self.record_call(*c) for c in calls]

    def is_breaker_tripped(self, agent_did: str, session_id: str) -> bool:
        p = self._profiles.get(f"{agent_did}:{session_id}")
        if p is None or not p.breaker_tripped:
            return False
        if p.breaker_tripped_at is not None and not self._cooling(p, _now()):
            p.breaker_tripped = False
            return False
        return True

    def reset_breaker(self, agent_did: str, session_id: str) -> None:
        p = self._profiles.get(f"{agent_did}:{session_id}")
        if p is not None:
            p.breaker_tripped = False
            p.breaker_tripped_at = None

    def get_agent_stats(self, agent_did: str, session_id: str) -> dict:
        p = self._profiles.get(f"{agent_did}:{session_id}")
        if p is None:
            return {"total_calls": 0, "window_calls": 0, "breaker_tripped": False}
        return {
            "total_calls": p.total_calls,
            "window_calls": len(p.calls),
            "breaker_tripped": p.breaker_tripped,
            "ring_distribution": dict(p.ring_call_counts),
        }

    @property
    def breach_history(self) -> list[BreachEvent]:
        return list(self._breach_history)

    @property
    def breach_count(self) -> int:
        return len(self._breach_history)
