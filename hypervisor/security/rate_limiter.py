"""Per-agent, per-ring token-bucket rate limiting.

Parity target: reference ``security/rate_limiter.py:17-176``.

* Ring defaults (rate rps, burst): R0 (100, 200), R1 (50, 100), R2 (20, 40),
  R3 (5, 10); unknown rings (20, 40).
* One bucket per ``agent:session``; the ring is read only when the bucket is
  created, and only :meth:`AgentRateLimiter.update_ring` recreates it full (Q20).
* Refill is lazy on consume/available: ``tokens = min(cap, tokens + dt·rate)``.

Batched twin: kernel K17 (``token_bucket``) refills and consumes thousands of
buckets against one injected ``now_us``.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from typing import Optional

from hypervisor._clock import now as _now
from hypervisor._devsel import device_variant
from hypervisor.models import ExecutionRing


class RateLimitExceeded(Exception):
    """The agent's bucket did not hold enough tokens."""


@dataclass
class TokenBucket:
    capacity: float
    tokens: float
    refill_rate: float
    last_refill: datetime = field(default_factory=_now)

    def _refill(self) -> None:
        t = _now()
        dt = (t - self.last_refill).total_seconds()
        self.tokens = min(self.capacity, self.tokens + dt * self.refill_rate)
        self.last_refill = t

    def consume(self, tokens: float = 1.0) -> bool:
        self._refill()
        if self.tokens >= tokens:
            self.tokens -= tokens
            return True
        return False

    @property
    def available(self) -> float:
        self._refill()
        return self.tokens


DEFAULT_RING_LIMITS: dict[ExecutionRing, tuple[float, float]] = {
    ExecutionRing.RING_0_ROOT: (100.0, 200.0),
    ExecutionRing.RING_1_PRIVILEGED: (50.0, 100.0),
    ExecutionRing.RING_2_STANDARD: (20.0, 40.0),
    ExecutionRing.RING_3_SANDBOX: (5.0, 10.0),
}
FALLBACK_LIMIT = (20.0, 40.0)


@dataclass
class RateLimitStats:
    agent_did: str
    ring: ExecutionRing
    total_requests: int = 0
    rejected_requests: int = 0
    tokens_available: float = 0.0
    capacity: float = 0.0


class AgentRateLimiter:
    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceAgentRateLimiter (batched kernel path)."""
        return device_variant(cls, AgentRateLimiter, "DeviceAgentRateLimiter", device)

    def __init__(self, ring_limits: Optional[dict[ExecutionRing, tuple[float, float]]] = None, device=None) -> None:
        self._limits = ring_limits or dict(DEFAULT_RING_LIMITS)
        self._buckets: dict[str, TokenBucket] = {}
        self._stats: dict[str, RateLimitStats] = {}

    def _new_bucket(self, ring: ExecutionRing) -> TokenBucket:
        rate, cap = self._limits.get(ring, FALLBACK_LIMIT)
        return TokenBucket(capacity=cap, tokens=cap, refill_rate=rate)

    def _get_or_create_bucket(self, key: str, ring: ExecutionRing) -> TokenBucket:
        b = self._buckets.get(key)
        if b is None:
            b = self._buckets[key] = self._new_bucket(ring)
        return b

    def check(self, agent_did: str, session_id: str, ring: ExecutionRing, cost: float = 1.0) -> bool:
        key = f"{agent_did}:{session_id}"
        bucket = self._get_or_create_bucket(key, ring)
        st = self._stats.get(key)
        if st is None:
            st = self._stats[key] = RateLimitStats(agent_did=agent_did, ring=ring)
        st.total_requests += 1
        if bucket.consume(cost):
            return True
        st.rejected_requests += 1
        raise RateLimitExceeded(
            f"Agent {agent_did} exceeded rate limit for ring {ring.value} ({st.rejected_requests} rejections)"
        )

    def try_check(self, agent_did: str, session_id: str, ring: ExecutionRing, cost: float = 1.0) -> bool:
        try:
            return self.check(agent_did, session_id, ring, cost)
        except RateLimitExceeded:
            return False

    def check_batch(self, requests, now=None) -> list[bool]:
        """``try_check`` over ``(agent_did, session_id, ring[, cost])`` tuples in
        order (the device variant serves them with one K17 launch)."""
        return [self.try_check(*q) for q in requests]

    def update_ring(self, agent_did: str, session_id: str, new_ring: ExecutionRing) -> None:
        key = f"{agent_did}:{session_id}"
        self._buckets[key] = self._new_bucket(new_ring)
        st = self._stats.get(key)
        if st is not None:
            st.ring = new_ring

    def get_stats(self, agent_did: str, session_id: str) -> Optional[RateLimitStats]:
        key = f"{agent_did}:{session_id}"
        st = self._stats.get(key)
        if st is not None:
            b = self._buckets.get(key)
            if b is not None:
                st.tokens_available = b.available
                st.capacity = b.capacity
        return st

    @property
    def tracked_agents(self) -> int:
        return len(self._buckets)
