"""Action classifier: manifest action → (ring, ω, reversibility).

Parity target: reference ``rings/classifier.py:16-77``.  Lookup order is
override, then cache, then derivation from the descriptor; cached results are
returned by identity.  Overrides carry confidence 0.9 and fall back to the cached
classification or (Ring 3, ω 0.5, NONE).

Fix: overrides test ``is not None``, so an explicit
``RING_0_ROOT`` or ``risk_weight=0.0`` override is honoured (the reference's
``ring or …`` silently dropped both).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from hypervisor.models import ActionDescriptor, ExecutionRing, ReversibilityLevel


@dataclass
class ClassificationResult:
    action_id: str
    ring: ExecutionRing
    risk_weight: float
    reversibility: ReversibilityLevel
    confidence: float = 1.0


class ActionClassifier:
    def __init__(self) -> None:
        self._cache: dict[str, ClassificationResult] = {}
        self._overrides: dict[str, ClassificationResult] = {}

    def classify(self, action: ActionDescriptor) -> ClassificationResult:
        aid = action.action_id
        hit = self._overrides.get(aid) or self._cache.get(aid)
        if hit is not None:
            return hit
        res = ClassificationResult(aid, action.required_ring, action.risk_weight, action.reversibility)
        self._cache[aid] = res
        return res

    def set_override(
        self,
        action_id: str,
        ring: Optional[ExecutionRing] = None,
        risk_weight: Optional[float] = None,
    ) -> None:
        base = self._cache.get(action_id)
        if ring is None:
            ring = base.ring if base else ExecutionRing.RING_3_SANDBOX
        if risk_weight is None:
            risk_weight = base.risk_weight if base else 0.5
        self._overrides[action_id] = ClassificationResult(
            action_id=action_id,
            ring=ring,
            risk_weight=risk_weight,
            reversibility=base.reversibility if base else ReversibilityLevel.NONE,
            confidence=0.9,
        )

    def clear_cache(self) -> None:
        self._cache.clear()
