"""CMVK adapter: behavioural drift checks that can trigger slashing.

Parity target: reference ``integrations/cmvk_adapter.py:26-250``.

* no verifier → drift 0, NONE, passed;
* otherwise ``verify_embeddings(claimed, observed, metric, threshold_profile,
  explain=True)`` → ``.drift_score`` (default 0) and ``.explanation``;
* severity (≥): critical 0.75, high 0.50, medium 0.30, low 0.15;
  ``passed`` ⇔ NONE/LOW; ``should_slash`` ⇔ HIGH/CRITICAL; ``should_demote`` ⇔
  MEDIUM; ``on_drift_detected`` fires for every failed check.

The severity bucketing is the device predicate ``drift_classify`` (K22) for
batched verification; :func:`classify_drift` is its scalar twin.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Any, Callable, Optional, Protocol

from hypervisor._clock import now as _now


class CMVKVerifier(Protocol):
    def verify_embeddings(
        self,
        embedding_a: Any,
        embedding_b: Any,
        metric: str = "cosine",
        weights: Any = None,
        threshold_profile: Optional[str] = None,
        explain: bool = False,
    ) -> Any: ...


class DriftSeverity(str, Enum):
    NONE = "none"
    LOW = "low"
    MEDIUM = "medium"
    HIGH = "high"
    CRITICAL = "critical"


@dataclass
class DriftCheckResult:
    agent_did: str
    session_id: str
    drift_score: float
    severity: DriftSeverity
    passed: bool
    explanation: Optional[str] = None
    action_id: Optional[str] = None
    checked_at: datetime = field(default_factory=_now)

    @property
    def should_slash(self) -> bool:
        return self.severity in (DriftSeverity.HIGH, DriftSeverity.CRITICAL)

    @property
    def should_demote(self) -> bool:
        return self.severity == DriftSeverity.MEDIUM


@dataclass
class DriftThresholds:
    low: float = 0.15
    medium: float = 0.30
    high: float = 0.50
    critical: float = 0.75


def classify_drift(score: float, th: DriftThresholds) -> DriftSeverity:
    if score >= th.critical:
        return DriftSeverity.CRITICAL
    if score >= th.high:
        return DriftSeverity.HIGH
    if score >= th.medium:
        return DriftSeverity.MEDIUM
    if score >= th.low:
        return DriftSeverity.LOW
    return DriftSeverity.NONE


class CMVKAdapter:
    def __init__(
        self,
        verifier: Optional[CMVKVerifier] = None,
        thresholds: Optional[DriftThresholds] = None,
        on_drift_detected: Optional[Callable[[DriftCheckResult], None]] = None,
    ) -> None:
        self._verifier = verifier
        self.thresholds = thresholds or DriftThresholds()
        self._on_drift_detected = on_drift_detected
        self._check_history: list[DriftCheckResult] = []

    def check_behavioral_drift(
        self,
        agent_did: str,
        session_id: str,
        claimed_embedding: Any,
        observed_embedding: Any,
        action_id: Optional[str] = None,
        metric: str = "cosine",
        threshold_profile: Optional[str] = None,
    ) -> DriftCheckResult:
        if self._verifier is None:
            res = DriftCheckResult(agent_did, session_id, 0.0, DriftSeverity.NONE, True, action_id=action_id)
            self._check_history.append(res)
            return res
        out = self._verifier.verify_embeddings(
            embedding_a=claimed_embedding,
            embedding_b=observed_embedding,
            metric=metric,
            threshold_profile=threshold_profile,
            explain=True,
        )
        drift = getattr(out, "drift_score", 0.0)
        expl = getattr(out, "explanation", None)
        sev = self._classify_severity(drift)
        res = DriftCheckResult(
            agent_did=agent_did,
            session_id=session_id,
            drift_score=drift,
            severity=sev,
            passed=sev in (DriftSeverity.NONE, DriftSeverity.LOW),
            explanation=str(expl) if expl else None,
            action_id=action_id,
        )
        self._check_history.append(res)
        if not res.passed and self._on_drift_detected:
            self._on_drift_detected(res)
        return res

    def record_drift_batch(
        self,
        agent_dids,
        session_ids,
        drift_scores,
        action_ids=None,
        device="cpu",
    ) -> list[DriftCheckResult]:
        """Classify many already-computed drift scores (e.g. a bulk verifier's
        output tensor) with one K22-drift launch on ``device`` and record them
        like :meth:`check_behavioral_drift` (history, drift callback)."""
        import torch

        from agent_hypervisor_amd.ops import ledger as LG

        th = self.thresholds
        d = drift_scores if isinstance(drift_scores, torch.Tensor) else torch.tensor(
            [float(x) for x in drift_scores], dtype=torch.float64)
        d = d.to(device=device, dtype=torch.float64).contiguous()
        sev = LG.drift_severity(d, th.low, th.medium, th.high, th.critical)
        host = torch.stack([d, sev.to(torch.float64)]).cpu().tolist()
        out = []
        for i, (agent, session) in enumerate(zip(agent_dids, session_ids)):
            s = DriftSeverity(LG.SEVERITY[int(host[1][i])])
            res = DriftCheckResult(agent_did=agent, session_id=session, drift_score=host[0][i], severity=s,
                                   passed=s in (DriftSeverity.NONE, DriftSeverity.LOW),
                                   action_id=action_ids[i] if action_ids else None)
            self._check_history.append(res)
            if not res.passed and self._on_drift_detected:
                self._on_drift_detected(res)
            out.append(res)
        return out

    def get_agent_drift_history(self, agent_did: str, session_id: Optional[str] = None) -> list[DriftCheckResult]:
        return [
            r
            for r in self._check_history
            if r.agent_did == agent_did and (session_id is None or r.session_id == session_id)
        ]

    def get_drift_rate(self, agent_did: str, session_id: Optional[str] = None) -> float:
        h = self.get_agent_drift_history(agent_did, session_id)
        return sum(1 for r in h if not r.passed) / len(h) if h else 0.0

    def get_mean_drift_score(self, agent_did: str, session_id: Optional[str] = None) -> float:
        h = self.get_agent_drift_history(agent_did, session_id)
        return sum(r.drift_score for r in h) / len(h) if h else 0.0

    @property
    def total_checks(self) -> int:
        return len(self._check_history)

    @property
    def total_violations(self) -> int:
        return sum(1 for r in self._check_history if not r.passed)

    def _classify_severity(self, drift_score: float) -> DriftSeverity:
        return classify_drift(drift_score, self.thresholds)
