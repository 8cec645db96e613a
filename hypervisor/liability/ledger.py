"""Persistent per-agent liability ledger and admission decisions.

Parity target: reference ``liability/ledger.py:17-177``.  Risk of an agent::

    +0.15 · max(sev, 0.5)   per SLASH_RECEIVED / SLASH_CASCADED
    +0.10 · max(sev, 0.3)   per QUARANTINE_ENTERED
    +0.05 · sev             per FAULT_ATTRIBUTED
    −0.05                   per CLEAN_SESSION
    clamp to [0, 1];  ≥ 0.6 deny, ≥ 0.3 probation, else admit

(the code's ``max(sev, floor)`` behaviour is preserved over the docstring's,
SURVEY Appendix A Q22).  Cross-rank aggregation of these partials uses
fixed-point int64 (collective X03, ``agent_hypervisor_amd.parallel.collectives``)
so every rank computes the identical rounded risk.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now
from hypervisor._devsel import device_variant


class LedgerEntryType(str, Enum):
    VOUCH_GIVEN = "vouch_given"
    VOUCH_RECEIVED = "vouch_received"
    VOUCH_RELEASED = "vouch_released"
    SLASH_RECEIVED = "slash_received"
    SLASH_CASCADED = "slash_cascaded"
    QUARANTINE_ENTERED = "quarantine_entered"
    QUARANTINE_RELEASED = "quarantine_released"
    FAULT_ATTRIBUTED = "fault_attributed"
    CLEAN_SESSION = "clean_session"


@dataclass
class LedgerEntry:
    entry_id: str = field(default_factory=lambda: _C.hex_id("", 12))
    agent_did: str = ""
    entry_type: LedgerEntryType = LedgerEntryType.CLEAN_SESSION
    session_id: str = ""
    timestamp: datetime = field(default_factory=_now)
    severity: float = 0.0
    details: str = ""
    related_agent: Optional[str] = None


@dataclass
class AgentRiskProfile:
    agent_did: str
    total_entries: int = 0
    slash_count: int = 0
    quarantine_count: int = 0
    clean_session_count: int = 0
    fault_score_avg: float = 0.0
    risk_score: float = 0.0
    recommendation: str = "admit"


_SLASH = (LedgerEntryType.SLASH_RECEIVED, LedgerEntryType.SLASH_CASCADED)


def risk_increment(entry_type: LedgerEntryType, severity: float) -> float:
    """Contribution of one ledger entry to the unclamped risk (kernel K22 twin)."""
    if entry_type in _SLASH:
        return 0.15 * max(severity, 0.5)
    if entry_type == LedgerEntryType.QUARANTINE_ENTERED:
        return 0.10 * max(severity, 0.3)
    if entry_type == LedgerEntryType.FAULT_ATTRIBUTED:
        return 0.05 * severity
    if entry_type == LedgerEntryType.CLEAN_SESSION:
        return -0.05
    return 0.0


class LiabilityLedger:
    PROBATION_THRESHOLD = 0.3
    DENY_THRESHOLD = 0.6

    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceLiabilityLedger (batched kernel path)."""
        return device_variant(cls, LiabilityLedger, "DeviceLiabilityLedger", device)

    def __init__(self, device=None) -> None:
        self._entries: list[LedgerEntry] = []
        self._by_agent: dict[str, list[LedgerEntry]] = {}

    def record(
        self,
        agent_did: str,
        entry_type: LedgerEntryType,
        session_id: str = "",
        severity: float = 0.0,
        details: str = "",
        related_agent: Optional[str] = None,
    ) -> LedgerEntry:
        e = LedgerEntry(
            agent_did=agent_did,
            entry_type=entry_type,
            session_id=session_id,
            severity=severity,
            details=details,
            related_agent=related_agent,
        )
        self._entries.append(e)
        self._by_agent.setdefault(agent_did, []).append(e)
        return e

    def get_agent_history(self, agent_did: str) -> list[LedgerEntry]:
        return list(self._by_agent.get(agent_did, ()))

    def recommendation_for(self, risk: float) -> str:
        if risk >= self.DENY_THRESHOLD:
            return "deny"
        if risk >= self.PROBATION_THRESHOLD:
            return "probation"
        return "admit"

    def compute_risk_profile(self, agent_did: str) -> AgentRiskProfile:
        hist = self._by_agent.get(agent_did)
        if not hist:
            return AgentRiskProfile(agent_did=agent_did, recommendation="admit")
        slashes = quars = cleans = 0
        faults: list[float] = []
        risk = 0.0
        for e in hist:
            t = e.entry_type
            if t in _SLASH:
                slashes += 1
            elif t == LedgerEntryType.QUARANTINE_ENTERED:
                quars += 1
            elif t == LedgerEntryType.FAULT_ATTRIBUTED:
                faults.append(e.severity)
            elif t == LedgerEntryType.CLEAN_SESSION:
                cleans += 1
            risk += risk_increment(t, e.severity)
        risk = min(1.0, max(0.0, risk))
        return AgentRiskProfile(
            agent_did=agent_did,
            total_entries=len(hist),
            slash_count=slashes,
            quarantine_count=quars,
            clean_session_count=cleans,
            fault_score_avg=round(sum(faults) / len(faults), 4) if faults else 0.0,
            risk_score=round(risk, 4),
            recommendation=self.recommendation_for(risk),
        )

    def compute_risk_profiles(self, agent_dids) -> list[AgentRiskProfile]:
        """Profiles of many agents (one K22 launch in the device variant)."""
        return [self.compute_risk_profile(a) for a in agent_dids]

    def should_admit(self, agent_did: str) -> tuple[bool, str]:
        prof = self.compute_risk_profile(agent_did)
        if prof.recommendation == "deny":
            return False, f"Risk score {prof.risk_score:.2f} exceeds threshold"
        return True, prof.recommendation

    @property
    def total_entries(self) -> int:
        return len(self._entries)

    @property
    def tracked_agents(self) -> list[str]:
        return list(self._by_agent)
