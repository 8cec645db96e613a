"""IATP adapter: capability manifests → actions, σ hint and ring hint.

Parity target: reference ``integrations/iatp_adapter.py:30-253``.

* trust level string → :class:`IATPTrustLevel` (unknown strings → UNKNOWN);
  ring hint: verified_partner → 1, trusted/standard → 2, unknown/untrusted → 3;
* ``sigma_hint = clamp(trust_score / 10, 0, 1)`` (dict path default score 5);
* dict actions → :class:`ActionDescriptor` with reversibility mapped (unknown →
  NONE); the protocol path synthesises one ``"{agent}:default"`` action;
* both paths cache the analysis per agent.

Fix: ``undo_window`` strings like ``"5m"`` / ``"2h"`` are
converted to seconds (the reference stripped the unit and kept the number);
parity mode keeps the reference's stripping.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Any, Optional, Protocol

from hypervisor import config as _cfg
from hypervisor._clock import now as _now
from hypervisor.models import ActionDescriptor, ExecutionRing, ReversibilityLevel


class IATPManifest(Protocol):
    agent_id: str
    trust_level: Any
    capabilities: Any
    scopes: list[str]

    def calculate_trust_score(self) -> int: ...


class IATPTrustLevel(str, Enum):
    VERIFIED_PARTNER = "verified_partner"
    TRUSTED = "trusted"
    STANDARD = "standard"
    UNKNOWN = "unknown"
    UNTRUSTED = "untrusted"


TRUST_LEVEL_RING_HINTS = {
    IATPTrustLevel.VERIFIED_PARTNER: ExecutionRing.RING_1_PRIVILEGED,
    IATPTrustLevel.TRUSTED: ExecutionRing.RING_2_STANDARD,
    IATPTrustLevel.STANDARD: ExecutionRing.RING_2_STANDARD,
    IATPTrustLevel.UNKNOWN: ExecutionRing.RING_3_SANDBOX,
    IATPTrustLevel.UNTRUSTED: ExecutionRing.RING_3_SANDBOX,
}

REVERSIBILITY_MAP = {
    "full": ReversibilityLevel.FULL,
    "partial": ReversibilityLevel.PARTIAL,
    "none": ReversibilityLevel.NONE,
}

_UNIT_SECONDS = {"s": 1, "m": 60, "h": 3600}


@dataclass
class ManifestAnalysis:
    agent_did: str
    trust_level: IATPTrustLevel
    ring_hint: ExecutionRing
    iatp_trust_score: int
    sigma_hint: float
    actions: list[ActionDescriptor]
    scopes: list[str]
    has_reversible_actions: bool
    has_non_reversible_actions: bool
    analyzed_at: datetime = field(default_factory=_now)


def _trust_level(raw: Any) -> IATPTrustLevel:
    try:
        return IATPTrustLevel(raw)
    except ValueError:
        return IATPTrustLevel.UNKNOWN


def parse_undo_window(text: Any) -> int:
    """Seconds in an IATP undo window such as ``"30s"``, ``"5m"``, ``"2h"``."""
    if not text:
        return 0
    try:
        s = str(text).strip()
        if _cfg.parity_mode():
            return int(s.rstrip("s").rstrip("m").rstrip("h"))
        if s and s[-1] in _UNIT_SECONDS:
            return int(float(s[:-1]) * _UNIT_SECONDS[s[-1]])
        return int(s)
    except (ValueError, AttributeError):
        return 0


class IATPAdapter:
    def __init__(self) -> None:
        self._manifest_cache: dict[str, ManifestAnalysis] = {}

    def _finish(self, agent: str, level: IATPTrustLevel, score: Any, actions, scopes) -> ManifestAnalysis:
        a = ManifestAnalysis(
            agent_did=agent,
            trust_level=level,
            ring_hint=TRUST_LEVEL_RING_HINTS.get(level, ExecutionRing.RING_3_SANDBOX),
            iatp_trust_score=score,
            sigma_hint=min(max(score / 10.0, 0.0), 1.0),
            actions=actions,
            scopes=scopes,
            has_reversible_actions=any(x.reversibility != ReversibilityLevel.NONE for x in actions),
            has_non_reversible_actions=any(
                x.reversibility == ReversibilityLevel.NONE and not x.is_read_only for x in actions
            ),
        )
        self._manifest_cache[agent] = a
        return a

    def analyze_manifest(self, manifest: IATPManifest) -> ManifestAnalysis:
        tl = manifest.trust_level
        level = _trust_level(str(getattr(tl, "value", tl)))
        score = manifest.calculate_trust_score()
        actions = self._extract_actions(manifest)
        scopes = list(manifest.scopes) if manifest.scopes else []
        return self._finish(manifest.agent_id, level, score, actions, scopes)

    def analyze_manifest_dict(self, manifest_dict: dict) -> ManifestAnalysis:
        actions = [
            ActionDescriptor(
                action_id=c.get("action_id", "unknown"),
                name=c.get("name", ""),
                execute_api=c.get("execute_api", ""),
                undo_api=c.get("undo_api"),
                reversibility=REVERSIBILITY_MAP.get(c.get("reversibility", "none"), ReversibilityLevel.NONE),
                is_read_only=c.get("is_read_only", False),
                is_admin=c.get("is_admin", False),
            )
            for c in manifest_dict.get("actions", [])
        ]
        return self._finish(
            manifest_dict.get("agent_id", "unknown"),
            _trust_level(manifest_dict.get("trust_level", "unknown")),
            manifest_dict.get("trust_score", 5),
            actions,
            manifest_dict.get("scopes", []),
        )

    def get_cached_analysis(self, agent_did: str) -> Optional[ManifestAnalysis]:
        return self._manifest_cache.get(agent_did)

    def _extract_actions(self, manifest: IATPManifest) -> list[ActionDescriptor]:
        caps = manifest.capabilities
        if caps is None:
            return []
        rev_raw = getattr(caps, "reversibility", "none")
        rev = REVERSIBILITY_MAP.get(str(getattr(rev_raw, "value", rev_raw)), ReversibilityLevel.NONE)
        aid = manifest.agent_id
        return [
            ActionDescriptor(
                action_id=f"{aid}:default",
                name=f"Default action for {aid}",
                execute_api=f"/api/{aid}/execute",
                undo_api=f"/api/{aid}/undo" if rev != ReversibilityLevel.NONE else None,
                reversibility=rev,
                undo_window_seconds=parse_undo_window(getattr(caps, "undo_window", None)),
            )
        ]
