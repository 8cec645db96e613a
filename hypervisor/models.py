"""L0 data model: enums and records shared by every engine.

Behavioural parity with reference ``src/hypervisor/models.py:12-132``:

* ring derivation from σ_eff uses **strict** ``>`` at 0.95 (with consensus) and
  0.60, and never yields Ring 0 (models.py:34-42);
* ω for each reversibility level is the exact fp64 midpoint of its range
  (models.py:52-66), so ``FULL → 0.2``, ``PARTIAL → 0.65``, ``NONE → 0.95``;
* ``ActionDescriptor.required_ring`` precedence: admin → 0, irreversible
  writes → 1, read-only → 3, everything else → 2 (models.py:122-132).

The same thresholds are compiled into the gfx950 ring-gate kernel
(``csrc/include/ahv/semantics.h``); ``tests/test_kernels_host.py`` checks the two
agree element-for-element.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Optional

from hypervisor._clock import now as _now

__all__ = [
    "ConsistencyMode",
    "ExecutionRing",
    "ReversibilityLevel",
    "SessionState",
    "SessionConfig",
    "SessionParticipant",
    "ActionDescriptor",
]

RING1_SIGMA = 0.95
RING2_SIGMA = 0.60


class ConsistencyMode(str, Enum):
    """STRONG: consensus before effects; EVENTUAL: gossip convergence."""

    STRONG = "strong"
    EVENTUAL = "eventual"


class ExecutionRing(int, Enum):
    """Four privilege rings; a lower value is more privileged.

    0 root (SRE witness), 1 privileged (irreversible, consensus),
    2 standard (reversible), 3 sandbox (read-only, default).
    """

    RING_0_ROOT = 0
    RING_1_PRIVILEGED = 1
    RING_2_STANDARD = 2
    RING_3_SANDBOX = 3

    @classmethod
    def from_sigma_eff(cls, sigma_eff: float, has_consensus: bool = False) -> "ExecutionRing":
        if has_consensus and sigma_eff > RING1_SIGMA:
            return _RING1
        if sigma_eff > RING2_SIGMA:
            return _RING2
        return _RING3


_RING1 = ExecutionRing.RING_1_PRIVILEGED
_RING2 = ExecutionRing.RING_2_STANDARD
_RING3 = ExecutionRing.RING_3_SANDBOX

# (lo, hi) risk-weight band per reversibility value
_OMEGA_BANDS = {"full": (0.1, 0.3), "partial": (0.5, 0.8), "none": (0.9, 1.0)}
_OMEGA_MID = {k: (lo + hi) / 2 for k, (lo, hi) in _OMEGA_BANDS.items()}


class ReversibilityLevel(str, Enum):
    """How far an action's effects can be undone."""

    FULL = "full"
    PARTIAL = "partial"
    NONE = "none"

    @property
    def risk_weight_range(self) -> tuple[float, float]:
        return _OMEGA_BANDS[self.value]

    @property
    def default_risk_weight(self) -> float:
        return _OMEGA_MID[self.value]


class SessionState(str, Enum):
    """created → handshaking → active → terminating → archived."""

    CREATED = "created"
    HANDSHAKING = "handshaking"
    ACTIVE = "active"
    TERMINATING = "terminating"
    ARCHIVED = "archived"


@dataclass
class SessionConfig:
    consistency_mode: ConsistencyMode = ConsistencyMode.EVENTUAL
    max_participants: int = 10
    max_duration_seconds: int = 3600
    min_sigma_eff: float = 0.60
    enable_audit: bool = True
    enable_blockchain_commitment: bool = False


@dataclass
class SessionParticipant:
    agent_did: str
    ring: ExecutionRing = ExecutionRing.RING_3_SANDBOX
    sigma_raw: float = 0.0
    sigma_eff: float = 0.0
    joined_at: datetime = field(default_factory=_now)
    is_active: bool = True


@dataclass
class ActionDescriptor:
    """An action declared in an IATP capability manifest."""

    action_id: str
    name: str
    execute_api: str
    undo_api: Optional[str] = None
    reversibility: ReversibilityLevel = ReversibilityLevel.NONE
    undo_window_seconds: int = 0
    compensation_method: Optional[str] = None
    is_read_only: bool = False
    is_admin: bool = False

    @property
    def risk_weight(self) -> float:
        return _OMEGA_MID[self.reversibility.value]

    @property
    def required_ring(self) -> ExecutionRing:
        if self.is_admin:
            return ExecutionRing.RING_0_ROOT
        if self.is_read_only:
            return _RING3
        if self.reversibility is ReversibilityLevel.NONE or self.reversibility == "none":
            return _RING1
        return _RING2
