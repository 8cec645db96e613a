"""Reversibility registry: every declared action → Execute_API / Undo_API.

Parity target: reference ``reversibility/registry.py:16-106``.  Session-scoped,
populated from the IATP manifest at join; a duplicate ``action_id`` overwrites.
An unknown action has ω = 0.95 (the NONE midpoint).
``has_non_reversible_actions()`` is what makes ``join_session`` force STRONG
consistency.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from hypervisor.models import ActionDescriptor, ReversibilityLevel


@dataclass
class ReversibilityEntry:
    action_id: str
    execute_api: str
    undo_api: Optional[str]
    reversibility: ReversibilityLevel
    undo_window_seconds: int
    compensation_method: Optional[str]
    risk_weight: float
    undo_api_healthy: bool = True
    last_health_check: Optional[str] = None


class ReversibilityRegistry:
    def __init__(self, session_id: str) -> None:
        self.session_id = session_id
        self._entries: dict[str, ReversibilityEntry] = {}
        self._irreversible = 0  # count of NONE entries (O(1) mode negotiation)

    def register(self, action: ActionDescriptor) -> ReversibilityEntry:
        old = self._entries.get(action.action_id)
        if old is not None and old.reversibility == ReversibilityLevel.NONE:
            self._irreversible -= 1
        e = ReversibilityEntry(
            action_id=action.action_id,
            execute_api=action.execute_api,
            undo_api=action.undo_api,
            reversibility=action.reversibility,
            undo_window_seconds=action.undo_window_seconds,
            compensation_method=action.compensation_method,
            risk_weight=action.risk_weight,
        )
        self._entries[action.action_id] = e
        if e.reversibility == ReversibilityLevel.NONE:
            self._irreversible += 1
        return e

    def register_from_manifest(self, actions: list[ActionDescriptor]) -> int:
        for a in actions:
            self.register(a)
        return len(actions)

    def get(self, action_id: str) -> Optional[ReversibilityEntry]:
        return self._entries.get(action_id)

    def get_undo_api(self, action_id: str) -> Optional[str]:
        e = self._entries.get(action_id)
        return e.undo_api if e is not None else None

    def is_reversible(self, action_id: str) -> bool:
        e = self._entries.get(action_id)
        return e is not None and e.reversibility != ReversibilityLevel.NONE

    def get_risk_weight(self, action_id: str) -> float:
        e = self._entries.get(action_id)
        return e.risk_weight if e is not None else ReversibilityLevel.NONE.default_risk_weight

    def has_non_reversible_actions(self) -> bool:
        if not self._entries:
            return False
        # entries are mutable dataclasses: trust the counter only when it is positive
        if self._irreversible > 0:
            return True
        return any(e.reversibility == ReversibilityLevel.NONE for e in self._entries.values())

    def mark_undo_unhealthy(self, action_id: str) -> None:
        e = self._entries.get(action_id)
        if e is not None:
            e.undo_api_healthy = False

    @property
    def entries(self) -> list[ReversibilityEntry]:
        return list(self._entries.values())

    @property
    def non_reversible_actions(self) -> list[str]:
        return [e.action_id for e in self._entries.values() if e.reversibility == ReversibilityLevel.NONE]
