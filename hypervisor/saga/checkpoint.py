"""Semantic checkpoints: record *which goal* a step achieved so replay can skip it.

Parity target: reference ``saga/checkpoint.py:18-163``.
``goal_hash = sha256(f"{goal}:{step_id}").hexdigest()[:16]`` (native SHA-256;
batched form: kernel K12).  The replay plan is the steps without a valid
checkpoint, in order.

Fix: the reference indexed checkpoints by goal hash
*globally*, so the same goal/step saved in a second saga silently hid the first
saga's checkpoint from ``is_achieved``.  The index here is keyed by
(saga, goal hash); parity mode restores the global index.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from typing import Any, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor import config as _cfg
from hypervisor._clock import now as _now


@dataclass
class SemanticCheckpoint:
    checkpoint_id: str = field(default_factory=lambda: _C.hex_id("ckpt:", 8))
    saga_id: str = ""
    step_id: str = ""
    goal_description: str = ""
    goal_hash: str = ""
    achieved_at: datetime = field(default_factory=_now)
    state_snapshot: dict[str, Any] = field(default_factory=dict)
    is_valid: bool = True
    invalidated_reason: Optional[str] = None

    @staticmethod
    def compute_goal_hash(goal: str, step_id: str) -> str:
        return _C.sha256_hex(f"{goal}:{step_id}")[:16]


class CheckpointManager:
    def __init__(self) -> None:
        self._checkpoints: dict[str, list[SemanticCheckpoint]] = {}
        self._by_goal_hash: dict[Any, SemanticCheckpoint] = {}

    @staticmethod
    def _key(saga_id: str, goal_hash: str):
        return goal_hash if _cfg.parity_mode() else (saga_id, goal_hash)

    def save(
        self,
        saga_id: str,
        step_id: str,
        goal_description: str,
        state_snapshot: Optional[dict] = None,
    ) -> SemanticCheckpoint:
        gh = SemanticCheckpoint.compute_goal_hash(goal_description, step_id)
        c = SemanticCheckpoint(
            saga_id=saga_id,
            step_id=step_id,
            goal_description=goal_description,
            goal_hash=gh,
            state_snapshot=state_snapshot or {},
        )
        self._checkpoints.setdefault(saga_id, []).append(c)
        self._by_goal_hash[self._key(saga_id, gh)] = c
        return c

    def _lookup(self, saga_id: str, goal_description: str, step_id: str) -> Optional[SemanticCheckpoint]:
        gh = SemanticCheckpoint.compute_goal_hash(goal_description, step_id)
        c = self._by_goal_hash.get(self._key(saga_id, gh))
        if c is not None and c.saga_id == saga_id and c.is_valid:
            return c
        return None

    def is_achieved(self, saga_id: str, goal_description: str, step_id: str) -> bool:
        return self._lookup(saga_id, goal_description, step_id) is not None

    def get_checkpoint(self, saga_id: str, goal_description: str, step_id: str) -> Optional[SemanticCheckpoint]:
        return self._lookup(saga_id, goal_description, step_id)

    def invalidate(self, saga_id: str, step_id: str, reason: str = "") -> int:
        n = 0
        for c in self._checkpoints.get(saga_id, ()):
            if c.step_id == step_id and c.is_valid:
                c.is_valid = False
                c.invalidated_reason = reason
                n += 1
        return n

    def get_saga_checkpoints(self, saga_id: str) -> list[SemanticCheckpoint]:
        return [c for c in self._checkpoints.get(saga_id, ()) if c.is_valid]

    def get_replay_plan(self, saga_id: str, steps: list[str]) -> list[str]:
        done = {c.step_id for c in self.get_saga_checkpoints(saga_id)}
        return [s for s in steps if s not in done]

    # -- persistence / audit (K12) ----------------------------------------------
    def verify(self, device: Optional[str] = None) -> list[str]:
        """Ids of checkpoints whose goal hash does not match sha256(goal:step)[:16],
        every checkpoint re-hashed in one batched K12 launch."""
        from hypervisor.audit.batch_verify import verify_audit

        return verify_audit((), device=device, checkpoints=[self]).bad_checkpoints

    def export_records(self) -> list[dict]:
        return [
            {"checkpoint_id": c.checkpoint_id, "saga_id": c.saga_id, "step_id": c.step_id,
             "goal_description": c.goal_description, "goal_hash": c.goal_hash,
             "achieved_at": c.achieved_at.isoformat(), "state_snapshot": c.state_snapshot,
             "is_valid": c.is_valid, "invalidated_reason": c.invalidated_reason}
            for cps in self._checkpoints.values() for c in cps
        ]

    @classmethod
    def from_records(cls, records: list[dict], verify: bool = True,
                     device: Optional[str] = None) -> "CheckpointManager":
        """Rebuild a manager from :meth:`export_records`; with ``verify`` every goal
        hash is re-derived (K12) and a mismatch raises ``ValueError``."""
        mgr = cls()
        for r in records:
            c = SemanticCheckpoint(
                checkpoint_id=r["checkpoint_id"], saga_id=r["saga_id"], step_id=r["step_id"],
                goal_description=r["goal_description"], goal_hash=r["goal_hash"],
                achieved_at=datetime.fromisoformat(r["achieved_at"]), state_snapshot=dict(r["state_snapshot"]),
                is_valid=r["is_valid"], invalidated_reason=r["invalidated_reason"])
            mgr._checkpoints.setdefault(c.saga_id, []).append(c)
            mgr._by_goal_hash[cls._key(c.saga_id, c.goal_hash)] = c
        if verify:
            bad = mgr.verify(device)
            if bad:
                raise ValueError(f"checkpoint {bad[0]}: goal hash does not match its goal ({len(bad)} bad)")
        return mgr

    @property
    def total_checkpoints(self) -> int:
        return sum(len(v) for v in self._checkpoints.values())

    @property
    def valid_checkpoints(self) -> int:
        return sum(1 for v in self._checkpoints.values() for c in v if c.is_valid)
