"""Saga state machines for steps and sagas.

Parity target: reference ``saga/state_machine.py:17-156``.

Step FSM::

    PENDING → EXECUTING → COMMITTED → COMPENSATING → COMPENSATED
                        ↘ FAILED                   ↘ COMPENSATION_FAILED

Saga FSM::

    RUNNING → COMPENSATING | COMPLETED | FAILED
    COMPENSATING → COMPLETED | FAILED | ESCALATED

An invalid edge raises :class:`SagaStateError` ("Invalid step transition: a → b.
Allowed: [...]").  ``started_at`` is stamped on EXECUTING; ``completed_at`` on
COMMITTED / COMPENSATED / COMPENSATION_FAILED / FAILED and on terminal saga
states.  ``Saga.to_dict`` is the persistence format (kept key-for-key).

The same two tables are encoded as 7×7 / 5×5 bit masks in
``csrc/include/ahv/semantics.h`` for the batched saga kernels (K13/K14); the
integer codes are the ``CODE`` attribute of each enum member.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Any, Optional

from hypervisor._clock import now as _now


class StepState(str, Enum):
    PENDING = "pending"
    EXECUTING = "executing"
    COMMITTED = "committed"
    COMPENSATING = "compensating"
    COMPENSATED = "compensated"
    COMPENSATION_FAILED = "compensation_failed"
    FAILED = "failed"


class SagaState(str, Enum):
    RUNNING = "running"
    COMPENSATING = "compensating"
    COMPLETED = "completed"
    FAILED = "failed"
    ESCALATED = "escalated"


# integer codes shared with the device FSM tables (declaration order)
STEP_CODE = {s: i for i, s in enumerate(StepState)}
SAGA_CODE = {s: i for i, s in enumerate(SagaState)}

STEP_TRANSITIONS: dict[StepState, set[StepState]] = {
    StepState.PENDING: {StepState.EXECUTING},
    StepState.EXECUTING: {StepState.COMMITTED, StepState.FAILED},
    StepState.COMMITTED: {StepState.COMPENSATING},
    StepState.COMPENSATING: {StepState.COMPENSATED, StepState.COMPENSATION_FAILED},
    StepState.COMPENSATED: set(),
    StepState.COMPENSATION_FAILED: set(),
    StepState.FAILED: set(),
}

SAGA_TRANSITIONS: dict[SagaState, set[SagaState]] = {
    SagaState.RUNNING: {SagaState.COMPENSATING, SagaState.COMPLETED, SagaState.FAILED},
    SagaState.COMPENSATING: {SagaState.COMPLETED, SagaState.FAILED, SagaState.ESCALATED},
    SagaState.COMPLETED: set(),
    SagaState.FAILED: set(),
    SagaState.ESCALATED: set(),
}

_STEP_STAMPS_COMPLETED = frozenset(
    {StepState.COMMITTED, StepState.COMPENSATED, StepState.COMPENSATION_FAILED, StepState.FAILED}
)
_SAGA_TERMINAL = frozenset({SagaState.COMPLETED, SagaState.FAILED, SagaState.ESCALATED})


def step_transition_mask() -> list[int]:
    """Row bit masks of STEP_TRANSITIONS (row = from-code, bit = to-code)."""
    return [sum(1 << STEP_CODE[t] for t in STEP_TRANSITIONS[s]) for s in StepState]


def saga_transition_mask() -> list[int]:
    return [sum(1 << SAGA_CODE[t] for t in SAGA_TRANSITIONS[s]) for s in SagaState]


class SagaStateError(Exception):
    """Invalid saga/step transition or unknown saga/step id."""


@dataclass
class SagaStep:
    step_id: str
    action_id: str
    agent_did: str
    execute_api: str
    undo_api: Optional[str] = None
    state: StepState = StepState.PENDING
    execute_result: Optional[Any] = None
    compensation_result: Optional[Any] = None
    error: Optional[str] = None
    started_at: Optional[datetime] = None
    completed_at: Optional[datetime] = None
    timeout_seconds: int = 300
    max_retries: int = 0
    retry_count: int = 0

    def transition(self, new_state: StepState) -> None:
        allowed = STEP_TRANSITIONS.get(self.state, ())
        if new_state not in allowed:
            raise SagaStateError(
                f"Invalid step transition: {self.state.value} → {new_state.value}. "
                f"Allowed: {[s.value for s in allowed]}"
            )
        self.state = new_state
        if new_state is StepState.EXECUTING:
            self.started_at = _now()
        elif new_state in _STEP_STAMPS_COMPLETED:
            self.completed_at = _now()


@dataclass
class Saga:
    saga_id: str
    session_id: str
    steps: list[SagaStep] = field(default_factory=list)
    state: SagaState = SagaState.RUNNING
    created_at: datetime = field(default_factory=_now)
    completed_at: Optional[datetime] = None
    error: Optional[str] = None

    def transition(self, new_state: SagaState) -> None:
        allowed = SAGA_TRANSITIONS.get(self.state, ())
        if new_state not in allowed:
            raise SagaStateError(
                f"Invalid saga transition: {self.state.value} → {new_state.value}. "
                f"Allowed: {[s.value for s in allowed]}"
            )
        self.state = new_state
        if new_state in _SAGA_TERMINAL:
            self.completed_at = _now()

    @property
    def committed_steps(self) -> list[SagaStep]:
        return [s for s in self.steps if s.state == StepState.COMMITTED]

    @property
    def committed_steps_reversed(self) -> list[SagaStep]:
        return self.committed_steps[::-1]

    def to_dict(self) -> dict:
        return {
            "saga_id": self.saga_id,
            "session_id": self.session_id,
            "state": self.state.value,
            "created_at": self.created_at.isoformat(),
            "completed_at": self.completed_at.isoformat() if self.completed_at else None,
            "error": self.error,
            "steps": [
                {
                    "step_id": s.step_id,
                    "action_id": s.action_id,
                    "agent_did": s.agent_did,
                    "state": s.state.value,
                    "error": s.error,
                }
                for s in self.steps
            ],
        }

    @classmethod
    def from_dict(cls, d: dict) -> "Saga":
        """Inverse of :meth:`to_dict` (resume from the persisted format)."""
        saga = cls(
            saga_id=d["saga_id"],
            session_id=d["session_id"],
            state=SagaState(d["state"]),
            created_at=datetime.fromisoformat(d["created_at"]),
            completed_at=datetime.fromisoformat(d["completed_at"]) if d.get("completed_at") else None,
            error=d.get("error"),
        )
        for s in d.get("steps", []):
            saga.steps.append(
                SagaStep(
                    step_id=s["step_id"],
                    action_id=s["action_id"],
                    agent_did=s["agent_did"],
                    execute_api="",
                    state=StepState(s["state"]),
                    error=s.get("error"),
                )
            )
        return saga
