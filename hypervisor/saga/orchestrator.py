"""Saga orchestrator: forward execution with timeout/retry, reverse-order
compensation with escalation.

Parity target: reference ``saga/orchestrator.py:24-222``.

``execute_step`` runs ``1 + max_retries`` attempts.  Each attempt sets
``retry_count``, moves the step to EXECUTING and awaits ``executor()`` under the
step timeout; success stores the result and commits.  A timeout records
``SagaTimeoutError("Step … timed out after Ns (attempt k/n)")``, any other
exception its ``str``, and the step goes FAILED; between attempts the step is put
back to PENDING directly (outside the FSM, Q15) and the orchestrator sleeps
``1.0 s × (attempt + 1)``.  When attempts run out the last error is re-raised.

``compensate`` walks committed steps in reverse: no Undo_API →
COMPENSATION_FAILED ("No Undo_API available"); otherwise COMPENSATING →
``compensator(step)`` under the timeout → COMPENSATED, or COMPENSATION_FAILED with
"Compensation timed out…" / "Compensation failed: …".  Any failure escalates the
saga ("{n} step(s) failed compensation — Joint Liability slashing triggered"),
otherwise it completes.  The compensator must return an awaitable (Q16).

The await itself uses :func:`hypervisor.saga._timeout.await_with_timeout`
(inline await + loop timer) instead of a Task per step.  The batched form of
this state machine — thousands of sagas per launch, hipGraph-captured step loop —
is ``agent_hypervisor_amd.models.saga_engine``.
"""

from __future__ import annotations

import asyncio
from typing import Any, Callable, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor.saga._timeout import await_with_timeout
from hypervisor.saga.state_machine import Saga, SagaState, SagaStateError, SagaStep, StepState

_uuid4 = _C.uuid4


class SagaTimeoutError(Exception):
    """A saga step (or its compensation) exceeded its timeout."""


class SagaOrchestrator:
    DEFAULT_MAX_RETRIES = 2  # declared by the reference, unused by add_step (Q14)
    DEFAULT_RETRY_DELAY_SECONDS = 1.0

    def __init__(self) -> None:
        self._sagas: dict[str, Saga] = {}

    def create_saga(self, session_id: str, saga_id: Optional[str] = None) -> Saga:
        """``saga_id``: an explicit id (the sharded façade mints ids that route to the owner rank)."""
        saga = Saga(saga_id=saga_id or _uuid4("saga:"), session_id=session_id)
        self._sagas[saga.saga_id] = saga
        return saga

    def add_step(
        self,
        saga_id: str,
        action_id: str,
        agent_did: str,
        execute_api: str,
        undo_api: Optional[str] = None,
        timeout_seconds: int = 300,
        max_retries: int = 0,
    ) -> SagaStep:
        saga = self._get_saga(saga_id)
        step = SagaStep(
            step_id=_uuid4("step:"),
            action_id=action_id,
            agent_did=agent_did,
            execute_api=execute_api,
            undo_api=undo_api,
            timeout_seconds=timeout_seconds,
            max_retries=max_retries,
        )
        saga.steps.append(step)
        return step

    async def execute_step(self, saga_id: str, step_id: str, executor: Callable[..., Any]) -> Any:
        saga = self._get_saga(saga_id)
        step = self._get_step(saga, step_id)
        attempts = 1 + step.max_retries
        last: Optional[Exception] = None
        for attempt in range(attempts):
            step.retry_count = attempt
            step.transition(StepState.EXECUTING)
            try:
                result = await await_with_timeout(executor(), step.timeout_seconds)
            except asyncio.TimeoutError:
                last = SagaTimeoutError(
                    f"Step {step_id} timed out after {step.timeout_seconds}s "
                    f"(attempt {attempt + 1}/{attempts})"
                )
            except Exception as e:  # executor failure
                last = e
            else:
                step.execute_result = result
                step.transition(StepState.COMMITTED)
                return result
            step.error = str(last)
            step.transition(StepState.FAILED)
            if attempt < attempts - 1:
                step.state = StepState.PENDING
                step.error = None
                await asyncio.sleep(self.DEFAULT_RETRY_DELAY_SECONDS * (attempt + 1))
        if last is not None:
            raise last
        raise SagaStateError("Step execution failed with no error captured")

    async def compensate(self, saga_id: str, compensator: Callable[[SagaStep], Any]) -> list[SagaStep]:
        saga = self._get_saga(saga_id)
        saga.transition(SagaState.COMPENSATING)
        failed: list[SagaStep] = []
        for step in saga.committed_steps_reversed:
            if not step.undo_api:
                step.state = StepState.COMPENSATION_FAILED
                step.error = "No Undo_API available"
                failed.append(step)
                continue
            step.transition(StepState.COMPENSATING)
            try:
                res = await await_with_timeout(compensator(step), step.timeout_seconds)
            except asyncio.TimeoutError:
                step.error = f"Compensation timed out after {step.timeout_seconds}s"
            except Exception as e:
                step.error = f"Compensation failed: {e}"
            else:
                step.compensation_result = res
                step.transition(StepState.COMPENSATED)
                continue
            step.transition(StepState.COMPENSATION_FAILED)
            failed.append(step)
        if failed:
            saga.transition(SagaState.ESCALATED)
            saga.error = (
                f"{len(failed)} step(s) failed compensation — Joint Liability slashing triggered"
            )
        else:
            saga.transition(SagaState.COMPLETED)
        return failed

    async def execute_sagas(
        self,
        saga_ids: list[str],
        executors: dict[str, Callable[..., Any]],
        compensator: Optional[Callable[[SagaStep], Any]] = None,
        compensate: bool = True,
        device: Optional[str] = None,
    ) -> list[Saga]:
        """Run many sagas to completion: each saga executes its steps in order
        (``execute_step`` semantics, ``executors[step_id]``); on the first step
        that exhausts its attempts it is compensated (``compensate``) or marked
        FAILED, otherwise COMPLETED.  Sagas run concurrently.

        With ``device`` the coroutines are still awaited here, but the state
        machine runs as one replay of the hipGraph-captured K13/K14 step loop
        (:mod:`agent_hypervisor_amd.models.saga_runner`) and its states are
        written back into these Saga objects."""
        sagas = [self._get_saga(i) for i in saga_ids]
        if device is not None:
            from agent_hypervisor_amd.models.saga_runner import runner_for

            await runner_for(device).run(self, sagas, executors, compensator, compensate)
            return sagas

        async def one(saga: Saga) -> None:
            for step in saga.steps:
                try:
                    await self.execute_step(saga.saga_id, step.step_id, executors[step.step_id])
                except Exception:
                    if compensate:
                        await self.compensate(saga.saga_id, compensator)
                    else:
                        saga.transition(SagaState.FAILED)
                    return
            saga.transition(SagaState.COMPLETED)

        await asyncio.gather(*(one(s) for s in sagas))
        return sagas

    def get_saga(self, saga_id: str) -> Optional[Saga]:
        return self._sagas.get(saga_id)

    @property
    def sagas(self) -> list[Saga]:
        """Every saga of this orchestrator, in creation order."""
        return list(self._sagas.values())

    @property
    def active_sagas(self) -> list[Saga]:
        return [
            s for s in self._sagas.values() if s.state in (SagaState.RUNNING, SagaState.COMPENSATING)
        ]

    def _get_saga(self, saga_id: str) -> Saga:
        saga = self._sagas.get(saga_id)
        if saga is None:
            raise SagaStateError(f"Saga {saga_id} not found")
        return saga

    def _get_step(self, saga: Saga, step_id: str) -> SagaStep:
        for st in saga.steps:
            if st.step_id == step_id:
                return st
        raise SagaStateError(f"Step {step_id} not found in saga {saga.saga_id}")
