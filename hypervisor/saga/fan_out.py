"""Parallel saga fan-out with ALL / MAJORITY / ANY success policies.

Parity target: reference ``saga/fan_out.py:19-192``.

* ALL: ``success == total`` (vacuously true for zero branches); MAJORITY:
  ``success > total/2``; ANY: ``success ≥ 1``.
* Each branch: EXECUTING → ``executor()`` under the step timeout → COMMITTED;
  any exception (timeout included) → FAILED with ``error = str(e)``.  All branches
  run concurrently under one overall ``timeout_seconds``.
* ``compensation_needed`` lists succeeded step ids only when the policy failed;
  no compensation is run here.

Fix: a timed-out branch records
``"Branch timed out after Ns"`` — ``str(TimeoutError())`` is empty, so the
reference's ``failure_count`` did not count timeouts.  Parity mode keeps "".

Batched policy evaluation (segmented success counts over thousands of groups)
is kernel K15 (``fanout_policy``).
"""

from __future__ import annotations

import asyncio
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Callable, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor import config as _cfg
from hypervisor.saga._timeout import await_with_timeout
from hypervisor.saga.state_machine import SagaStep, StepState


class FanOutPolicy(str, Enum):
    ALL_MUST_SUCCEED = "all_must_succeed"
    MAJORITY_MUST_SUCCEED = "majority_must_succeed"
    ANY_MUST_SUCCEED = "any_must_succeed"


POLICY_CODE = {p: i for i, p in enumerate(FanOutPolicy)}


def policy_satisfied(policy: FanOutPolicy, success: int, total: int) -> bool:
    """Scalar twin of the K15 device predicate."""
    if policy == FanOutPolicy.ALL_MUST_SUCCEED:
        return success == total
    if policy == FanOutPolicy.MAJORITY_MUST_SUCCEED:
        return success > total / 2
    if policy == FanOutPolicy.ANY_MUST_SUCCEED:
        return success >= 1
    return False


@dataclass
class FanOutBranch:
    branch_id: str = field(default_factory=lambda: _C.hex_id("branch:", 8))
    step: Optional[SagaStep] = None
    result: Any = None
    error: Optional[str] = None
    succeeded: bool = False


@dataclass
class FanOutGroup:
    group_id: str = field(default_factory=lambda: _C.hex_id("fanout:", 8))
    saga_id: str = ""
    policy: FanOutPolicy = FanOutPolicy.ALL_MUST_SUCCEED
    branches: list[FanOutBranch] = field(default_factory=list)
    resolved: bool = False
    policy_satisfied: bool = False
    compensation_needed: list[str] = field(default_factory=list)

    @property
    def success_count(self) -> int:
        return sum(1 for b in self.branches if b.succeeded)

    @property
    def failure_count(self) -> int:
        return sum(1 for b in self.branches if not b.succeeded and b.error)

    @property
    def total_branches(self) -> int:
        return len(self.branches)

    def check_policy(self) -> bool:
        return policy_satisfied(self.policy, self.success_count, self.total_branches)


class FanOutOrchestrator:
    def __init__(self) -> None:
        self._groups: dict[str, FanOutGroup] = {}

    def create_group(self, saga_id: str, policy: FanOutPolicy = FanOutPolicy.ALL_MUST_SUCCEED) -> FanOutGroup:
        g = FanOutGroup(saga_id=saga_id, policy=policy)
        self._groups[g.group_id] = g
        return g

    def add_branch(self, group_id: str, step: SagaStep) -> FanOutBranch:
        g = self._get_group(group_id)
        b = FanOutBranch(step=step)
        g.branches.append(b)
        return b

    async def execute(
        self,
        group_id: str,
        executors: dict[str, Callable[..., Any]],
        timeout_seconds: int = 300,
    ) -> FanOutGroup:
        g = self._get_group(group_id)
        await self.run_branches(g, executors, timeout_seconds)
        g.policy_satisfied = g.check_policy()
        g.resolved = True
        if not g.policy_satisfied:
            g.compensation_needed = [b.step.step_id for b in g.branches if b.succeeded and b.step]
        return g

    async def execute_groups(
        self,
        group_ids: list[str],
        executors: dict[str, Callable[..., Any]],
        timeout_seconds: int = 300,
        device: Optional[str] = None,
    ) -> list[FanOutGroup]:
        """:meth:`execute` for many groups at once (all branches concurrent).
        With ``device`` every group's policy and compensation list come from one
        K15 launch over the gathered branch outcomes."""
        groups = [self._get_group(i) for i in group_ids]
        if device is not None:
            from agent_hypervisor_amd.models.saga_runner import execute_fanout_groups

            return await execute_fanout_groups(self, groups, executors, timeout_seconds, device)
        await asyncio.gather(*(self.execute(g.group_id, executors, timeout_seconds) for g in groups))
        return groups

    async def run_branches(self, g: FanOutGroup, executors: dict[str, Callable[..., Any]],
                           timeout_seconds: int) -> None:
        """Every branch of ``g`` concurrently under one overall timeout."""
        parity = _cfg.parity_mode()

        async def run(b: FanOutBranch) -> None:
            st = b.step
            if st is None:
                b.error = "No step assigned"
                return
            fn = executors.get(st.step_id)
            if fn is None:
                b.error = f"No executor for step {st.step_id}"
                return
            try:
                st.transition(StepState.EXECUTING)
                res = await await_with_timeout(fn(), st.timeout_seconds)
            except asyncio.TimeoutError as e:
                msg = str(e) if parity else f"Branch timed out after {st.timeout_seconds}s"
                self._fail(b, msg)
            except Exception as e:
                self._fail(b, str(e))
            else:
                b.result = res
                b.succeeded = True
                st.execute_result = res
                st.transition(StepState.COMMITTED)

        await asyncio.wait_for(
            asyncio.gather(*(run(b) for b in g.branches), return_exceptions=True),
            timeout=timeout_seconds,
        )

    @staticmethod
    def _fail(b: FanOutBranch, msg: str) -> None:
        b.error = msg
        b.succeeded = False
        b.step.error = msg
        b.step.transition(StepState.FAILED)

    def get_group(self, group_id: str) -> Optional[FanOutGroup]:
        return self._groups.get(group_id)

    def _get_group(self, group_id: str) -> FanOutGroup:
        g = self._groups.get(group_id)
        if g is None:
            raise ValueError(f"Fan-out group {group_id} not found")
        return g

    @property
    def active_groups(self) -> list[FanOutGroup]:
        return [g for g in self._groups.values() if not g.resolved]
