"""Declarative saga definitions (dict / YAML-loaded dict).

Parity target: reference ``saga/dsl.py:48-238``.  Required: ``name``,
``session_id``, a non-empty ``steps`` list, and per step ``id``, ``action_id``,
``agent``; step ids are unique.  ``fan_out`` entries need a valid policy string,
≥ 2 branches and existing step ids.  Step defaults: timeout 300, retries 0;
``saga_id`` defaults to ``saga:<8 hex>``.

Addition: :meth:`SagaDSLParser.parse_yaml` accepts YAML text (safe loader), which
the reference's docstring promised but never implemented.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor.saga.fan_out import FanOutPolicy
from hypervisor.saga.state_machine import SagaStep


class SagaDSLError(Exception):
    """Invalid saga definition."""


def _short_saga_id() -> str:
    return _C.hex_id("saga:", 8)


@dataclass
class SagaDSLStep:
    id: str = ""
    action_id: str = ""
    agent: str = ""
    execute_api: str = ""
    undo_api: Optional[str] = None
    timeout: int = 300
    retries: int = 0
    checkpoint_goal: Optional[str] = None


@dataclass
class SagaDSLFanOut:
    policy: FanOutPolicy = FanOutPolicy.ALL_MUST_SUCCEED
    branch_step_ids: list[str] = field(default_factory=list)


@dataclass
class SagaDefinition:
    name: str = ""
    session_id: str = ""
    saga_id: str = field(default_factory=_short_saga_id)
    steps: list[SagaDSLStep] = field(default_factory=list)
    fan_outs: list[SagaDSLFanOut] = field(default_factory=list)
    metadata: dict[str, Any] = field(default_factory=dict)

    @property
    def step_ids(self) -> list[str]:
        return [s.id for s in self.steps]

    @property
    def fan_out_step_ids(self) -> set[str]:
        return {sid for fo in self.fan_outs for sid in fo.branch_step_ids}

    @property
    def sequential_steps(self) -> list[SagaDSLStep]:
        fo = self.fan_out_step_ids
        return [s for s in self.steps if s.id not in fo]


class SagaDSLParser:
    def parse(self, definition: dict[str, Any]) -> SagaDefinition:
        name = definition.get("name", "")
        if not name:
            raise SagaDSLError("Saga definition must have a 'name'")
        session_id = definition.get("session_id", "")
        if not session_id:
            raise SagaDSLError("Saga definition must have a 'session_id'")
        raw_steps = definition.get("steps", [])
        if not raw_steps:
            raise SagaDSLError("Saga must have at least one step")
        steps: list[SagaDSLStep] = []
        seen: set[str] = set()
        for raw in raw_steps:
            st = self._parse_step(raw)
            if st.id in seen:
                raise SagaDSLError(f"Duplicate step ID: {st.id}")
            seen.add(st.id)
            steps.append(st)
        fan_outs = [self._parse_fan_out(fo, seen) for fo in definition.get("fan_out", [])]
        return SagaDefinition(
            name=name,
            session_id=session_id,
            saga_id=definition["saga_id"] if "saga_id" in definition else _short_saga_id(),
            steps=steps,
            fan_outs=fan_outs,
            metadata=definition.get("metadata", {}),
        )

    def parse_yaml(self, text: str) -> SagaDefinition:
        import yaml

        data = yaml.safe_load(text)
        if not isinstance(data, dict):
            raise SagaDSLError("YAML saga definition must be a mapping")
        return self.parse(data)

    def _parse_step(self, raw: dict) -> SagaDSLStep:
        sid = raw.get("id", "")
        if not sid:
            raise SagaDSLError("Each step must have an 'id'")
        action = raw.get("action_id", "")
        if not action:
            raise SagaDSLError(f"Step {sid} must have an 'action_id'")
        agent = raw.get("agent", "")
        if not agent:
            raise SagaDSLError(f"Step {sid} must have an 'agent'")
        return SagaDSLStep(
            id=sid,
            action_id=action,
            agent=agent,
            execute_api=raw.get("execute_api", ""),
            undo_api=raw.get("undo_api"),
            timeout=raw.get("timeout", 300),
            retries=raw.get("retries", 0),
            checkpoint_goal=raw.get("checkpoint_goal"),
        )

    def _parse_fan_out(self, raw: dict, valid_step_ids: set[str]) -> SagaDSLFanOut:
        pstr = raw.get("policy", "all_must_succeed")
        try:
            policy = FanOutPolicy(pstr)
        except ValueError:
            raise SagaDSLError(
                f"Invalid fan-out policy: {pstr}. Valid: {[p.value for p in FanOutPolicy]}"
            ) from None
        branches = raw.get("branches", [])
        if len(branches) < 2:
            raise SagaDSLError("Fan-out must have at least 2 branches")
        for bid in branches:
            if bid not in valid_step_ids:
                raise SagaDSLError(f"Fan-out branch '{bid}' is not a valid step ID")
        return SagaDSLFanOut(policy=policy, branch_step_ids=branches)

    def to_saga_steps(self, definition: SagaDefinition) -> list[SagaStep]:
        return [
            SagaStep(
                step_id=s.id,
                action_id=s.action_id,
                agent_did=s.agent,
                execute_api=s.execute_api,
                undo_api=s.undo_api,
                timeout_seconds=s.timeout,
                max_retries=s.retries,
            )
            for s in definition.steps
        ]

    def validate(self, definition: dict[str, Any]) -> list[str]:
        errs: list[str] = []
        if not definition.get("name"):
            errs.append("Missing 'name'")
        if not definition.get("session_id"):
            errs.append("Missing 'session_id'")
        steps = definition.get("steps")
        if not steps:
            errs.append("Missing 'steps'")
            return errs
        ids: set[str] = set()
        for i, st in enumerate(steps):
            sid = st.get("id")
            if not sid:
                errs.append(f"Step {i} missing 'id'")
            elif sid in ids:
                errs.append(f"Duplicate step ID: {sid}")
            else:
                ids.add(sid)
            label = st.get("id", i)
            if not st.get("action_id"):
                errs.append(f"Step {label} missing 'action_id'")
            if not st.get("agent"):
                errs.append(f"Step {label} missing 'agent'")
        return errs
