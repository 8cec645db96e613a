"""Sagas: step/saga state machines, orchestrator (execute, retries, timeouts,
reverse-order compensation and escalation), fan-out policies, semantic
checkpoints and the declarative DSL (reference saga/*.py; SURVEY §2 C28–C35)."""

from __future__ import annotations

import asyncio

import pytest

from hypervisor import config
from hypervisor.saga.checkpoint import CheckpointManager, SemanticCheckpoint
from hypervisor.saga.dsl import SagaDSLError, SagaDSLParser
from hypervisor.saga.fan_out import FanOutOrchestrator, FanOutPolicy, policy_satisfied
from hypervisor.saga.orchestrator import SagaOrchestrator, SagaTimeoutError
from hypervisor.saga.state_machine import Saga, SagaState, SagaStateError, SagaStep, StepState


def _step(sid="s1", undo="/undo", timeout=300, retries=0) -> SagaStep:
    return SagaStep(step_id=sid, action_id="act", agent_did="did:a", execute_api="/x", undo_api=undo,
                    timeout_seconds=timeout, max_retries=retries)


def _orch() -> SagaOrchestrator:
    o = SagaOrchestrator()
    o.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    return o


async def _ok():
    return {"ok": True}


async def _boom():
    raise RuntimeError("boom")


# ------------------------------------------------------------ state machines


class TestStepStateMachine:
    def test_happy_path_stamps(self):
        s = _step()
        s.transition(StepState.EXECUTING)
        assert s.started_at is not None and s.completed_at is None
        s.transition(StepState.COMMITTED)
        assert s.completed_at is not None

    @pytest.mark.parametrize("path", [
        ["executing", "failed"],
        ["executing", "committed", "compensating", "compensated"],
        ["executing", "committed", "compensating", "compensation_failed"],
    ])
    def test_valid_paths(self, path):
        s = _step()
        for p in path:
            s.transition(StepState(p))
        assert s.state.value == path[-1]

    @pytest.mark.parametrize("src,dst", [("pending", "committed"), ("committed", "executing"),
                                         ("compensated", "compensating"), ("failed", "executing"),
                                         ("pending", "compensating")])
    def test_invalid(self, src, dst):
        s = _step()
        s.state = StepState(src)
        with pytest.raises(SagaStateError, match="Invalid step transition"):
            s.transition(StepState(dst))


class TestSagaStateMachine:
    def test_paths(self):
        g = Saga("g", "s")
        g.transition(SagaState.COMPENSATING)
        g.transition(SagaState.ESCALATED)
        assert g.completed_at is not None
        h = Saga("h", "s")
        h.transition(SagaState.COMPLETED)
        with pytest.raises(SagaStateError, match="Invalid saga transition"):
            h.transition(SagaState.RUNNING)

    def test_committed_views_and_roundtrip(self):
        g = Saga("g", "s", steps=[_step("a"), _step("b"), _step("c")])
        for s in g.steps[:2]:
            s.transition(StepState.EXECUTING)
            s.transition(StepState.COMMITTED)
        assert [s.step_id for s in g.committed_steps_reversed] == ["b", "a"]
        d = g.to_dict()
        back = Saga.from_dict(d)
        assert back.to_dict() == d


# -------------------------------------------------------------- orchestrator


class TestOrchestrator:
    async def test_execute_commits(self):
        o = _orch()
        g = o.create_saga("sess")
        assert g.saga_id.startswith("saga:") and o.active_sagas == [g]
        st = o.add_step(g.saga_id, "deploy", "did:a", "/deploy", undo_api="/undeploy")
        assert st.step_id.startswith("step:")
        assert await o.execute_step(g.saga_id, st.step_id, _ok) == {"ok": True}
        assert st.state == StepState.COMMITTED and st.execute_result == {"ok": True}

    async def test_failure_sets_error_and_raises(self):
        o = _orch()
        g = o.create_saga("sess")
        st = o.add_step(g.saga_id, "a", "d", "/x")
        with pytest.raises(RuntimeError, match="boom"):
            await o.execute_step(g.saga_id, st.step_id, _boom)
        assert st.state == StepState.FAILED and st.error == "boom"

    async def test_retries_then_success(self):
        o = _orch()
        g = o.create_saga("sess")
        st = o.add_step(g.saga_id, "a", "d", "/x", max_retries=2)
        calls = {"n": 0}

        async def flaky():
            calls["n"] += 1
            if calls["n"] < 3:
                raise RuntimeError("transient")
            return "done"

        assert await o.execute_step(g.saga_id, st.step_id, flaky) == "done"
        assert st.retry_count == 2 and st.state == StepState.COMMITTED and st.error is None

    async def test_timeout(self):
        o = _orch()
        g = o.create_saga("sess")
        st = o.add_step(g.saga_id, "a", "d", "/x", timeout_seconds=0)

        async def slow():
            await asyncio.sleep(0.05)

        st.timeout_seconds = 0.01
        with pytest.raises(SagaTimeoutError, match="timed out"):
            await o.execute_step(g.saga_id, st.step_id, slow)
        assert st.state == StepState.FAILED

    async def test_unknown_ids(self):
        o = _orch()
        with pytest.raises(SagaStateError, match="not found"):
            o.add_step("saga:nope", "a", "d", "/x")
        g = o.create_saga("s")
        with pytest.raises(SagaStateError, match="not found"):
            await o.execute_step(g.saga_id, "step:nope", _ok)

    async def test_compensation_reverse_order_completes(self):
        o = _orch()
        g = o.create_saga("s")
        steps = [o.add_step(g.saga_id, f"a{k}", "d", "/x", undo_api="/u") for k in range(3)]
        for st in steps:
            await o.execute_step(g.saga_id, st.step_id, _ok)
        order = []

        async def comp(step):
            order.append(step.step_id)
            return "undone"

        failed = await o.compensate(g.saga_id, comp)
        assert failed == [] and order == [s.step_id for s in reversed(steps)]
        assert g.state == SagaState.COMPLETED and all(s.state == StepState.COMPENSATED for s in steps)
        assert o.active_sagas == []

    async def test_compensation_failures_escalate(self):
        o = _orch()
        g = o.create_saga("s")
        a = o.add_step(g.saga_id, "a", "d", "/x", undo_api=None)
        b = o.add_step(g.saga_id, "b", "d", "/x", undo_api="/u")
        for st in (a, b):
            await o.execute_step(g.saga_id, st.step_id, _ok)

        async def bad(step):
            raise RuntimeError("undo down")

        failed = await o.compensate(g.saga_id, bad)
        assert {s.step_id for s in failed} == {a.step_id, b.step_id}
        assert a.error == "No Undo_API available" and b.error == "Compensation failed: undo down"
        assert g.state == SagaState.ESCALATED and "2 step(s) failed compensation" in g.error

    async def test_sagas_listing(self):
        o = _orch()
        g1, g2 = o.create_saga("s"), o.create_saga("s")
        assert o.sagas == [g1, g2] and o.get_saga(g2.saga_id) is g2 and o.get_saga("x") is None


# --------------------------------------------------------------------- fan-out


class TestFanOut:
    @pytest.mark.parametrize("policy,succ,total,ok", [
        ("all_must_succeed", 3, 3, True), ("all_must_succeed", 2, 3, False),
        ("majority_must_succeed", 2, 3, True), ("majority_must_succeed", 2, 4, False),
        ("any_must_succeed", 1, 5, True), ("any_must_succeed", 0, 5, False),
        ("all_must_succeed", 0, 0, True),
    ])
    def test_policy(self, policy, succ, total, ok):
        assert policy_satisfied(FanOutPolicy(policy), succ, total) == ok

    async def test_execute_all_success(self):
        fo = FanOutOrchestrator()
        g = fo.create_group("saga", FanOutPolicy.ALL_MUST_SUCCEED)
        steps = [_step(f"b{k}") for k in range(3)]
        for s in steps:
            fo.add_branch(g.group_id, s)
        assert fo.active_groups == [g]
        out = await fo.execute(g.group_id, {s.step_id: _ok for s in steps})
        assert out.resolved and out.policy_satisfied and out.success_count == 3 and out.compensation_needed == []
        assert all(s.state == StepState.COMMITTED for s in steps) and fo.active_groups == []

    async def test_policy_failure_lists_compensation(self):
        fo = FanOutOrchestrator()
        g = fo.create_group("saga", FanOutPolicy.MAJORITY_MUST_SUCCEED)
        steps = [_step(f"b{k}") for k in range(3)]
        for s in steps:
            fo.add_branch(g.group_id, s)
        out = await fo.execute(g.group_id, {"b0": _ok, "b1": _boom})  # b2 has no executor
        assert not out.policy_satisfied and out.failure_count == 2
        assert out.compensation_needed == ["b0"]
        assert steps[1].state == StepState.FAILED and steps[1].error == "boom"
        assert out.branches[2].error == "No executor for step b2"

    async def test_branch_timeout_message(self):
        fo = FanOutOrchestrator()
        g = fo.create_group("saga", FanOutPolicy.ANY_MUST_SUCCEED)
        s = _step("slow")
        s.timeout_seconds = 0.01
        fo.add_branch(g.group_id, s)

        async def slow():
            await asyncio.sleep(0.05)

        out = await fo.execute(g.group_id, {"slow": slow})
        assert not out.policy_satisfied and out.branches[0].error.startswith("Branch timed out")

    def test_unknown_group(self):
        fo = FanOutOrchestrator()
        assert fo.get_group("x") is None
        with pytest.raises(ValueError):
            fo.add_branch("x", _step())


# ---------------------------------------------------------------- checkpoints


class TestCheckpoints:
    def test_save_and_lookup(self):
        cm = CheckpointManager()
        c = cm.save("g1", "s1", "db migrated", {"rows": 10})
        assert c.goal_hash == SemanticCheckpoint.compute_goal_hash("db migrated", "s1") and len(c.goal_hash) == 16
        assert cm.is_achieved("g1", "db migrated", "s1")
        assert not cm.is_achieved("g1", "db migrated", "s2")
        assert cm.get_checkpoint("g1", "db migrated", "s1").state_snapshot == {"rows": 10}

    def test_invalidate_and_replay_plan(self):
        cm = CheckpointManager()
        cm.save("g", "s1", "goal1")
        cm.save("g", "s2", "goal2")
        assert cm.get_replay_plan("g", ["s1", "s2", "s3"]) == ["s3"]
        assert cm.invalidate("g", "s1", "drift") == 1
        assert cm.get_replay_plan("g", ["s1", "s2", "s3"]) == ["s1", "s3"]
        assert cm.total_checkpoints == 2 and cm.valid_checkpoints == 1
        assert not cm.is_achieved("g", "goal1", "s1")

    def test_same_goal_in_two_sagas_is_independent(self):
        cm = CheckpointManager()
        cm.save("g1", "s", "same goal")
        cm.save("g2", "s", "same goal")
        assert cm.is_achieved("g1", "same goal", "s") and cm.is_achieved("g2", "same goal", "s")

    def test_parity_mode_reproduces_global_goal_index(self):
        config.set_parity_mode(True)
        cm = CheckpointManager()
        cm.save("g1", "s", "same goal")
        cm.save("g2", "s", "same goal")
        # reference indexes by goal hash only: the later save shadows the first (Q17)
        assert not cm.is_achieved("g1", "same goal", "s")


# ------------------------------------------------------------------------ DSL


DEF = {
    "name": "deploy",
    "session_id": "sess",
    "steps": [
        {"id": "build", "action_id": "ci.build", "agent": "did:ci", "execute_api": "/b", "undo_api": "/ub"},
        {"id": "test-a", "action_id": "ci.test", "agent": "did:ci", "timeout": 60, "retries": 2},
        {"id": "test-b", "action_id": "ci.test", "agent": "did:ci2", "checkpoint_goal": "tests green"},
    ],
    "fan_out": [{"policy": "majority_must_succeed", "branches": ["test-a", "test-b"]}],
    "metadata": {"owner": "team"},
}


class TestDSL:
    def test_parse(self):
        d = SagaDSLParser().parse(DEF)
        assert d.name == "deploy" and d.step_ids == ["build", "test-a", "test-b"]
        assert d.saga_id.startswith("saga:") and d.metadata == {"owner": "team"}
        assert d.fan_outs[0].policy == FanOutPolicy.MAJORITY_MUST_SUCCEED
        assert [s.id for s in d.sequential_steps] == ["build"] and d.fan_out_step_ids == {"test-a", "test-b"}
        assert d.steps[1].timeout == 60 and d.steps[1].retries == 2 and d.steps[2].checkpoint_goal == "tests green"

    def test_to_saga_steps(self):
        p = SagaDSLParser()
        steps = p.to_saga_steps(p.parse(DEF))
        assert [s.step_id for s in steps] == ["build", "test-a", "test-b"]
        assert steps[0].undo_api == "/ub" and steps[1].max_retries == 2 and steps[1].timeout_seconds == 60

    def test_yaml(self):
        text = """
name: y
session_id: s
saga_id: saga:fixed
steps:
  - {id: one, action_id: a, agent: did:x}
"""
        d = SagaDSLParser().parse_yaml(text)
        assert d.saga_id == "saga:fixed" and d.steps[0].agent == "did:x"
        with pytest.raises(SagaDSLError, match="mapping"):
            SagaDSLParser().parse_yaml("- just a list")

    @pytest.mark.parametrize("mutate,msg", [
        (lambda d: d.pop("name"), "'name'"),
        (lambda d: d.pop("session_id"), "'session_id'"),
        (lambda d: d.update(steps=[]), "at least one step"),
        (lambda d: d["steps"].append(dict(d["steps"][0])), "Duplicate step ID"),
        (lambda d: d["steps"][0].pop("agent"), "must have an 'agent'"),
        (lambda d: d["steps"][0].pop("action_id"), "must have an 'action_id'"),
        (lambda d: d.update(fan_out=[{"policy": "bogus", "branches": ["test-a", "test-b"]}]), "Invalid fan-out"),
        (lambda d: d.update(fan_out=[{"branches": ["test-a"]}]), "at least 2 branches"),
        (lambda d: d.update(fan_out=[{"branches": ["test-a", "nope"]}]), "not a valid step ID"),
    ])
    def test_errors(self, mutate, msg):
        import copy

        d = copy.deepcopy(DEF)
        mutate(d)
        with pytest.raises(SagaDSLError, match=msg):
            SagaDSLParser().parse(d)

    def test_validate_collects_all(self):
        errs = SagaDSLParser().validate({"steps": [{"id": "a"}, {"id": "a", "action_id": "x", "agent": "y"}]})
        assert "Missing 'name'" in errs and "Missing 'session_id'" in errs
        assert "Duplicate step ID: a" in errs and "Step a missing 'action_id'" in errs
        assert SagaDSLParser().validate({"name": "n", "session_id": "s"}) == ["Missing 'steps'"]
