"""SagaOrchestrator.execute_sagas / FanOutOrchestrator.execute_groups on the
device FSM (K13/K14 step-loop graph, K15 policy) vs the host orchestrators.

Both run the same stub coroutines — scripted per step: fail N attempts (by
exception or by exceeding the step timeout) before succeeding or never,
compensators that succeed, raise or time out — and every saga / step / group
field the reference exposes is compared.  ``cpu`` drives the kernels' host
twins; ``cuda`` the gfx950 graph replay (``-m gpu``)."""

from __future__ import annotations

import asyncio
import random

import pytest

from hypervisor.saga.fan_out import FanOutOrchestrator, FanOutPolicy
from hypervisor.saga.orchestrator import SagaOrchestrator
from hypervisor.saga.state_machine import SagaStep

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
TIMEOUT = 0.02


def _script(seed: int, n_sagas: int, k_choices=(1, 3, 5)):
    rng = random.Random(seed)
    plan = []
    for _ in range(n_sagas):
        steps = []
        for _ in range(rng.choice(k_choices)):
            steps.append(dict(
                fails=rng.choice([0, 0, 0, 1, 2, 99]),  # 99: never succeeds
                kind=rng.choice(["exc", "exc", "timeout"]),
                retries=rng.choice([0, 0, 1, 2]),
                undo=rng.random() < 0.85,
                comp=rng.choice(["ok", "ok", "ok", "exc", "timeout"]),
            ))
        plan.append(steps)
    return plan


def _build(orch: SagaOrchestrator, plan):
    ids, executors, comp_of = [], {}, {}
    for i, steps in enumerate(plan):
        sg = orch.create_saga(f"session-{i}")
        ids.append(sg.saga_id)
        for k, spec in enumerate(steps):
            st = orch.add_step(sg.saga_id, f"a{i}.{k}", "did:x", "/exec", "/undo" if spec["undo"] else None,
                               timeout_seconds=TIMEOUT, max_retries=spec["retries"])
            calls = {"n": 0}

            async def ex(spec=spec, calls=calls, tag=(i, k)):
                calls["n"] += 1
                if calls["n"] <= spec["fails"]:
                    if spec["kind"] == "timeout":
                        await asyncio.sleep(TIMEOUT * 5)
                    raise RuntimeError(f"boom {tag} #{calls['n']}")
                return {"ok": tag}

            executors[st.step_id] = ex
            comp_of[st.step_id] = spec["comp"]

    async def compensator(step: SagaStep):
        mode = comp_of[step.step_id]
        if mode == "exc":
            raise ValueError(f"undo failed {step.action_id}")
        if mode == "timeout":
            await asyncio.sleep(TIMEOUT * 5)
        return f"undone {step.action_id}"

    return ids, executors, compensator


def _view(orch, ids):
    out = []
    for sid in ids:
        sg = orch.get_saga(sid)
        out.append((sg.state, sg.error, [(st.action_id, st.state, st.retry_count,
                                          st.error.replace(st.step_id, "<id>") if st.error else st.error,
                                          st.execute_result, st.compensation_result) for st in sg.steps]))
    return out


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("compensate", [True, False])
def test_execute_sagas_device_matches_host(device, compensate):
    if device == "cuda":
        import torch

        if not torch.cuda.is_available():
            pytest.fail("GPU test selected but no HIP device is visible")
    plan = _script(11 if compensate else 12, 60)
    host, dev = SagaOrchestrator(), SagaOrchestrator()
    host.DEFAULT_RETRY_DELAY_SECONDS = dev.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    h_ids, h_ex, h_comp = _build(host, plan)
    d_ids, d_ex, d_comp = _build(dev, plan)
    asyncio.run(host.execute_sagas(h_ids, h_ex, h_comp, compensate=compensate))
    asyncio.run(dev.execute_sagas(d_ids, d_ex, d_comp, compensate=compensate, device=device))
    hv, dv = _view(host, h_ids), _view(dev, d_ids)
    assert hv == dv
    states = {s for s, _, _ in hv}
    assert len(states) >= 2  # the script exercises more than one outcome
    # a second batch of the same shape replays the captured graph with new outcomes
    plan2 = _script(21, 60)
    h2, d2 = SagaOrchestrator(), dev
    h2.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    h_ids, h_ex, h_comp = _build(h2, plan2)
    d_ids, d_ex, d_comp = _build(d2, plan2)
    asyncio.run(h2.execute_sagas(h_ids, h_ex, h_comp, compensate=compensate))
    asyncio.run(d2.execute_sagas(d_ids, d_ex, d_comp, compensate=compensate, device=device))
    assert _view(h2, h_ids) == _view(d2, d_ids)


@pytest.mark.parametrize("device", DEVICES)
def test_fanout_groups_device_matches_host(device):
    if device == "cuda":
        import torch

        if not torch.cuda.is_available():
            pytest.fail("GPU test selected but no HIP device is visible")
    rng = random.Random(3)
    spec = [(rng.choice(list(FanOutPolicy)), [rng.random() < 0.6 for _ in range(rng.randint(0, 6))])
            for _ in range(80)]

    def build(fo: FanOutOrchestrator):
        gids, ex = [], {}
        for gi, (pol, outcomes) in enumerate(spec):
            g = fo.create_group(f"saga-{gi}", pol)
            gids.append(g.group_id)
            for bi, ok in enumerate(outcomes):
                st = SagaStep(step_id=f"step:{gi}:{bi}", action_id="a", agent_did="d", execute_api="/x",
                              timeout_seconds=1)
                fo.add_branch(g.group_id, st)

                async def run(ok=ok, tag=(gi, bi)):
                    if not ok:
                        raise RuntimeError(f"branch {tag} failed")
                    return tag

                ex[st.step_id] = run
        return gids, ex

    host, dev = FanOutOrchestrator(), FanOutOrchestrator()
    hg, hx = build(host)
    dg, dx = build(dev)
    asyncio.run(host.execute_groups(hg, hx))
    asyncio.run(dev.execute_groups(dg, dx, device=device))

    def view(fo, gids):
        return [(g.policy_satisfied, g.resolved, g.compensation_needed, g.success_count, g.failure_count,
                 [(b.succeeded, b.error, b.result) for b in g.branches]) for g in map(fo.get_group, gids)]

    assert view(host, hg) == view(dev, dg)


@pytest.mark.parametrize("delay", [0.0, 0.001])
def test_device_runner_mixed_executor_kinds_match_host(delay):
    """Executors that are plain functions (returning a non-awaitable: a failed
    attempt, as in the reference), futures, coroutines that raise before
    suspending, and retry delays — the device-decided rounds call each executor
    exactly as often as the host orchestrator does."""
    calls_h, calls_d = {}, {}

    def build(orch, calls):
        ids, ex = [], {}
        loop_kinds = ["coro", "raise_now", "plain", "future", "suspend"]
        for i in range(25):
            sg = orch.create_saga(f"s{i}")
            ids.append(sg.saga_id)
            for k in range(3):
                kind = loop_kinds[(i + k) % len(loop_kinds)]
                st = orch.add_step(sg.saga_id, f"a{i}.{k}", "did:x", "/e", "/u", timeout_seconds=1, max_retries=1)
                key = (i, k)

                def mk(kind=kind, key=key):
                    def fn():
                        calls[key] = calls.get(key, 0) + 1
                        if kind == "plain":
                            return "not awaitable"
                        if kind == "future":
                            f = asyncio.get_running_loop().create_future()
                            f.set_result(key)
                            return f

                        async def co():
                            if kind == "raise_now" and calls[key] == 1:
                                raise RuntimeError("first attempt fails")
                            if kind == "suspend":
                                await asyncio.sleep(0)
                            return key
                        return co()
                    return fn
                ex[st.step_id] = mk()
        return ids, ex

    async def comp(step):
        return "undone"

    host, dev = SagaOrchestrator(), SagaOrchestrator()
    host.DEFAULT_RETRY_DELAY_SECONDS = dev.DEFAULT_RETRY_DELAY_SECONDS = delay
    h_ids, h_ex = build(host, calls_h)
    d_ids, d_ex = build(dev, calls_d)
    asyncio.run(host.execute_sagas(h_ids, h_ex, comp))
    asyncio.run(dev.execute_sagas(d_ids, d_ex, comp, device="cpu"))
    assert _view(host, h_ids) == _view(dev, d_ids)
    assert calls_h == calls_d


def test_device_runner_writes_back_through_device_store_steps():
    """execute_sagas(device=...) on a device-store hypervisor's orchestrator: the
    states land in the store's step rows (the views' setters), as the host
    orchestrator's would."""
    from agent_hypervisor_amd.models.store import GovernanceStore
    from hypervisor import Hypervisor, SessionConfig

    st = GovernanceStore("cpu", caps={"S": 64, "G": 64, "T": 256})
    hv = Hypervisor(store=st)

    async def go():
        m = await hv.create_session(SessionConfig(), "did:c")
        orch = m.saga
        ids, ex = [], {}
        for i in range(6):
            sg = orch.create_saga(m.sso.session_id)
            ids.append(sg.saga_id)
            for k in range(3):
                step = orch.add_step(sg.saga_id, f"a{i}.{k}", "did:x", "/e", "/u", max_retries=0)
                fail = (i + k) % 4 == 0

                async def run(fail=fail):
                    if fail:
                        raise RuntimeError("no")
                    return "ok"
                ex[step.step_id] = run

        async def comp(step):
            return "undone"
        await orch.execute_sagas(ids, ex, comp, device="cpu")
        return orch, ids

    orch, ids = asyncio.run(go())
    states = [(orch.get_saga(i).state.value, [s_.state.value for s_ in orch.get_saga(i).steps]) for i in ids]
    assert any(s == "completed" for s, _ in states) and any("failed" in ss for _, ss in states)
    # the values read back come from the device rows
    row = orch.get_saga(ids[1]).steps[0]
    assert row.state.value == states[1][1][0] and "state" not in row.__dict__
    st.close()
