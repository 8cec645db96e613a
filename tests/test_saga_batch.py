"""Batched saga chains (K13/K14, BASELINE config 4) against the scalar
SagaOrchestrator, the fused kernel against the hipGraph step loop, and the
device against the host twin."""

from __future__ import annotations

import asyncio
import os

import pytest
import torch

from agent_hypervisor_amd.models.saga_engine import NEVER, SagaBatchEngine, SagaOutcomes
from hypervisor.saga.orchestrator import SagaOrchestrator

STATE_FIELDS = ("step_state", "retry_count", "step_error", "started_us", "completed_us", "saga_state",
                "saga_completed_us", "failed_step", "comp_failed", "tick")


def test_extension_binds_torch_runtime():
    """_C must share torch's HIP runtime and RCCL (one runtime per process)."""
    import torch as _t

    from agent_hypervisor_amd._native import C

    libs = C.runtime_libraries()
    tdir = os.path.dirname(_t.__file__)
    assert libs["hip"].startswith(tdir) and libs["rccl"].startswith(tdir), libs


def _scalar_reference(o: SagaOutcomes, s: int, K: int, compensate=True):
    """Drive the Python orchestrator with executors that follow the outcome table."""
    orch = SagaOrchestrator()
    orch.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    g = orch.create_saga("sess")
    steps = []
    for k in range(K):
        steps.append(orch.add_step(g.saga_id, f"a{k}", "did:x", "/x",
                                   undo_api="/u" if o.has_undo[s, k] else None,
                                   max_retries=int(o.max_retries[s, k])))

    async def run():
        for k, st in enumerate(steps):
            calls = {"n": 0}
            fails = int(o.fail_attempts[s, k])

            async def ex(calls=calls, fails=fails):
                calls["n"] += 1
                if fails == NEVER or calls["n"] <= fails:
                    raise RuntimeError("executor failed")
                return "ok"

            try:
                await orch.execute_step(g.saga_id, st.step_id, ex)
            except RuntimeError:
                if compensate:
                    cf = {st2.step_id: int(o.comp_fail[s, j]) for j, st2 in enumerate(steps)}

                    async def comp(step):
                        if cf[step.step_id]:
                            raise RuntimeError("undo down")
                        return "undone"

                    await orch.compensate(g.saga_id, comp)
                return
        from hypervisor.saga.state_machine import SagaState

        g.transition(SagaState.COMPLETED)

    asyncio.run(run())
    return g


@pytest.mark.parametrize("retries", [0, 2])
def test_fused_host_matches_orchestrator(retries):
    S, K = 300, 10
    o = SagaOutcomes.synthetic(S, K, p_fail=0.08, p_comp_fail=0.2, p_no_undo=0.15, max_retries=retries, seed=5)
    # some steps succeed after transient failures
    o.fail_attempts[::7, 3] = 1
    eng = SagaBatchEngine(S, K, device="cpu")
    stats = eng.run(o, now_us=1_000_000)
    for s in range(S):
        ref = _scalar_reference(o, s, K)
        got = eng.materialize(s)
        assert got.state == ref.state, s
        assert [st.state for st in got.steps] == [st.state for st in ref.steps], s
        assert [st.retry_count for st in got.steps] == [st.retry_count for st in ref.steps], s
        assert [st.error is None for st in got.steps] == [st.error is None for st in ref.steps], s
        assert [st.error == "No Undo_API available" for st in got.steps] == [
            st.error == "No Undo_API available" for st in ref.steps], s
        assert (got.completed_at is None) == (ref.completed_at is None)
        assert got.error == ref.error
    assert int(stats.sum()) > 0
    assert int(stats[0] + stats[1]) == S  # every saga ends COMPLETED or ESCALATED when compensating


def test_without_compensation_sagas_fail():
    S, K = 50, 4
    o = SagaOutcomes.synthetic(S, K, p_fail=0.3, seed=2)
    eng = SagaBatchEngine(S, K, device="cpu", compensate=False)
    st = eng.run(o, now_us=5)
    failed = int((o.fail_attempts == NEVER).any(dim=1).sum())
    assert int(st[2]) == failed and int(st[0]) == S - failed and int(st[3]) == 0


def test_timestamps_strictly_ordered():
    o = SagaOutcomes.synthetic(20, 10, p_fail=0.2, seed=9)
    eng = SagaBatchEngine(20, 10, device="cpu")
    eng.run(o, now_us=1000)
    for s in range(20):
        t = [x for x in eng.started_us[s].tolist() + eng.completed_us[s].tolist() if x]
        assert len(set(t)) == len(t) and min(t) >= 1000


def test_step_loop_equals_fused_cpu():
    S, K = 200, 10
    o = SagaOutcomes.synthetic(S, K, p_fail=0.1, p_comp_fail=0.1, p_no_undo=0.1, max_retries=1, seed=3)
    a, b = SagaBatchEngine(S, K, device="cpu"), SagaBatchEngine(S, K, device="cpu")
    sa = a.run(o, now_us=77).clone()
    sb = b.run_step_loop(o, now_us=77).clone()
    assert torch.equal(sa, sb)
    for f in STATE_FIELDS:
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_bad_shapes():
    eng = SagaBatchEngine(4, 3, device="cpu")
    with pytest.raises(ValueError):
        eng.run(SagaOutcomes.synthetic(4, 2))
    with pytest.raises(ValueError):
        SagaBatchEngine(4, 65, device="cpu")


@pytest.mark.gpu
def test_device_fused_and_graph_loop_match_host(cuda_device):
    S, K = 100_000, 10
    o = SagaOutcomes.synthetic(S, K, p_fail=0.05, p_comp_fail=0.1, p_no_undo=0.05, max_retries=1, seed=11)
    host = SagaBatchEngine(S, K, device="cpu")
    hs = host.run(o, now_us=123456).clone()
    dev = SagaBatchEngine(S, K, device=str(cuda_device))
    od = o.to(cuda_device)
    ds = dev.run(od, now_us=123456).clone()
    torch.cuda.synchronize(cuda_device)
    assert torch.equal(ds.cpu(), hs)
    for f in STATE_FIELDS:
        assert torch.equal(getattr(dev, f).cpu(), getattr(host, f)), f
    loop = SagaBatchEngine(S, K, device=str(cuda_device))
    loop.run_step_loop(od, now_us=123456)
    loop.replay()
    loop.replay()
    torch.cuda.synchronize(cuda_device)
    assert torch.equal(loop.stats.cpu(), hs)
    for f in STATE_FIELDS:
        assert torch.equal(getattr(loop, f).cpu(), getattr(host, f)), f
