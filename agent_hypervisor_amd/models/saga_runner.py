"""Real saga executions driven through the device saga FSM (K13/K14) and
fan-out policy (K15).

:meth:`hypervisor.saga.orchestrator.SagaOrchestrator.execute_sagas` and
:meth:`hypervisor.saga.fan_out.FanOutOrchestrator.execute_groups` with a
``device`` land here.  The split of work:

* **host** — awaits the user's executor / compensator coroutines, concurrently
  across sagas (``asyncio.gather``), step by step in each saga's order: step k
  runs only in sagas whose steps < k committed, compensations walk committed
  steps in reverse — exactly the calls the reference orchestrator makes
  (saga/orchestrator.py:77-198).  Each step's outcome is reduced to the FSM's
  inputs: failing attempts before success (255 = never), the last failure's
  kind (exception / timeout), the compensation outcome, Undo_API presence and
  max_retries;
* **device** — one replay of the hipGraph-captured step loop (init, K ×
  execute, decide, K × compensate, finish; :class:`SagaBatchEngine`) turns
  those tables into every step/saga state, retry count, error code, transition
  timestamp and the batch counters.  The graph is captured once per (sagas,
  steps) shape and replayed for every later batch: outcomes are loaded into
  persistent buffers and the time base is a device scalar.

The resulting states are written back into the orchestrator's ``Saga`` /
``SagaStep`` objects; host-only payloads (executor results, exception texts)
are attached from the host side.  Sagas are batched by step count.
"""

from __future__ import annotations

import asyncio
from types import CoroutineType
from typing import Any, Callable, Optional, Sequence

import torch

from agent_hypervisor_amd.models.saga_engine import (
    ERR_COMP,
    ERR_COMP_TIMEOUT,
    ERR_EXEC,
    ERR_NO_UNDO,
    ERR_NONE,
    ERR_TIMEOUT,
    NEVER,
    SAGA_NAMES,
    STEP_NAMES,
    SagaBatchEngine,
    SagaOutcomes,
)
from hypervisor import _clock
from hypervisor.saga._timeout import await_with_timeout, resume_with_deadline

u8 = torch.uint8
_KIND_EXC, _KIND_TIMEOUT = 1, 2


class SagaBatchRunner:
    """Per-device cache of step-loop engines (one per batch shape)."""

    def __init__(self, device) -> None:
        from agent_hypervisor_amd.models.engine import resolve_device

        self.device = resolve_device(device)
        self._engines: dict[tuple[int, int, bool], SagaBatchEngine] = {}
        self.last_stats: Optional[list[int]] = None

    def engine(self, S: int, K: int, compensate: bool) -> SagaBatchEngine:
        key = (S, K, compensate)
        e = self._engines.get(key)
        if e is None:
            e = self._engines[key] = SagaBatchEngine(S, K, device=str(self.device), compensate=compensate)
        return e

    async def run(self, orch, sagas: Sequence, executors: dict[str, Callable[[], Any]],
                  compensator: Optional[Callable[[Any], Any]] = None, compensate: bool = True) -> list[int]:
        """Run every saga to completion; returns the batch counters
        [completed, escalated, failed, compensated steps] summed over shapes."""
        for sg in sagas:
            for st in sg.steps:
                if st.step_id not in executors:
                    raise ValueError(f"No executor for step {st.step_id}")
        by_k: dict[int, list] = {}
        for sg in sagas:
            by_k.setdefault(len(sg.steps), []).append(sg)
        total = [0, 0, 0, 0]
        for K, group in by_k.items():
            if K == 0:
                continue
            stats = await self._run_group(orch, group, K, executors, compensator, compensate)
            total = [a + b for a, b in zip(total, stats)]
        self.last_stats = total
        return total

    async def _run_group(self, orch, sagas, K, executors, compensator, compensate) -> list[int]:
        S = len(sagas)
        delay = float(orch.DEFAULT_RETRY_DELAY_SECONDS)
        # outcome tables filled element-wise on the host: flat bytearrays (row s·K + k),
        # turned into tensors once
        fa, fk, cf = bytearray(S * K), bytearray(S * K), bytearray(S * K)
        hu = bytearray(1 if st.undo_api else 0 for sg in sagas for st in sg.steps)
        mr = bytearray(min(int(st.max_retries), 254) for sg in sagas for st in sg.steps)
        results: dict[tuple[int, int], Any] = {}
        errors: dict[tuple[int, int], str] = {}
        comp_results: dict[tuple[int, int], Any] = {}
        comp_errors: dict[tuple[int, int], str] = {}

        loop = asyncio.get_running_loop()

        async def attempts(s: int, k: int):
            st = sagas[s].steps[k]
            n = 1 + int(st.max_retries)
            fn = executors[st.step_id]
            tmo = st.timeout_seconds
            kind, err = 0, None
            for at in range(n):
                try:
                    c = fn()
                    if type(c) is CoroutineType and tmo is not None and tmo > 0:
                        # started inline: a coroutine that finishes without suspending
                        # needs no deadline timer (await_with_timeout semantics otherwise)
                        when = loop.time() + tmo
                        try:
                            y = c.send(None)
                        except StopIteration as e:
                            res = e.value
                        else:
                            res = await resume_with_deadline(c, y, when)
                    else:
                        res = await await_with_timeout(c, tmo)
                except asyncio.TimeoutError:
                    kind = _KIND_TIMEOUT
                    err = f"Step {st.step_id} timed out after {st.timeout_seconds}s (attempt {at + 1}/{n})"
                except Exception as e:  # executor failure
                    kind, err = _KIND_EXC, str(e)
                else:
                    results[(s, k)] = res
                    return at, 0
                if at < n - 1:
                    await asyncio.sleep(delay * (at + 1))
            errors[(s, k)] = err
            return NEVER, kind

        failed_at: dict[int, int] = {}

        async def forward(s: int) -> None:  # the saga's steps in order, until one fails
            for k in range(K):
                nf, kind = await attempts(s, k)
                fa[s * K + k], fk[s * K + k] = nf, kind
                if nf == NEVER:
                    failed_at[s] = k
                    return

        await asyncio.gather(*(forward(s) for s in range(S)))  # sagas run concurrently
        if compensate and failed_at:
            if compensator is None:
                raise ValueError("compensate=True needs a compensator")

            async def comp(s: int, k: int) -> int:
                st = sagas[s].steps[k]
                try:
                    res = await await_with_timeout(compensator(st), st.timeout_seconds)
                except asyncio.TimeoutError:
                    comp_errors[(s, k)] = f"Compensation timed out after {st.timeout_seconds}s"
                    return _KIND_TIMEOUT
                except Exception as e:
                    comp_errors[(s, k)] = f"Compensation failed: {e}"
                    return _KIND_EXC
                comp_results[(s, k)] = res
                return 0

            async def backward(s: int, f: int) -> None:  # committed steps in reverse order
                for k in range(f - 1, -1, -1):
                    if hu[s * K + k]:
                        cf[s * K + k] = await comp(s, k)

            await asyncio.gather(*(backward(s, f) for s, f in failed_at.items()))
        # device FSM: one replay of the captured step loop over the gathered outcomes
        eng = self.engine(S, K, compensate)
        tab = lambda b: torch.frombuffer(b, dtype=u8).view(S, K)  # noqa: E731
        handle = eng.load_outcomes(SagaOutcomes(tab(fa), tab(fk), tab(cf), tab(hu), tab(mr)))
        stats = eng.run_step_loop(handle, now_us=_clock.now_us(), graph=True)
        self._write_back(eng, sagas, results, errors, comp_results, comp_errors)
        return [int(x) for x in stats.cpu().tolist()]

    @staticmethod
    def _write_back(eng, sagas, results, errors, comp_results, comp_errors) -> None:
        from hypervisor.saga.state_machine import SagaState, StepState

        cols = torch.stack([eng.step_state.to(torch.int64), eng.retry_count.to(torch.int64),
                            eng.step_error.to(torch.int64), eng.started_us, eng.completed_us]).cpu().tolist()
        sg_cols = torch.stack([eng.saga_state.to(torch.int64), eng.saga_completed_us,
                               eng.comp_failed.to(torch.int64)]).cpu().tolist()
        # Per-batch lookup tables: enum members by code, and one datetime per distinct
        # device timestamp (the step loop stamps from one time base, so few distinct
        # values) — this loop touches every step of the batch.
        step_enum = [StepState(n) for n in STEP_NAMES]
        saga_enum = [SagaState(n) for n in SAGA_NAMES]
        stamps: dict[int, Any] = {0: None}

        def ts(us: int):
            d = stamps.get(us)
            if d is None and us:
                d = stamps[us] = _clock.from_us(us)
            return d

        st_state, st_retry, st_err, st_start, st_done = cols
        for s, sg in enumerate(sagas):
            row_state, row_retry, row_err = st_state[s], st_retry[s], st_err[s]
            row_start, row_done = st_start[s], st_done[s]
            for k, st in enumerate(sg.steps):
                st.state = step_enum[row_state[k]]
                st.retry_count = row_retry[k]
                st.started_at, st.completed_at = ts(row_start[k]), ts(row_done[k])
                code = row_err[k]
                if code == ERR_NONE:
                    st.error = None
                elif code in (ERR_EXEC, ERR_TIMEOUT):
                    st.error = errors.get((s, k))
                elif code == ERR_NO_UNDO:
                    st.error = "No Undo_API available"
                elif code in (ERR_COMP, ERR_COMP_TIMEOUT):
                    st.error = comp_errors.get((s, k))
                r = results.get((s, k), results)  # the dict itself marks "absent"
                if r is not results:
                    st.execute_result = r
                if (s, k) in comp_results:
                    st.compensation_result = comp_results[(s, k)]
            sg.state = saga_enum[sg_cols[0][s]]
            sg.completed_at = ts(sg_cols[1][s])
            if sg.state is SagaState.ESCALATED:
                sg.error = f"{sg_cols[2][s]} step(s) failed compensation — Joint Liability slashing triggered"
_RUNNERS: dict[str, SagaBatchRunner] = {}


def runner_for(device) -> SagaBatchRunner:
    key = str(device)
    r = _RUNNERS.get(key)
    if r is None:
        r = _RUNNERS[key] = SagaBatchRunner(device)
    return r


async def execute_fanout_groups(orch, groups, executors, timeout_seconds: int, device) -> list:
    """Branches of every group run concurrently on the host; one K15 launch
    decides every group's policy and which succeeded branches to compensate."""
    from agent_hypervisor_amd.ops import saga as SG
    from hypervisor.saga.fan_out import POLICY_CODE

    async def one(g):
        # the per-branch body of FanOutOrchestrator.execute, without the policy step
        await orch.run_branches(g, executors, timeout_seconds)

    await asyncio.gather(*(one(g) for g in groups))
    offs = [0]
    succ = []
    for g in groups:
        succ.extend(1 if b.succeeded else 0 for b in g.branches)
        offs.append(len(succ))
    dev = torch.device(device)
    i32 = torch.int32
    packed = torch.tensor(offs + [POLICY_CODE[g.policy] for g in groups] + succ, dtype=torch.int64).to(dev)
    G = len(groups)
    sat, _, comp = SG.fanout_policy(packed[: G + 1].to(i32), packed[G + 1: 2 * G + 1].to(u8),
                                    packed[2 * G + 1:].to(u8))
    host = torch.cat([sat.to(torch.int64), comp.to(torch.int64)]).cpu().tolist()
    for j, g in enumerate(groups):
        g.policy_satisfied = bool(host[j])
        g.resolved = True
        flags = host[G + offs[j]: G + offs[j + 1]]
        g.compensation_needed = [b.step.step_id for b, f in zip(g.branches, flags) if f and b.step]
    return list(groups)
