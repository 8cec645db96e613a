"""Real saga executions driven through the device saga FSM (K13/K14) and
fan-out policy (K15).

:meth:`hypervisor.saga.orchestrator.SagaOrchestrator.execute_sagas` and
:meth:`hypervisor.saga.fan_out.FanOutOrchestrator.execute_groups` with a
``device`` land here.  The split of work:

* **device** — the saga state machine (K13/K14 phase kernels of
  :class:`SagaBatchEngine`) decides what runs: after the execute phase of step
  k it reports which sagas committed step k (those, and only those, run step
  k+1); after the decide phase, which committed steps of which sagas are
  compensated, round by round in reverse step order.  Every state, retry count,
  error code, transition timestamp and the batch counters are device state;
* **host** — awaits exactly the executor / compensator coroutines the device
  asked for, all sagas of a round at once: a coroutine that finishes without
  suspending (the common case) is driven inline, the rest run concurrently
  under ``asyncio.gather`` with the reference's deadline, retry and delay
  semantics (saga/orchestrator.py:77-198).  Each step's outcome is reduced to
  the FSM's inputs — failing attempts before success (255 = never), the last
  failure's kind (exception / timeout), the compensation outcome — and uploaded
  as one row per round.

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
_ST_COMMITTED = STEP_NAMES.index("committed")
_UNSET = object()
_SG_RUNNING, _SG_COMPENSATING = SAGA_NAMES.index("running"), SAGA_NAMES.index("compensating")


class _Setter:
    """``obj[name] = v`` as ``setattr`` (the write-back's slow path)."""

    __slots__ = ("obj",)

    def __init__(self, obj) -> None:
        self.obj = obj

    def __setitem__(self, name: str, value) -> None:
        setattr(self.obj, name, value)


class _Resume:
    """Awaitable continuing a coroutine already started with ``send(None)``."""

    __slots__ = ("coro", "first")

    def __init__(self, coro, first) -> None:
        self.coro, self.first = coro, first

    def __await__(self):
        coro, y = self.coro, self.first
        while True:
            try:
                x = yield y
            except BaseException as e:  # noqa: BLE001 - thrown into the coroutine (cancellation)
                try:
                    y = coro.throw(e)
                except StopIteration as stop:
                    return stop.value
            else:
                try:
                    y = coro.send(x)
                except StopIteration as stop:
                    return stop.value


def _resume(coro, first):
    return _Resume(coro, first)


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
        rows = [sg.steps for sg in sagas]
        hu = bytearray(1 if st.undo_api else 0 for row in rows for st in row)
        mr = bytearray(min(int(st.max_retries), 254) for row in rows for st in row)
        # per (saga, step) host payloads, flat at s·K + k (_UNSET = none)
        results: list = [_UNSET] * (S * K)
        errors: list = [None] * (S * K)
        comp_results: list = [_UNSET] * (S * K)
        comp_errors: list = [None] * (S * K)
        loop = asyncio.get_running_loop()

        # device state machine, driven phase by phase: the outcome rows of step k
        # are uploaded just before its execute phase, and after it the device
        # says which sagas run step k+1
        eng = self.engine(S, K, compensate)
        zero = bytearray(S * K)
        tab = lambda b: torch.frombuffer(b, dtype=u8).view(S, K)  # noqa: E731
        handle = eng.load_outcomes(SagaOutcomes(tab(zero), tab(zero), tab(zero), tab(hu), tab(mr)))
        prep = eng._prepared(handle)  # [K, S] rows the phase kernels read
        now = _clock.now_us()
        args = eng._args(handle, now)
        eng.now_dev.fill_(now)
        eng._spread.begin()
        eng._phase(args, 0)

        def upload(name: str, k: int, row: bytearray) -> None:
            prep[name][k].copy_(torch.frombuffer(row, dtype=u8))

        async def attempts(s: int, k: int, fa_row: bytearray, fk_row: bytearray, at0: int = 0,
                           started=None, first=None) -> None:
            """Attempts ``at0``… of step k of saga s with full await semantics
            (suspending executors, deadlines, retry delays).  ``started``: the
            (coroutine, first yield) of attempt ``at0``, already begun inline;
            ``first``: what the executor returned for attempt ``at0`` when that
            was not a coroutine."""
            st = rows[s][k]
            n = 1 + int(st.max_retries)
            fn = executors[st.step_id]
            tmo = st.timeout_seconds
            kind, err = 0, None
            for at in range(at0, n):
                try:
                    if started is not None:
                        c, y = started
                        started = None
                        res = await (resume_with_deadline(c, y, loop.time() + tmo) if tmo is not None and tmo > 0
                                     else _resume(c, y))
                    else:
                        c = fn() if first is None else first
                        first = None
                        if type(c) is CoroutineType and tmo is not None and tmo > 0:
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
                    results[s * K + k] = res
                    fa_row[s] = at
                    return
                if at < n - 1:
                    await asyncio.sleep(delay * (at + 1))
            errors[s * K + k] = err
            fa_row[s], fk_row[s] = NEVER, kind

        def inline(s: int, k: int, fa_row: bytearray, fk_row: bytearray):
            """Run step k of saga s here if its executor never suspends (the
            common case); returns None when done, else the coroutine finishing it."""
            st = rows[s][k]
            n = 1 + int(st.max_retries)
            fn = executors[st.step_id]
            err = None
            for at in range(n):
                try:
                    c = fn()
                    if type(c) is not CoroutineType:  # other awaitables (or none): the full path
                        return attempts(s, k, fa_row, fk_row, at, first=c)
                    try:
                        y = c.send(None)
                    except StopIteration as e:
                        results[s * K + k] = e.value
                        fa_row[s] = at
                        return None
                    return attempts(s, k, fa_row, fk_row, at, (c, y))
                except Exception as e:  # raised before suspending: a failed attempt
                    err = str(e)
                if at < n - 1 and delay > 0:
                    return attempts(s, k, fa_row, fk_row, at + 1)  # the retry waits its delay
            errors[s * K + k] = err
            fa_row[s], fk_row[s] = NEVER, _KIND_EXC
            return None

        runnable = list(range(S))
        for k in range(K):
            fa_row, fk_row = bytearray(S), bytearray(S)
            slow = [c for c in (inline(s, k, fa_row, fk_row) for s in runnable) if c is not None]
            if slow:
                await asyncio.gather(*slow)  # suspending executors: concurrently, across sagas
            upload("fail_attempts", k, fa_row)
            upload("fail_kind", k, fk_row)
            eng._phase(args, 1, k)
            if k + 1 < K:  # the device picks the sagas whose step k committed
                runnable = torch.nonzero((eng._step_state[k] == _ST_COMMITTED)
                                         & (eng.saga_state == _SG_RUNNING)).flatten().tolist()
                if not runnable:
                    break
        eng._phase(args, 2)
        if compensate and bool((eng.saga_state == _SG_COMPENSATING).any()):
            if compensator is None:
                raise ValueError("compensate=True needs a compensator")
            has_undo = prep["has_undo"]

            async def comp(s: int, k: int, cf_row: bytearray, first=None, started=None) -> None:
                st = rows[s][k]
                tmo = st.timeout_seconds
                try:
                    if started is not None:
                        c, y = started
                        res = await (resume_with_deadline(c, y, loop.time() + tmo) if tmo is not None and tmo > 0
                                     else _resume(c, y))
                    else:
                        res = await await_with_timeout(compensator(st) if first is None else first, tmo)
                except asyncio.TimeoutError:
                    comp_errors[s * K + k] = f"Compensation timed out after {st.timeout_seconds}s"
                    cf_row[s] = _KIND_TIMEOUT
                    return
                except Exception as e:
                    comp_errors[s * K + k] = f"Compensation failed: {e}"
                    cf_row[s] = _KIND_EXC
                    return
                comp_results[s * K + k] = res

            def comp_inline(s: int, k: int, cf_row: bytearray):
                """A compensator coroutine that finishes without suspending is driven
                here; otherwise the awaitable finishing it (deadline armed)."""
                st = rows[s][k]
                try:
                    c = compensator(st)
                    if type(c) is not CoroutineType:
                        return comp(s, k, cf_row, c)
                    try:
                        y = c.send(None)
                    except StopIteration as e:
                        comp_results[s * K + k] = e.value
                        return None
                except Exception as e:
                    comp_errors[s * K + k] = f"Compensation failed: {e}"
                    cf_row[s] = _KIND_EXC
                    return None
                return comp(s, k, cf_row, None, (c, y))

            for k in range(K - 1, -1, -1):  # committed steps in reverse order, all sagas at once
                todo = torch.nonzero((eng.saga_state == _SG_COMPENSATING) & (eng._step_state[k] == _ST_COMMITTED)
                                     & (has_undo[k] != 0)).flatten().tolist()
                if todo:
                    cf_row = bytearray(S)
                    slow = [c for c in (comp_inline(s, k, cf_row) for s in todo) if c is not None]
                    if slow:
                        await asyncio.gather(*slow)
                    upload("comp_fail", k, cf_row)
                eng._phase(args, 3, k)  # also fails the committed steps without an Undo_API
        eng._phase(args, 4)
        stats = eng._spread.copy_into(eng.stats)
        self._write_back(eng, sagas, results, errors, comp_results, comp_errors)
        return [int(x) for x in stats.cpu().tolist()]

    @staticmethod
    def _write_back(eng, sagas, results, errors, comp_results, comp_errors) -> None:
        from hypervisor.saga.state_machine import SagaState, SagaStep, StepState

        K = eng.K
        cols = torch.stack([eng.step_state.to(torch.int64), eng.retry_count.to(torch.int64),
                            eng.step_error.to(torch.int64), eng.started_us, eng.completed_us]).cpu().tolist()
        sg_cols = torch.stack([eng.saga_state.to(torch.int64), eng.saga_completed_us,
                               eng.comp_failed.to(torch.int64)]).cpu().tolist()
        # Per-batch lookup tables: enum members by code, and one datetime per distinct
        # device timestamp (the phases stamp from one time base, so few distinct values)
        step_enum = [StepState(n) for n in STEP_NAMES]
        saga_enum = [SagaState(n) for n in SAGA_NAMES]
        st_state, st_retry, st_err, st_start, st_done = cols
        seen = set()
        for rows_ in (st_start, st_done, [sg_cols[1]]):
            for r in rows_:
                seen.update(r)
        stamps = {us: (_clock.from_us(us) if us else None) for us in seen}
        no_undo = "No Undo_API available"
        escalated = SagaState.ESCALATED
        for s, sg in enumerate(sagas):
            row_state, row_retry, row_err = st_state[s], st_retry[s], st_err[s]
            row_start, row_done = st_start[s], st_done[s]
            base = s * K
            for k, st in enumerate(sg.steps):
                code = row_err[k]
                if code == ERR_NONE:
                    err = None
                elif code == ERR_EXEC or code == ERR_TIMEOUT:
                    err = errors[base + k]
                elif code == ERR_NO_UNDO:
                    err = no_undo
                else:  # ERR_COMP, ERR_COMP_TIMEOUT
                    err = comp_errors[base + k]
                # plain SagaSteps take the fields in one dict update; views with
                # properties (device-store steps) through their setters
                d = st.__dict__ if type(st) is SagaStep else _Setter(st)
                d["state"] = step_enum[row_state[k]]
                d["retry_count"] = row_retry[k]
                d["started_at"] = stamps[row_start[k]]
                d["completed_at"] = stamps[row_done[k]]
                d["error"] = err
                r = results[base + k]
                if r is not _UNSET:
                    d["execute_result"] = r
                r = comp_results[base + k]
                if r is not _UNSET:
                    d["compensation_result"] = r
            sg.state = saga_enum[sg_cols[0][s]]
            sg.completed_at = stamps[sg_cols[1][s]]
            if sg.state is escalated:
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
