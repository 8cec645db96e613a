"""Low-overhead awaiting with a deadline.

``asyncio.wait_for`` (Python 3.10) wraps the awaitable in a new Task and costs
several event-loop iterations; on the saga hot path that was ~28 % of the
reference pipeline.  :func:`await_with_timeout` instead awaits the
awaitable inline and arms a loop timer that cancels the *current* task when the
deadline passes (the technique of Python 3.11's ``asyncio.timeout``), converting
that cancellation into ``asyncio.TimeoutError``.

Behaviour kept from ``wait_for`` where callers can observe it: a non-awaitable
raises the same ``TypeError`` message, ``timeout=None`` waits forever, and
``timeout <= 0`` delegates to ``wait_for`` itself.

A coroutine is driven by hand up to its first suspension before any timer is
armed: one that completes without suspending (a synchronous executor, a cache
hit) costs no loop timer at all.  The deadline is still taken when the await
starts, so a coroutine that first suspends late times out exactly when the eager
timer would have fired.
"""

from __future__ import annotations

import asyncio
from inspect import isawaitable
from types import CoroutineType

_NOT_AWAITABLE = "An asyncio.Future, a coroutine or an awaitable is required"


async def await_with_timeout(aw, timeout):
    if type(aw) is not CoroutineType and not isawaitable(aw):
        raise TypeError(_NOT_AWAITABLE)
    if timeout is None:
        return await aw
    if timeout <= 0:
        return await asyncio.wait_for(aw, timeout)
    loop = asyncio.get_running_loop()
    task = asyncio.current_task(loop)
    if type(aw) is CoroutineType:
        return await _Deadline(aw, loop, loop.time() + timeout, task)
    state = [False]

    def _expire() -> None:
        state[0] = True
        task.cancel()

    handle = loop.call_later(timeout, _expire)
    try:
        return await aw
    except asyncio.CancelledError:
        if state[0]:
            raise asyncio.TimeoutError() from None
        raise
    finally:
        handle.cancel()


def resume_with_deadline(coro, first, when):
    """Awaitable continuing ``coro`` — already started by the caller with
    ``coro.send(None)``, which yielded ``first`` — under a deadline at loop time
    ``when`` (batch runners start coroutines inline and only pay for the timer
    when one actually suspends)."""
    loop = asyncio.get_running_loop()
    return _Deadline(coro, loop, when, asyncio.current_task(loop), first, True)


class _Deadline:
    """Awaitable that delegates to ``coro`` like ``yield from`` and arms the
    cancelling timer (due at ``when``) only once ``coro`` first suspends."""

    __slots__ = ("coro", "loop", "when", "task", "first", "started")

    def __init__(self, coro, loop, when, task, first=None, started=False) -> None:
        self.coro, self.loop, self.when, self.task = coro, loop, when, task
        self.first, self.started = first, started

    def __await__(self):
        coro = self.coro
        if self.started:
            y = self.first
        else:
            try:
                y = coro.send(None)
            except StopIteration as e:  # finished without suspending: no timer needed
                return e.value
        expired = [False]
        task = self.task

        def _expire() -> None:
            expired[0] = True
            task.cancel()

        handle = self.loop.call_at(self.when, _expire)
        try:
            while True:
                try:
                    v = yield y
                except GeneratorExit:
                    coro.close()
                    raise
                except BaseException as exc:  # thrown in by the task (cancellation)
                    try:
                        y = coro.throw(exc)
                    except StopIteration as e:
                        return e.value
                else:
                    try:
                        y = coro.send(v)
                    except StopIteration as e:
                        return e.value
        except asyncio.CancelledError:
            if expired[0]:
                raise asyncio.TimeoutError() from None
            raise
        finally:
            handle.cancel()
