"""await_with_timeout (hypervisor/saga/_timeout.py): the inline deadline used on
every saga step (reference saga/orchestrator.py:85-88 uses asyncio.wait_for).
Checked against asyncio.wait_for's observable behaviour: results, exceptions,
timeouts, outer cancellation, and the lazily armed timer of the coroutine path."""

import asyncio
import time

import pytest

from hypervisor.saga._timeout import await_with_timeout


def run(coro):
    return asyncio.run(coro)


def test_synchronous_coroutine_returns_without_a_timer():
    async def quick():
        return 7

    async def main():
        loop = asyncio.get_running_loop()
        before = len(loop._scheduled)
        v = await await_with_timeout(quick(), 5)
        return v, len(loop._scheduled) - before

    assert run(main()) == (7, 0)


def test_suspending_coroutine_result_and_exception():
    async def slow_ok():
        await asyncio.sleep(0)
        await asyncio.sleep(0.001)
        return "done"

    async def slow_fail():
        await asyncio.sleep(0)
        raise ValueError("boom")

    async def sync_fail():
        raise KeyError("k")

    assert run(await_with_timeout(slow_ok(), 5)) == "done"
    with pytest.raises(ValueError, match="boom"):
        run(await_with_timeout(slow_fail(), 5))
    with pytest.raises(KeyError):
        run(await_with_timeout(sync_fail(), 5))


def test_timeout_raises_timeout_error_and_cancels_the_coroutine():
    seen = []

    async def hang():
        try:
            await asyncio.sleep(10)
        except asyncio.CancelledError:
            seen.append("cancelled")
            raise

    t0 = time.perf_counter()
    with pytest.raises(asyncio.TimeoutError):
        run(await_with_timeout(hang(), 0.02))
    assert time.perf_counter() - t0 < 2 and seen == ["cancelled"]


def test_deadline_counts_from_the_await_not_the_first_suspension():
    async def busy_then_sleep():
        t = time.perf_counter()
        while time.perf_counter() - t < 0.05:  # synchronous work past the deadline
            pass
        await asyncio.sleep(0.2)
        return "late"

    with pytest.raises(asyncio.TimeoutError):
        run(await_with_timeout(busy_then_sleep(), 0.03))


def test_outer_cancellation_is_not_a_timeout():
    async def main():
        async def hang():
            await asyncio.sleep(10)

        async def waiter():
            return await await_with_timeout(hang(), 5)

        t = asyncio.ensure_future(waiter())
        await asyncio.sleep(0.01)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        return True

    assert run(main())


def test_futures_and_non_awaitables():
    async def main():
        loop = asyncio.get_running_loop()
        f = loop.create_future()
        loop.call_later(0.005, f.set_result, 3)
        return await await_with_timeout(f, 1), await await_with_timeout(asyncio.sleep(0, "x"), None)

    assert run(main()) == (3, "x")
    with pytest.raises(TypeError, match="awaitable is required"):
        run(await_with_timeout(42, 1))
