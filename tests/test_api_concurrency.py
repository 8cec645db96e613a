"""Thousands of concurrent reference pipelines through one device store.

Regression: the saga step's posted EXECUTING transition is awaited only after the
executor ran, by which time thousands of other sessions' commands may have been
posted and its result slot recycled ("store result slot recycled").  Posted
results that are read later are kept (``GovernanceStore.post(..., keep=True)``).
"""

from __future__ import annotations

import asyncio
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))

from bench_api import reference_pipeline  # noqa: E402


def _gather(device: str, n: int) -> list:
    async def go():
        return await asyncio.gather(*[reference_pipeline(device) for _ in range(n)])

    return asyncio.run(go())


def test_concurrent_pipelines_cpu_twin():
    roots = _gather("cpu", 3000)
    assert len(roots) == 3000 and len(set(roots)) == 3000 and all(len(r) == 64 for r in roots)


@pytest.mark.gpu
def test_concurrent_pipelines_gfx950():
    roots = _gather("cuda", 5000)
    assert len(roots) == 5000 and len(set(roots)) == 5000 and all(len(r) == 64 for r in roots)


def test_cancelled_step_discards_its_kept_result():
    """A cancelled executor leaves no kept result behind in the store."""
    from hypervisor import Hypervisor, SessionConfig

    async def go():
        hv = Hypervisor(device="cpu")
        m = await hv.create_session(SessionConfig(), "did:admin")
        sid = m.sso.session_id
        await hv.join_session(sid, "did:a", sigma_raw=0.8)
        g = m.saga.create_saga(sid)
        st = m.saga.add_step(g.saga_id, "a", "did:a", "/x")
        st2 = m.saga.add_step(g.saga_id, "b", "did:a", "/y")
        await m.saga.execute_step(g.saga_id, st.step_id, executor=lambda: asyncio.sleep(0))  # state known: speculates
        t = asyncio.ensure_future(m.saga.execute_step(g.saga_id, st2.step_id, executor=lambda: asyncio.sleep(10)))
        await asyncio.sleep(0.01)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        hv._store.verify_deferred(block=True)  # speculated posts verified: only leaks would remain kept
        return hv._store.info()

    info = _run(go())
    assert info.get("kept", 0) == 0, info


def _run(coro):
    return asyncio.run(coro)
