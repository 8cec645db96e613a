"""Lifecycle speculation on the device store: joins, activations and step
transitions whose outcome this process already knows (it is the only writer of the
row) are posted without waiting; the device's answers are verified at the store's
next interaction (``GovernanceStore.post_checked`` / ``verify_deferred``)."""

from __future__ import annotations

import asyncio

import pytest

from agent_hypervisor_amd.models.store import StoreError
from hypervisor import Hypervisor, SessionConfig
from hypervisor.models import SessionState


def _run(coro):
    return asyncio.run(coro)


DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.mark.parametrize("dev", DEVICES)
def test_known_outcomes_are_posted_without_waiting(dev):
    async def go():
        hv = Hypervisor(device=dev)
        st = hv._store
        st.verify_deferred(block=True)
        m = await hv.create_session(SessionConfig(max_participants=2), "did:admin")
        sid = m.sso.session_id
        ring = await hv.join_session(sid, "did:a", sigma_raw=0.8)
        assert len(st._deferred) >= 1  # the join was speculated
        await hv.activate_session(sid)
        g = m.saga.create_saga(sid)
        s1 = m.saga.add_step(g.saga_id, "a", "did:a", "/x")
        assert await m.saga.execute_step(g.saga_id, s1.step_id, executor=lambda: asyncio.sleep(0, "ok")) == "ok"
        st.verify_deferred(block=True)  # every speculation agreed with the device
        assert m.sso.state == SessionState.ACTIVE and s1.state.value == "committed"
        # outcomes that are refusals take the awaited path: the device's own error
        await hv.join_session(sid, "did:b", sigma_raw=0.9)
        with pytest.raises(Exception, match="capacity"):
            await hv.join_session(sid, "did:c", sigma_raw=0.9)
        with pytest.raises(Exception, match="already in session"):
            await hv.join_session(sid, "did:a", sigma_raw=0.9)
        return int(ring)

    assert _run(go()) == 2


@pytest.mark.parametrize("dev", DEVICES)
def test_a_wrong_prediction_surfaces_at_the_next_store_call(dev):
    async def go():
        hv = Hypervisor(device=dev)
        st = hv._store
        m = await hv.create_session(SessionConfig(max_participants=1), "did:admin")
        sid = m.sso.session_id
        await hv.join_session(sid, "did:a", sigma_raw=0.8)
        m.sso._m_cfg = (5, 0.0)  # corrupt the mirror: the host now predicts admission, the device refuses
        await hv.join_session(sid, "did:b", sigma_raw=0.8)
        with pytest.raises(StoreError, match="diverged"):
            st.verify_deferred(block=True)

    _run(go())


def test_speculation_off_gives_the_same_results(monkeypatch):
    from hypervisor import _device

    async def pipeline():
        hv = Hypervisor(device="cpu")
        m = await hv.create_session(SessionConfig(), "did:admin")
        sid = m.sso.session_id
        r = [int(await hv.join_session(sid, d, sigma_raw=s)) for d, s in (("did:a", 0.8), ("did:b", 0.96), ("did:c", 0.3))]
        await hv.activate_session(sid)
        g = m.saga.create_saga(sid)
        st_ = m.saga.add_step(g.saga_id, "a", "did:a", "/x")
        await m.saga.execute_step(g.saga_id, st_.step_id, executor=lambda: asyncio.sleep(0))
        return r, [p.agent_did for p in m.sso.participants], st_.state.value, m.sso.state.value

    on = _run(pipeline())
    monkeypatch.setattr(_device, "_SPEC_LIFECYCLE", False)
    off = _run(pipeline())
    assert on == off


@pytest.mark.parametrize("dev", DEVICES)
def test_refused_create_never_lets_a_speculated_join_touch_the_live_row(dev):
    """An allocator bug that hands out a live row: the create is refused, and the join
    posted before its result carries the creation stamp, so the device refuses it too —
    the live session's participants are untouched; the divergence surfaces as StoreError."""
    from hypervisor import _device

    async def go():
        hv = Hypervisor(device=dev)
        st = hv._store
        a = await hv.create_session(SessionConfig(), "did:admin")
        await hv.join_session(a.sso.session_id, "did:a", sigma_raw=0.8)
        st.verify_deferred(block=True)
        b = _device.DeviceSession(st, SessionConfig(), "did:admin", session_id="session:intruder", slot=a.sso.slot)
        b._join_speculated(b._join_args("did:x", 0.9, 0.9, 1, 0), 0.9, True)  # predicted admissible
        with pytest.raises(StoreError):
            st.verify_deferred(block=True)
        st.verify_deferred(block=True)  # the remaining checks drained
        b._store = None  # b never owned the row: its finaliser must not release it
        return [p.agent_did for p in a.sso.participants]

    assert _run(go()) == ["did:a"]
