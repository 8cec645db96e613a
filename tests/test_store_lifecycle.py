"""Row lifecycle of the device state store: no live row is ever overwritten.

Rows (sessions, sagas, steps, vouch edges, delta rows + their payload-arena
records) are owned by the API objects that refer to them and reclaimed only after
the last reference is gone; creates refuse a row that is not free; full tables
grow (doubling) up to their ceiling and then refuse.  Reference semantics kept:
every session and delta lives as long as the process holds it
(``src/hypervisor/core.py:94-104``, ``audit/delta.py:85-115``).

Each check runs on the CPU twin here and on the gfx950 worker under ``-m gpu``
(``tests/test_gpu_store.py`` style: same command processor, private small-cap store).
"""

from __future__ import annotations

import asyncio
import gc

import pytest

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.models import store as _st
from agent_hypervisor_amd.models.store import GovernanceStore, StoreError
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import DeltaEngine, VFSChange
from hypervisor.models import SessionState


def _store(device: str, **caps) -> GovernanceStore:
    """A small-cap store whose tables may grow."""
    base = {"S": 4, "D": 64, "E": 4, "V": 4, "G": 4, "T": 4, "B": 1 << 14}
    base.update(caps)
    return GovernanceStore(device, caps=base)


def _fixed_store(device: str, **caps) -> GovernanceStore:
    """A store whose tables may not grow: reuse must come from reclaimed rows."""
    base = {"S": 4, "D": 64, "E": 4, "V": 4, "G": 4, "T": 4, "B": 1 << 14}
    base.update(caps)
    return GovernanceStore(device, caps=base, max_caps={k: base[k] for k in ("S", "D", "E", "V", "G", "T", "B")})


def _chg(i):
    return [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")]


async def _live_session(hv):
    a = await hv.create_session(SessionConfig(enable_audit=True), "did:mesh:admin")
    sid = a.sso.session_id
    await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    await hv.activate_session(sid)
    a.delta_engine.capture("did:mesh:a", _chg(0))
    return a


def check_live_session_survives_churn(device: str) -> None:
    """An ACTIVE session keeps its participants, state and chain through 100
    create/terminate cycles of other sessions — both when the others stay
    referenced (the table grows) and when they are dropped (rows are reused)."""

    async def run():
        st = _store(device)
        hv = Hypervisor(store=st)
        a = await _live_session(hv)
        slot = a.sso.slot
        for i in range(100):
            m = await hv.create_session(SessionConfig(), "did:mesh:admin")
            await hv.join_session(m.sso.session_id, f"did:mesh:x{i}", sigma_raw=0.7)
            await hv.activate_session(m.sso.session_id)
            m.delta_engine.capture(f"did:mesh:x{i}", _chg(i))
            await hv.terminate_session(m.sso.session_id)
        assert st.caps["S"] >= 101 and st.grows["S"] >= 5
        assert a.sso.slot == slot and a.sso.state is SessionState.ACTIVE
        assert [p.agent_did for p in a.sso.participants] == ["did:mesh:a"]
        a.delta_engine.capture("did:mesh:a", _chg(1))
        want = C.merkle_root([d.delta_hash for d in a.delta_engine.deltas])
        assert await hv.terminate_session(a.sso.session_id) == want

        # dropped sessions: their rows come back, the table never grows
        st2 = _fixed_store(device)
        hv2 = Hypervisor(store=st2)
        b = await _live_session(hv2)
        for i in range(100):
            tmp = Hypervisor(store=st2)
            m = await tmp.create_session(SessionConfig(), "did:mesh:admin")
            await tmp.join_session(m.sso.session_id, "did:mesh:y", sigma_raw=0.7)
            await tmp.activate_session(m.sso.session_id)
            m.delta_engine.capture("did:mesh:y", _chg(i))
            saga = m.saga.create_saga(m.sso.session_id)
            step = m.saga.add_step(saga.saga_id, "act", "did:mesh:y", "/api")
            await m.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
            await tmp.terminate_session(m.sso.session_id)
            del tmp, m, saga, step
            if i % 7 == 0:
                gc.collect()
        assert st2.caps["S"] == 4 and st2.grows == {k: 0 for k in st2.grows}
        assert b.sso.state is SessionState.ACTIVE and b.sso.participant_count == 1
        want = C.merkle_root([d.delta_hash for d in b.delta_engine.deltas])
        assert b.delta_engine.compute_merkle_root() == want
        st.close()
        st2.close()

    asyncio.run(run())


def check_full_fixed_table_refuses(device: str) -> None:
    async def run():
        st = _fixed_store(device)
        hv = Hypervisor(store=st)
        keep = [await hv.create_session(SessionConfig(), "did:a") for _ in range(4)]
        with pytest.raises(StoreError, match="full"):
            await hv.create_session(SessionConfig(), "did:a")
        assert all(m.sso.state is SessionState.HANDSHAKING for m in keep)
        # the device itself refuses a create on a live row (allocator bug guard)
        r = st.call(_st.OP_SESS_CREATE, [keep[0].sso.slot, 0, 0, 0, 10, 0, 1, 0, 0, 0], 2)
        assert r[0] == _st.ST_BAD_STATE and r[1] == 1  # HANDSHAKING
        assert keep[0].sso.state is SessionState.HANDSHAKING
        st.close()

    asyncio.run(run())


def check_long_capture_run(device: str, total: int) -> None:
    """``total`` captures through small delta/arena tables: an early session that
    stays live keeps a Merkle root equal to the host DeltaEngine's over the same
    fields, while dropped chains' rows and records are reused."""

    async def run():
        st = GovernanceStore(device, caps={"S": 64, "D": 4096, "B": 1 << 20, "G": 4, "T": 4, "E": 4, "V": 4})
        hv = Hypervisor(store=st)
        a = await _live_session(hv)
        n_early = 40
        for i in range(1, n_early):
            a.delta_engine.capture("did:mesh:a", _chg(i))
        done = n_early
        k = 0
        while done < total:
            tmp = Hypervisor(store=st)
            m = await tmp.create_session(SessionConfig(), "did:mesh:admin")
            await tmp.join_session(m.sso.session_id, "did:mesh:z", sigma_raw=0.9)
            await tmp.activate_session(m.sso.session_id)
            for i in range(50):
                m.delta_engine.capture("did:mesh:z", _chg(k * 50 + i))
            done += 50
            k += 1
            del tmp, m
            if k % 50 == 0:
                gc.collect()
        host = DeltaEngine(a.sso.session_id)
        for d in a.delta_engine.deltas:
            h = host.capture(d.agent_did, d.changes, delta_id=d.delta_id)
            h.timestamp = d.timestamp
        # recompute the host chain with the device's timestamps
        prev = None
        for h in host.deltas:
            h.parent_hash = prev
            h.compute_hash()
            prev = h.delta_hash
        assert [h.delta_hash for h in host.deltas] == [d.delta_hash for d in a.delta_engine.deltas]
        assert a.delta_engine.compute_merkle_root() == host.compute_merkle_root()
        assert a.delta_engine.verify_chain()
        assert st.caps["D"] <= 8192, "dropped chains' rows must be reused, not grown into"
        st.close()

    asyncio.run(run())


def check_vouch_edges_reused(device: str) -> None:
    async def run():
        st = _fixed_store(device)
        hv = Hypervisor(store=st)
        s = await hv.create_session(SessionConfig(), "did:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:a", sigma_raw=0.9)
        r1 = hv.vouching.vouch("did:a", "did:b", sid, 0.9)
        r2 = hv.vouching.vouch("did:c", "did:b", sid, 0.8)
        edges = {r1.edge, r2.edge}
        await hv.activate_session(sid)
        await hv.terminate_session(sid)
        # records keep their final state after the rows were freed
        assert not r1.is_active and r1.released_at is not None and r1.edge == -1
        assert [x.vouch_id for x in hv.vouching.records(sid)] == [r1.vouch_id, r2.vouch_id]
        # new bonds (another session) reuse the retired rows: only 4 exist
        got = set()
        for i in range(4):
            r = hv.vouching.vouch(f"did:v{i}", f"did:w{i}", "s-other", 0.9)
            got.add(r.edge)
        assert edges <= got and st.caps["E"] == 4
        assert hv.vouching.compute_sigma_eff("did:w0", "s-other", 0.3, 0.65) == pytest.approx(0.3 + 0.65 * 0.18)
        assert hv.vouching.get_vouchers_for("did:b", sid) == []
        st.close()

    asyncio.run(run())


def check_batched_reads_and_paging(device: str) -> None:
    async def run():
        st = _store(device, S=64, E=64, V=8)
        hv = Hypervisor(store=st)
        ms = []
        for i in range(20):
            m = await hv.create_session(SessionConfig(max_participants=5), "did:admin")
            for j in range(i % 4):
                await hv.join_session(m.sso.session_id, f"did:p{i}-{j}", sigma_raw=0.5 + 0.1 * j)
            ms.append(m)
        before = st.info()["posted"]
        hdr, parts = st.read_sessions([m.sso.slot for m in ms], parts=True)
        assert st.info()["posted"] - before == 1
        for i, m in enumerate(ms):
            assert int(hdr[i, 0]) & 0xFF == 1  # HANDSHAKING
            assert int(hdr[i, 1]) & 0xFFFFFFFF == i % 4
            assert [st.did(int(parts[i, k, 0])) for k in range(i % 4)] == [p.agent_did for p in m.sso.participants]
        # vouch listing pages through the bulk buffer
        v = hv.vouching
        for j in range(10):
            v.vouch(f"did:u{j}", "did:t", "s1", 0.9, bond_pct=0.01)
        v.LIST_PAGE = 3
        assert [r.voucher_did for r in v.get_vouchers_for("did:t", "s1")] == [f"did:u{j}" for j in range(10)]
        st.close()

    asyncio.run(run())


# ------------------------------------------------------------------ CPU twin


def test_live_session_survives_churn_cpu_twin():
    check_live_session_survives_churn("cpu")


def test_full_fixed_table_refuses_cpu_twin():
    check_full_fixed_table_refuses("cpu")


def test_long_capture_run_cpu_twin():
    check_long_capture_run("cpu", 300_000)


def test_vouch_edges_reused_cpu_twin():
    check_vouch_edges_reused("cpu")


def test_batched_reads_and_paging_cpu_twin():
    check_batched_reads_and_paging("cpu")


def test_arena_allocator_reuses_freed_records():
    st = GovernanceStore("cpu", caps={"D": 8, "B": 4096}, max_caps={"D": 8, "B": 4096})
    for _ in range(3):
        rows = [st.restore_delta(b"x" * 300) for _ in range(8)]  # 5 granules each: 40 of 64
        assert len({r[0] for r in rows}) == 8 and len({r[1] for r in rows}) == 8
        st.release_many("D", [r[0] for r in rows])
        st.reclaim("D")
    assert st.info()["payload_live"] == 0 and st.grows["B"] == 0
    st.close()


# ------------------------------------------------------------------ gfx950


@pytest.mark.gpu
def test_live_session_survives_churn_gpu():
    check_live_session_survives_churn("cuda")


@pytest.mark.gpu
def test_full_fixed_table_refuses_gpu():
    check_full_fixed_table_refuses("cuda")


@pytest.mark.gpu
def test_long_capture_run_gpu():
    check_long_capture_run("cuda", 300_000)


@pytest.mark.gpu
def test_vouch_edges_reused_gpu():
    check_vouch_edges_reused("cuda")


@pytest.mark.gpu
def test_batched_reads_and_paging_gpu():
    check_batched_reads_and_paging("cuda")
