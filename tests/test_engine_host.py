"""Batched governance pipeline, host twin (CPU): the same per-session body the
gfx950 kernel runs, checked against the scalar API path byte-for-byte."""

from __future__ import annotations

import hashlib

import pytest
import torch  # noqa: F401 - loaded before the native extension

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.models.engine import GovernanceEngine
from hypervisor import _clock
from hypervisor.audit.delta import DeltaEngine, VFSChange
from hypervisor.models import ExecutionRing

NOW = 1767225600123456  # 2026-01-01T00:00:00.123456Z


@pytest.fixture
def engine():
    eng = GovernanceEngine(device="cpu", session_capacity=256, agent_capacity=64, seed=42)
    eng.register_synthetic_agents(32, seed=7)
    return eng


def test_pipeline_status_and_lifecycle(engine):
    b = engine.run_pipeline(40, now_us=NOW)
    assert (b.status() == 0).all()
    t = engine.sessions
    s = b.slots()
    assert (t.sess_state[s] == 4).all()  # archived
    assert (t.part_count[s] == 1).all()
    assert (t.delta_count[s] == 3).all()
    assert (t.step_state[s] == 2).all()  # committed
    assert (t.saga_state[s] == 0).all()  # running (the benchmark never completes the saga)
    assert (t.committed_at_us[s] > 0).all()


def test_rings_follow_sigma(engine):
    b = engine.run_pipeline(32, now_us=NOW)
    s = b.slots()
    sig = engine.sessions.part_sigma_eff[s, 0]
    ring = engine.sessions.part_ring[s, 0]
    for x, r in zip(sig.tolist(), ring.tolist()):
        assert r == ExecutionRing.from_sigma_eff(x).value


def test_pipeline_matches_scalar_delta_engine(engine):
    b = engine.run_pipeline(16, now_us=NOW)
    for i in range(16):
        sid = b.session_id(i)
        agent = engine.interner.str(int(engine.agents.did[int(b.agent_ids[i])]))
        ticks = iter(range(1, 10))
        _clock.set_clock(lambda: _clock.from_us(NOW + next(ticks)))
        de = DeltaEngine(sid)
        for d in range(3):
            de.capture(agent, [VFSChange(path=f"/f{d}", operation="add", content_hash=f"h{d}")])
        _clock.set_clock(None)
        assert [x.delta_hash for x in de.deltas] == [b.delta_hash_hex(i, d) for d in range(3)]
        assert de.compute_merkle_root() == b.merkle_root_hex(i)


def test_materialized_session_verifies(engine):
    b = engine.run_pipeline(8, now_us=NOW)
    for i in range(8):
        m = b.materialize(i)
        assert m.sso.state.value == "archived"
        assert m.delta_engine.verify_chain()
        assert m.delta_engine.compute_merkle_root() == b.merkle_root_hex(i)


def test_ids_are_uuid4_and_unique(engine):
    b1 = engine.run_pipeline(50, now_us=NOW)
    b2 = engine.run_pipeline(50, now_us=NOW)
    ids = {b1.session_id(i) for i in range(50)} | {b2.session_id(i) for i in range(50)}
    assert len(ids) == 100
    sid = b1.session_id(0)
    assert sid.startswith("session:") and sid[8 + 14] == "4" and sid[8 + 19] in "89ab"
    assert b1.saga_id(0).startswith("saga:") and b1.step_id(0).startswith("step:")
    # host mirror of the device id generator
    assert C.uuid_from_counter(engine.seed, b1.id_base, "session:") == sid


@pytest.mark.parametrize("deltas", [0, 1, 2, 5, 8])
def test_variable_delta_counts(deltas):
    eng = GovernanceEngine(device="cpu", session_capacity=32, agent_capacity=8, seed=3)
    eng.register_agents(["did:mesh:a", "did:mesh:é\"\\x"], [0.8, 0.3])
    b = eng.run_pipeline(4, deltas=deltas, now_us=NOW)
    for i in range(4):
        m = b.materialize(i)
        assert m.delta_engine.verify_chain()
        root = m.delta_engine.compute_merkle_root()
        if deltas:
            assert root == b.merkle_root_hex(i)
        else:
            assert root is None and b.merkle_root_hex(i) == "0" * 64


def test_long_and_skewed_field_lengths():
    """Lanes with very different message lengths (ring-skew path on device)."""
    eng = GovernanceEngine(device="cpu", session_capacity=16, agent_capacity=8, seed=5)
    eng.register_agents(["did:x", "did:mesh:" + "y" * 300, "did:" + "ü" * 90], [0.5, 0.7, 0.99])
    b = eng.run_pipeline(6, now_us=NOW, changes=[("/path/{i}" + "z" * 150, "modify", None)])
    for i in range(6):
        m = b.materialize(i)
        assert m.delta_engine.verify_chain()
        assert m.delta_engine.compute_merkle_root() == b.merkle_root_hex(i)


def test_slot_ring_wraps():
    eng = GovernanceEngine(device="cpu", session_capacity=10, agent_capacity=4, seed=9)
    eng.register_synthetic_agents(4)
    eng.run_pipeline(7, now_us=NOW)
    b = eng.run_pipeline(7, now_us=NOW)  # wraps around the 10-row table
    assert b.slots().tolist() == [7, 8, 9, 0, 1, 2, 3]
    for i in range(7):
        assert b.materialize(i).delta_engine.compute_merkle_root() == b.merkle_root_hex(i)


def test_iso_time_base_matches_datetime():
    for us in [0, 1, 999999, 1767225600000000, 1767225600123456, 951782400000001, 4102444799999999]:
        assert C.iso_from_us(us) == _clock.from_us(us).isoformat()


def test_interner_escapes_like_json():
    import json

    from agent_hypervisor_amd.utils.interner import Interner

    it = Interner()
    for s in ["plain", 'q"uote', "back\\slash", "tab\tnl\n", "\x00\x1f\x7f", "é", "😀", "日本"]:
        i = it.intern(s)
        assert it.escaped(i).decode() == json.dumps(s)[1:-1]
        assert it.str(i) == s
        assert it.intern(s) == i


def test_pipeline_gcs_by_timestamp(engine):
    """GC retention counts deltas by timestamp against terminate − retention."""
    b = engine.run_pipeline(24, now_us=NOW)
    s = b.slots()
    assert (engine.sessions.gc_retained[s] == 3).all()
    assert (engine.sessions.bonds_released[s] == 0).all()  # batched sessions post no bonds
    # retention shorter than the session: deltas stamped now+1..now+3, terminate at now+6
    engine.gc_retention_us = 4  # cutoff now+2 → delta 1 expires
    b2 = engine.run_pipeline(8, now_us=NOW)
    assert (engine.sessions.gc_retained[b2.slots()] == 2).all()


def test_engine_rows_are_store_rows(engine):
    """One representation of session state: the engine's rows are its store's rows —
    the records in the payload arena are the hashed bytes, delta rows link the chain."""
    b = engine.run_pipeline(5, now_us=NOW)
    st = engine.store
    for i in range(5):
        recs = [b.record(i, d) for d in range(3)]
        assert [hashlib.sha256(r).hexdigest() for r in recs] == [b.delta_hash_hex(i, d) for d in range(3)]
        s = int(b.slots()[i])
        assert int(st.tables["s_dlast"][s]) == s * engine.dmax + 2
        assert int(st.tables["d_prev"][s * engine.dmax + 2]) == s * engine.dmax + 1
