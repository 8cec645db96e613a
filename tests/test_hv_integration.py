"""End-to-end scenarios through the :class:`Hypervisor` facade (reference
core.py and the scenario families of its integration suite: lifecycle, ring
enforcement, vouching + slashing, sagas, audit trail, GC, rogue agents,
manifest onboarding, drift demotion, Nexus cascades — SURVEY §4)."""

from __future__ import annotations

from types import SimpleNamespace

import pytest

import hypervisor as H
from hypervisor import config
from hypervisor.audit.delta import VFSChange
from hypervisor.integrations.cmvk_adapter import CMVKAdapter
from hypervisor.integrations.iatp_adapter import IATPAdapter
from hypervisor.integrations.nexus_adapter import NexusAdapter
from hypervisor.models import ActionDescriptor, ConsistencyMode, ExecutionRing, ReversibilityLevel, SessionConfig
from hypervisor.observability.event_bus import EventType, HypervisorEventBus
from hypervisor.session import SessionParticipantError

pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


def _cfg(**kw) -> SessionConfig:
    return SessionConfig(**kw)


async def _ok():
    return "ok"


class TestPublicSurface:
    def test_exports(self):
        assert H.__version__ == "2.0.0"
        for name in ("Hypervisor", "SessionConfig", "ExecutionRing", "VouchingEngine", "SlashingEngine",
                     "SagaOrchestrator", "DeltaEngine", "HypervisorEventBus", "RingEnforcer", "KillSwitch"):
            assert hasattr(H, name), name
        assert len(H.__all__) >= 58


class TestFullLifecycle:
    async def test_create_join_activate_audit_terminate(self):
        bus = HypervisorEventBus()
        hv = H.Hypervisor(event_bus=bus)
        m = await hv.create_session(_cfg(), "did:admin")
        sid = m.sso.session_id
        assert await hv.join_session(sid, "did:hi", sigma_raw=0.8) == ExecutionRing.RING_2_STANDARD
        assert await hv.join_session(sid, "did:lo", sigma_raw=0.3) == ExecutionRing.RING_3_SANDBOX
        await hv.activate_session(sid)
        for k in range(3):
            m.delta_engine.capture("did:hi", [VFSChange(f"/f{k}", "add", f"h{k}")])
        root = await hv.terminate_session(sid)
        assert root == m.delta_engine.compute_merkle_root()
        assert hv.commitment.verify(sid, root)
        assert m.sso.state.value == "archived" and hv.active_sessions == [] and hv.gc.is_purged(sid)
        types = [e.event_type for e in bus.query(session_id=sid)]
        assert types[0] == EventType.SESSION_CREATED and types[-1] == EventType.SESSION_ARCHIVED
        assert EventType.AUDIT_COMMITTED in types and types.count(EventType.RING_ASSIGNED) == 2

    async def test_audit_disabled_returns_no_root(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(enable_audit=False), "c")
        await hv.join_session(m.sso.session_id, "a", sigma_raw=0.7)
        m.delta_engine.capture("a", [])
        assert await hv.terminate_session(m.sso.session_id) is None
        assert hv.commitment.commitment_count == 0

    async def test_unknown_session(self):
        hv = H.Hypervisor()
        with pytest.raises(ValueError, match="not found"):
            await hv.join_session("session:nope", "a")
        with pytest.raises(ValueError):
            await hv.terminate_session("session:nope")
        assert hv.get_session("session:nope") is None

    async def test_capacity_enforced_through_facade(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(max_participants=1), "c")
        await hv.join_session(m.sso.session_id, "a")
        with pytest.raises(SessionParticipantError):
            await hv.join_session(m.sso.session_id, "b")

    async def test_gc_frees_vfs_on_terminate(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(), "c")
        sid = m.sso.session_id
        await hv.join_session(sid, "a", sigma_raw=0.7)
        await hv.activate_session(sid)
        m.sso.vfs.write("/big", "x" * 1000, "a")
        await hv.terminate_session(sid)
        assert m.sso.vfs.file_count == 0 and hv.gc.history[-1].purged_vfs_files == 1


class TestRingEnforcementIntegration:
    async def test_irreversible_manifest_forces_strong_consistency(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(), "c")
        acts = [ActionDescriptor("drop", "drop", "/drop", reversibility=ReversibilityLevel.NONE)]
        await hv.join_session(m.sso.session_id, "a", actions=acts, sigma_raw=0.9)
        assert m.sso.consistency_mode == ConsistencyMode.STRONG
        assert m.reversibility.non_reversible_actions == ["drop"]

    async def test_untrustworthy_history_sandboxes(self):
        from datetime import datetime, timezone

        from hypervisor.verification.history import TransactionRecord

        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(), "c")
        t = datetime(2026, 1, 1, tzinfo=timezone.utc)
        hist = [TransactionRecord(f"s{k}", "dup-hash-0000000000", t) for k in range(5)]
        ring = await hv.join_session(m.sso.session_id, "a", sigma_raw=0.9, declared_history=hist)
        assert ring == ExecutionRing.RING_3_SANDBOX

    def test_enforcer_matches_join_ring(self):
        hv = H.Hypervisor()
        act = ActionDescriptor("w", "w", "/w", undo_api="/u", reversibility=ReversibilityLevel.FULL)
        assert hv.ring_enforcer.check(ExecutionRing.RING_2_STANDARD, act, 0.8).allowed
        assert not hv.ring_enforcer.check(ExecutionRing.RING_3_SANDBOX, act, 0.8).allowed


class TestVouchingSlashingIntegration:
    async def test_bonds_released_on_terminate(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(), "c")
        sid = m.sso.session_id
        await hv.join_session(sid, "hi", sigma_raw=0.9)
        await hv.join_session(sid, "lo", sigma_raw=0.4)
        v = hv.vouching.vouch("hi", "lo", sid, 0.9)
        assert hv.vouching.compute_sigma_eff("lo", sid, 0.4, 0.5) == pytest.approx(0.4 + 0.5 * 0.18)
        await hv.terminate_session(sid)
        assert not v.is_active

    async def test_drift_slashes_vouchers_and_demotes(self):
        class Drifty:
            def verify_embeddings(self, **kw):
                return SimpleNamespace(drift_score=0.9, explanation="off-goal")

        slashed = []
        nexus = NexusAdapter(scorer=SimpleNamespace(
            slash_reputation=lambda **kw: slashed.append(kw), record_task_outcome=lambda *a: None,
            calculate_trust_score=lambda **kw: SimpleNamespace(total_score=500)))
        bus = HypervisorEventBus()
        hv = H.Hypervisor(cmvk=CMVKAdapter(Drifty()), nexus=nexus, event_bus=bus, demote_on_slash=True)
        m = await hv.create_session(_cfg(), "c")
        sid = m.sso.session_id
        await hv.join_session(sid, "voucher", sigma_raw=0.7)
        await hv.join_session(sid, "rogue", sigma_raw=0.7)
        hv.vouching.vouch("voucher", "rogue", sid, 0.7)
        res = await hv.verify_behavior(sid, "rogue", [1.0], [0.0])
        assert res.should_slash and hv.slashing.history[0].vouchee_did == "rogue"
        assert m.sso.get_participant("voucher").sigma_eff == pytest.approx(0.05)
        assert m.sso.get_participant("voucher").ring == ExecutionRing.RING_3_SANDBOX
        assert slashed and slashed[0]["severity"] == "critical"
        assert {EventType.BEHAVIOR_DRIFT, EventType.SLASH_EXECUTED} <= {e.event_type for e in bus.all_events}

    async def test_verify_behavior_without_cmvk(self):
        hv = H.Hypervisor()
        assert await hv.verify_behavior("s", "a", [1], [1]) is None


class TestManifestOnboarding:
    async def test_iatp_manifest_drives_sigma_and_actions(self):
        hv = H.Hypervisor(iatp=IATPAdapter())
        m = await hv.create_session(_cfg(), "c")
        manifest = {"agent_id": "did:m", "trust_level": "trusted", "trust_score": 8,
                    "actions": [{"action_id": "edit", "reversibility": "partial", "undo_api": "/u"}]}
        ring = await hv.join_session(m.sso.session_id, "did:m", manifest=manifest)
        assert ring == ExecutionRing.RING_2_STANDARD
        assert m.sso.get_participant("did:m").sigma_raw == 0.8
        assert m.reversibility.get("edit").reversibility == ReversibilityLevel.PARTIAL

    async def test_nexus_resolves_missing_sigma(self):
        nexus = NexusAdapter(scorer=SimpleNamespace(
            calculate_trust_score=lambda **kw: SimpleNamespace(total_score=650)))
        hv = H.Hypervisor(nexus=nexus)
        m = await hv.create_session(_cfg(), "c")
        assert await hv.join_session(m.sso.session_id, "a") == ExecutionRing.RING_2_STANDARD
        assert m.sso.get_participant("a").sigma_eff == 0.65

    async def test_nexus_caps_declared_sigma_with_history(self):
        nexus = NexusAdapter(scorer=SimpleNamespace(
            calculate_trust_score=lambda **kw: SimpleNamespace(total_score=300)))
        hv = H.Hypervisor(nexus=nexus)
        m = await hv.create_session(_cfg(), "c")
        ring = await hv.join_session(m.sso.session_id, "a", sigma_raw=0.9, agent_history=["x"])
        assert ring == ExecutionRing.RING_3_SANDBOX and m.sso.get_participant("a").sigma_eff == 0.3


class TestSagaIntegration:
    async def test_saga_with_compensation_in_session(self):
        hv = H.Hypervisor()
        m = await hv.create_session(_cfg(), "c")
        sid = m.sso.session_id
        g = m.saga.create_saga(sid)
        st = [m.saga.add_step(g.saga_id, f"a{k}", "did:x", "/x", undo_api="/u") for k in range(3)]
        for s in st[:2]:
            await m.saga.execute_step(g.saga_id, s.step_id, _ok)

        async def undo(step):
            return "undone"

        assert await m.saga.compensate(g.saga_id, undo) == []
        assert hv.find_saga(g.saga_id) == (m, g) and hv.find_saga("saga:none") == (None, None)
        assert [s.state.value for s in st] == ["compensated", "compensated", "pending"]


class TestGovernancePipeline:
    async def test_reference_pipeline_shape(self):
        """The bench's scalar pipeline: create → join → activate → saga step →
        3 deltas → terminate (BASELINE full_governance_pipeline)."""
        hv = H.Hypervisor()
        for _ in range(20):
            m = await hv.create_session(_cfg(), "did:admin")
            sid = m.sso.session_id
            await hv.join_session(sid, "did:agent", sigma_raw=0.8)
            await hv.activate_session(sid)
            g = m.saga.create_saga(sid)
            s = m.saga.add_step(g.saga_id, "act", "did:agent", "/x", undo_api="/u")
            await m.saga.execute_step(g.saga_id, s.step_id, _ok)
            for k in range(3):
                m.delta_engine.capture("did:agent", [VFSChange(f"/f{k}", "add", f"h{k}")])
            assert m.delta_engine.verify_chain()
            assert await hv.terminate_session(sid) is not None
        assert hv.commitment.commitment_count == 20 and len(hv.sessions) == 20

    def test_parity_mode_env_switch(self, monkeypatch):
        monkeypatch.setenv("AHV_PARITY_MODE", "1")
        monkeypatch.setenv("AHV_SESSION_CAPACITY", "4096")
        cap = config.RUNTIME.session_capacity
        try:
            config.reload()
            assert config.parity_mode() and config.RUNTIME.session_capacity == 4096
        finally:
            config.RUNTIME.session_capacity = cap
