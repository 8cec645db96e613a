"""Audit (delta chain, Merkle root, commitments, GC), observability (event
bus, causal trace ids), security (rate limiter, kill switch) and the
integration adapters (Nexus, CMVK, IATP) — reference audit/*.py,
observability/*.py, security/*.py, integrations/*.py (SURVEY §2 C36–C45)."""

from __future__ import annotations

import hashlib
import json
from datetime import datetime, timedelta, timezone
from types import SimpleNamespace

import pytest

from hypervisor import _clock, config
from hypervisor.audit.commitment import CommitmentEngine
from hypervisor.audit.delta import DeltaEngine, VFSChange, canonical_payload
from hypervisor.audit.gc import EphemeralGC, RetentionPolicy
from hypervisor.integrations.cmvk_adapter import CMVKAdapter, DriftSeverity, DriftThresholds
from hypervisor.integrations.iatp_adapter import IATPAdapter, IATPTrustLevel, parse_undo_window
from hypervisor.integrations.nexus_adapter import NexusAdapter
from hypervisor.models import ExecutionRing, ReversibilityLevel
from hypervisor.observability.causal_trace import CausalTraceId
from hypervisor.observability.event_bus import EventType, HypervisorEvent, HypervisorEventBus
from hypervisor.security.kill_switch import HandoffStatus, KillReason, KillSwitch
from hypervisor.security.rate_limiter import AgentRateLimiter, RateLimitExceeded
from hypervisor.session.sso import SessionVFS

T0 = datetime(2026, 5, 1, 8, 30, tzinfo=timezone.utc)


@pytest.fixture()
def clock():
    class C:
        t = T0

        def advance(self, **kw):
            self.t += timedelta(**kw)

    c = C()
    _clock.set_clock(lambda: c.t)
    return c


def _py_merkle(hashes):
    level = list(hashes)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [hashlib.sha256((level[i] + level[i + 1]).encode()).hexdigest() for i in range(0, len(level), 2)]
    return level[0]


# ---------------------------------------------------------------------- audit


class TestDeltaEngine:
    def test_capture_chain_and_hash_definition(self, clock):
        de = DeltaEngine("sess")
        d1 = de.capture("did:a", [VFSChange("/f", "add", "h1")])
        d2 = de.capture("did:b", [VFSChange("/g", "modify", "h2", "h1", "did:b")], delta_id="custom")
        assert d1.delta_id == "delta:1" and d2.delta_id == "custom" and de.turn_count == 2
        assert d1.parent_hash is None and d2.parent_hash == d1.delta_hash
        payload = json.dumps({
            "delta_id": "delta:1", "turn_id": 1, "session_id": "sess", "agent_did": "did:a",
            "timestamp": T0.isoformat(),
            "changes": [{"path": "/f", "operation": "add", "content_hash": "h1", "previous_hash": None}],
            "parent_hash": None,
        }, sort_keys=True)
        assert canonical_payload(d1) == payload.encode()
        assert d1.delta_hash == hashlib.sha256(payload.encode()).hexdigest()

    def test_merkle_root(self):
        de = DeltaEngine("s")
        assert de.compute_merkle_root() is None
        for k in range(7):
            de.capture("a", [VFSChange(f"/f{k}", "add", f"h{k}")])
            assert de.compute_merkle_root() == _py_merkle([d.delta_hash for d in de.deltas])

    def test_verify_chain_detects_tampering_without_repair(self):
        de = DeltaEngine("s")
        for k in range(3):
            de.capture("a", [VFSChange(f"/f{k}", "add")])
        assert de.verify_chain()
        de._deltas[1].changes[0].path = "/evil"
        stored = de._deltas[1].delta_hash
        assert not de.verify_chain() and not de.verify_chain()  # stays broken
        assert de._deltas[1].delta_hash == stored

    def test_parity_mode_reproduces_self_repairing_verify(self):
        config.set_parity_mode(True)
        de = DeltaEngine("s")
        for k in range(2):
            de.capture("a", [VFSChange(f"/f{k}", "add")])
        de._deltas[1].changes[0].path = "/evil"
        assert de.verify_chain()  # the reference recomputes and overwrites (Q02)

    def test_broken_parent_link(self):
        de = DeltaEngine("s")
        de.capture("a", [])
        de.capture("a", [])
        de._deltas[1].parent_hash = "0" * 64
        de._deltas[1].compute_hash()
        assert not de.verify_chain()

    def test_export_records_self_verify(self):
        de = DeltaEngine("s")
        de.capture("a", [VFSChange("/x", "delete", previous_hash="p")])
        rec = de.export_records()[0]
        assert hashlib.sha256(rec["payload"].encode()).hexdigest() == rec["delta_hash"]

    def test_prune_expired(self, clock):
        de = DeltaEngine("s")
        de.capture("a", [])
        clock.advance(days=100)
        de.capture("a", [])
        assert de.prune_expired(90) == 1 and len(de.deltas) == 1


class TestCommitment:
    def test_commit_verify_batch(self):
        ce = CommitmentEngine()
        r = ce.commit("s1", "root", ["a", "b"], 3)
        assert r.committed_to == "local" and ce.verify("s1", "root") and not ce.verify("s1", "other")
        assert not ce.verify("s2", "root") and ce.get_commitment("s1") is r
        ce.queue_for_batch(r)
        assert ce.flush_batch() == [r] and ce.flush_batch() == []
        ce.commit("s1", "root2", [], 0)
        assert ce.commitment_count == 1 and ce.all_commitments()[0].merkle_root == "root2"


class TestGC:
    def test_collect_purges_vfs_and_records(self):
        vfs = SessionVFS("s")
        vfs.write("/a", "x" * 10, "d")
        vfs.write("/b", "y", "d")
        gc = EphemeralGC()
        res = gc.collect("s", vfs=vfs, delta_count=4, estimated_vfs_bytes=11, estimated_delta_bytes=100)
        assert res.purged_vfs_files == 2 and vfs.file_count == 0
        assert res.retained_deltas == 4 and res.retained_hash
        assert res.storage_saved_bytes == 11 and res.savings_pct == pytest.approx(11 / 111 * 100)
        assert gc.is_purged("s") and gc.purged_session_count == 1 and len(gc.history) == 1

    def test_parity_mode_counts_without_purging(self):
        config.set_parity_mode(True)
        vfs = SessionVFS("s")
        vfs.write("/a", "x", "d")
        assert EphemeralGC().collect("s", vfs=vfs).purged_vfs_files == 1
        assert vfs.file_count == 1  # reference GC never frees the VFS (Q01)

    def test_delta_retention(self, clock):
        de = DeltaEngine("s")
        de.capture("a", [])
        clock.advance(days=31)
        de.capture("a", [])
        gc = EphemeralGC(RetentionPolicy(delta_retention_days=30))
        res = gc.collect("s", delta_engine=de, delta_count=2)
        assert res.retained_deltas == 1 and len(de.deltas) == 1
        assert gc.should_expire_deltas(T0) and not gc.should_expire_deltas(clock.t)

    def test_empty_savings(self):
        assert EphemeralGC().collect("s").savings_pct == 0.0


# -------------------------------------------------------------- observability


class TestEventBus:
    def test_emit_query_and_indexes(self):
        bus = HypervisorEventBus()
        bus.emit(HypervisorEvent(event_type=EventType.SESSION_CREATED, session_id="s1", agent_did="a"))
        bus.publish(EventType.SESSION_JOINED, "s1", "b", ring=2)
        bus.publish(EventType.SESSION_CREATED, "s2")
        assert bus.event_count == 3
        assert len(bus.query_by_type(EventType.SESSION_CREATED)) == 2
        assert len(bus.query_by_session("s1")) == 2 and len(bus.query_by_agent("b")) == 1
        assert bus.query(session_id="s1", event_type=EventType.SESSION_JOINED)[0].payload == {"ring": 2}
        assert [e.session_id for e in bus.query(limit=1)] == ["s2"]
        assert bus.type_counts() == {"session.created": 2, "session.joined": 1}

    def test_subscribers(self):
        bus = HypervisorEventBus()
        seen, all_seen = [], []
        bus.subscribe(EventType.SLASH_EXECUTED, seen.append)
        bus.subscribe(None, all_seen.append)
        bus.subscribe(EventType.SLASH_EXECUTED, None)  # ignored
        bus.publish(EventType.SLASH_EXECUTED)
        bus.publish(EventType.VFS_WRITE)
        assert len(seen) == 1 and len(all_seen) == 2

    def test_time_range_and_clear(self, clock):
        bus = HypervisorEventBus()
        bus.publish(EventType.VFS_WRITE)
        clock.advance(seconds=10)
        bus.publish(EventType.VFS_DELETE)
        assert len(bus.query_by_time_range(T0 + timedelta(seconds=5))) == 1
        assert len(bus.query_by_time_range(T0, T0)) == 1
        bus.clear()
        assert bus.event_count == 0 and bus.all_events == [] and bus.type_counts() == {}

    def test_event_to_dict(self):
        e = HypervisorEvent(event_type=EventType.AUDIT_COMMITTED, payload={"root": "r"})
        d = e.to_dict()
        assert d["event_type"] == "audit.committed" and len(d["event_id"]) == 16 and d["payload"] == {"root": "r"}

    def test_event_type_catalogue(self):
        assert len(EventType) == 40 and EventType("ring.breach_detected") == EventType.RING_BREACH_DETECTED


class TestCausalTrace:
    def test_child_sibling_ancestry(self):
        root = CausalTraceId()
        c = root.child()
        s = c.sibling()
        assert c.trace_id == root.trace_id and c.parent_span_id == root.span_id and c.depth == 1
        assert s.parent_span_id == root.span_id and s.depth == 1 and s.span_id != c.span_id
        assert root.is_ancestor_of(c) and not c.is_ancestor_of(root)
        assert not root.is_ancestor_of(CausalTraceId().child())

    def test_string_roundtrip(self):
        c = CausalTraceId().child()
        back = CausalTraceId.from_string(str(c))
        assert (back.trace_id, back.span_id, back.parent_span_id) == (c.trace_id, c.span_id, c.parent_span_id)
        assert str(CausalTraceId(trace_id="t", span_id="s")) == "t/s"
        with pytest.raises(ValueError):
            CausalTraceId.from_string("nope")


# ------------------------------------------------------------------- security


class TestRateLimiter:
    def test_ring_budgets(self, clock):
        rl = AgentRateLimiter()
        for _ in range(10):
            rl.check("a", "s", ExecutionRing.RING_3_SANDBOX)
        with pytest.raises(RateLimitExceeded, match="ring 3"):
            rl.check("a", "s", ExecutionRing.RING_3_SANDBOX)
        assert not rl.try_check("a", "s", ExecutionRing.RING_3_SANDBOX)
        st = rl.get_stats("a", "s")
        assert st.total_requests == 12 and st.rejected_requests == 2 and st.capacity == 10
        clock.advance(seconds=1)  # 5 tokens/s refill
        assert rl.get_stats("a", "s").tokens_available == pytest.approx(5.0)
        for _ in range(5):
            rl.check("a", "s", ExecutionRing.RING_3_SANDBOX)

    def test_update_ring_resets_bucket(self):
        rl = AgentRateLimiter()
        for _ in range(10):
            rl.check("a", "s", ExecutionRing.RING_3_SANDBOX)
        rl.update_ring("a", "s", ExecutionRing.RING_1_PRIVILEGED)
        assert rl.get_stats("a", "s").ring == ExecutionRing.RING_1_PRIVILEGED
        for _ in range(100):
            rl.check("a", "s", ExecutionRing.RING_1_PRIVILEGED)
        assert rl.tracked_agents == 1 and rl.get_stats("x", "y") is None

    def test_custom_limits_and_cost(self):
        rl = AgentRateLimiter({ExecutionRing.RING_2_STANDARD: (1.0, 3.0)})
        assert rl.try_check("a", "s", ExecutionRing.RING_2_STANDARD, cost=3.0)
        assert not rl.try_check("a", "s", ExecutionRing.RING_2_STANDARD, cost=1.0)
        assert rl.try_check("b", "s", ExecutionRing.RING_0_ROOT, cost=40.0)  # fallback (20/s, 40)


class TestKillSwitch:
    def test_handoff_to_substitute(self):
        ks = KillSwitch()
        ks.register_substitute("s", "bad")
        ks.register_substitute("s", "backup")
        r = ks.kill("bad", "s", KillReason.RING_BREACH, [{"step_id": "1", "saga_id": "g"}, {"step_id": "2"}])
        assert r.kill_id.startswith("kill:") and r.handoff_success_count == 2
        assert all(h.to_agent == "backup" and h.status == HandoffStatus.HANDED_OFF for h in r.handoffs)
        assert not r.compensation_triggered and ks.total_handoffs == 2

    def test_no_substitute_compensates(self):
        ks = KillSwitch()
        r = ks.kill("a", "s", KillReason.MANUAL, [{"step_id": "1"}], details="operator")
        assert r.handoffs[0].status == HandoffStatus.COMPENSATED and r.compensation_triggered
        assert ks.total_kills == 1 and ks.kill_history[0].details == "operator"

    def test_killed_agent_leaves_substitute_pool(self):
        ks = KillSwitch()
        ks.register_substitute("s", "a")
        ks.register_substitute("s", "b")
        ks.kill("a", "s", KillReason.MANUAL)
        r = ks.kill("b", "s", KillReason.MANUAL, [{"step_id": "x"}])
        assert r.handoffs[0].status == HandoffStatus.COMPENSATED
        ks.unregister_substitute("s", "zz")


# ---------------------------------------------------------------- integrations


class FakeScorer:
    def __init__(self, score=850):
        self.score, self.slashes, self.outcomes = score, [], []

    def calculate_trust_score(self, verification_level, history, capabilities):
        return SimpleNamespace(total_score=self.score, successful_tasks=7, failed_tasks=1)

    def slash_reputation(self, agent_did, reason, severity, evidence_hash):
        self.slashes.append((agent_did, severity))

    def record_task_outcome(self, agent_did, outcome):
        self.outcomes.append(outcome)


class TestNexus:
    def test_without_scorer(self):
        assert NexusAdapter().resolve_sigma("a") == 0.5

    def test_resolve_cache_and_tiers(self, clock):
        sc = FakeScorer(850)
        nx = NexusAdapter(scorer=sc, cache_ttl_seconds=60)
        assert nx.resolve_sigma("a") == 0.85
        r = nx.get_cached_result("a")
        assert r.tier == "trusted" and r.successful_tasks == 7
        sc.score = 200
        assert nx.resolve_sigma("a") == 0.85  # cached
        clock.advance(seconds=61)
        assert nx.resolve_sigma("a") == 0.2 and nx.get_cached_result("a").tier == "untrusted"
        for s, tier in [(950, "verified_partner"), (500, "standard"), (300, "probationary")]:
            assert nx._score_to_tier(s) == tier

    def test_reports_invalidate_cache(self):
        sc = FakeScorer()
        nx = NexusAdapter(scorer=sc)
        nx.resolve_sigma("a")
        nx.report_slash("a", "drift", severity="high")
        assert sc.slashes == [("a", "high")] and nx.get_cached_result("a") is None
        nx.resolve_sigma("a")
        nx.report_task_outcome("a", "success")
        assert sc.outcomes == ["success"] and nx.get_cached_result("a") is None
        nx.resolve_sigma("b")
        nx.invalidate_cache()
        assert nx.get_cached_result("b") is None

    async def test_verify_agent(self):
        class V:
            async def verify_peer(self, agent_did, min_score):
                return SimpleNamespace(is_verified=min_score <= 600)

        assert await NexusAdapter().verify_agent("a")
        assert await NexusAdapter(verifier=V()).verify_agent("a", 500)
        assert not await NexusAdapter(verifier=V()).verify_agent("a", 700)


class FakeVerifier:
    def __init__(self, scores):
        self.scores = list(scores)

    def verify_embeddings(self, embedding_a, embedding_b, metric, threshold_profile, explain):
        return SimpleNamespace(drift_score=self.scores.pop(0), explanation="diff")


class TestCMVK:
    def test_no_verifier_passes(self):
        r = CMVKAdapter().check_behavioral_drift("a", "s", [1], [1])
        assert r.passed and r.severity == DriftSeverity.NONE

    def test_severity_bands_and_callbacks(self):
        hits = []
        ad = CMVKAdapter(FakeVerifier([0.1, 0.2, 0.35, 0.6, 0.8]), on_drift_detected=hits.append)
        res = [ad.check_behavioral_drift("a", "s", None, None) for _ in range(5)]
        assert [r.severity.value for r in res] == ["none", "low", "medium", "high", "critical"]
        assert [r.passed for r in res] == [True, True, False, False, False]
        assert res[2].should_demote and res[3].should_slash and res[4].should_slash
        assert len(hits) == 3 and ad.total_checks == 5 and ad.total_violations == 3
        assert ad.get_drift_rate("a") == 0.6 and ad.get_mean_drift_score("a", "s") == pytest.approx(0.41)
        assert ad.get_drift_rate("zz") == 0.0 and res[4].explanation == "diff"

    def test_custom_thresholds(self):
        ad = CMVKAdapter(FakeVerifier([0.2]), thresholds=DriftThresholds(low=0.05, medium=0.1, high=0.15, critical=0.9))
        assert ad.check_behavioral_drift("a", "s", 0, 0).severity == DriftSeverity.HIGH


class TestIATP:
    @pytest.mark.parametrize("text,secs", [("30s", 30), ("5m", 300), ("2h", 7200), ("45", 45), ("", 0),
                                           (None, 0), ("bogus", 0), ("1.5m", 90)])
    def test_undo_window(self, text, secs):
        assert parse_undo_window(text) == secs

    def test_undo_window_parity_mode(self):
        config.set_parity_mode(True)
        assert parse_undo_window("5m") == 5  # reference strips the unit (Q21)

    def test_manifest_dict(self):
        ad = IATPAdapter()
        a = ad.analyze_manifest_dict({
            "agent_id": "did:x", "trust_level": "trusted", "trust_score": 8, "scopes": ["fs"],
            "actions": [{"action_id": "w", "reversibility": "full", "undo_api": "/u"},
                        {"action_id": "d", "reversibility": "none"},
                        {"action_id": "r", "is_read_only": True}],
        })
        assert a.trust_level == IATPTrustLevel.TRUSTED and a.ring_hint == ExecutionRing.RING_2_STANDARD
        assert a.sigma_hint == 0.8 and a.has_reversible_actions and a.has_non_reversible_actions
        assert a.actions[0].reversibility == ReversibilityLevel.FULL and ad.get_cached_analysis("did:x") is a

    def test_unknown_trust_level_sandboxed(self):
        a = IATPAdapter().analyze_manifest_dict({"agent_id": "x", "trust_level": "weird"})
        assert a.trust_level == IATPTrustLevel.UNKNOWN and a.ring_hint == ExecutionRing.RING_3_SANDBOX
        assert a.sigma_hint == 0.5 and a.actions == []

    def test_manifest_object(self):
        caps = SimpleNamespace(reversibility=SimpleNamespace(value="partial"), undo_window="10m")
        m = SimpleNamespace(agent_id="did:y", trust_level=SimpleNamespace(value="verified_partner"),
                            scopes=("a",), capabilities=caps, calculate_trust_score=lambda: 12)
        a = IATPAdapter().analyze_manifest(m)
        assert a.ring_hint == ExecutionRing.RING_1_PRIVILEGED and a.sigma_hint == 1.0
        act = a.actions[0]
        assert act.action_id == "did:y:default" and act.undo_api == "/api/did:y/undo"
        assert act.undo_window_seconds == 600 and a.scopes == ["a"]
