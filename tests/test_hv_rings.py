"""Execution rings, action classification, elevation/inheritance, breach
detection, reversibility registry and history verification (reference
rings/*.py, reversibility/registry.py, verification/history.py; SURVEY §2
C09–C15, C26, C27)."""

from __future__ import annotations

from datetime import datetime, timedelta, timezone

import pytest

from hypervisor import _clock
from hypervisor.models import ActionDescriptor, ExecutionRing, ReversibilityLevel
from hypervisor.reversibility.registry import ReversibilityRegistry
from hypervisor.rings.breach_detector import BreachSeverity, RingBreachDetector, classify_rate
from hypervisor.rings.classifier import ActionClassifier
from hypervisor.rings.elevation import RingElevationError, RingElevationManager
from hypervisor.rings.enforcer import RingEnforcer
from hypervisor.verification.history import TransactionHistoryVerifier, TransactionRecord, VerificationStatus

T0 = datetime(2026, 3, 1, 12, 0, tzinfo=timezone.utc)
R0, R1, R2, R3 = (ExecutionRing(k) for k in range(4))


def _act(aid="a", rev=ReversibilityLevel.FULL, undo="/undo", **kw) -> ActionDescriptor:
    return ActionDescriptor(action_id=aid, name=aid, execute_api=f"/{aid}", undo_api=undo, reversibility=rev, **kw)


class FakeClock:
    def __init__(self, t=T0):
        self.t = t
        _clock.set_clock(lambda: self.t)

    def advance(self, **kw):
        self.t += timedelta(**kw)


# --------------------------------------------------------------- models


class TestRingModel:
    @pytest.mark.parametrize("sigma,consensus,ring", [
        (0.0, False, R3), (0.60, False, R3), (0.6000001, False, R2), (0.99, False, R2),
        (0.95, True, R2), (0.951, True, R1), (0.5, True, R3),
    ])
    def test_from_sigma_eff(self, sigma, consensus, ring):
        assert ExecutionRing.from_sigma_eff(sigma, consensus) == ring

    def test_ordering_is_privilege(self):
        assert R0 < R1 < R2 < R3

    def test_risk_weights(self):
        assert _act(rev=ReversibilityLevel.FULL).risk_weight == pytest.approx(0.2)
        assert _act(rev=ReversibilityLevel.PARTIAL).risk_weight == pytest.approx(0.65)
        assert _act(rev=ReversibilityLevel.NONE).risk_weight == pytest.approx(0.95)
        assert ReversibilityLevel.PARTIAL.risk_weight_range == (0.5, 0.8)

    def test_required_ring(self):
        assert _act(is_admin=True, is_read_only=True).required_ring == R0
        assert _act(is_read_only=True, rev=ReversibilityLevel.NONE).required_ring == R3
        assert _act(rev=ReversibilityLevel.NONE).required_ring == R1
        assert _act(rev=ReversibilityLevel.PARTIAL).required_ring == R2
        assert _act(rev=ReversibilityLevel.FULL).required_ring == R2


# -------------------------------------------------------------- enforcer


class TestEnforcer:
    enf = RingEnforcer()

    def test_ring0_needs_witness(self):
        r = self.enf.check(R0, _act(is_admin=True), 1.0)
        assert not r.allowed and r.requires_sre_witness and "SRE Witness" in r.reason
        assert self.enf.check(R0, _act(is_admin=True), 1.0, has_sre_witness=True).allowed

    def test_ring1_needs_sigma_then_consensus(self):
        act = _act(rev=ReversibilityLevel.NONE)
        r = self.enf.check(R1, act, 0.9, has_consensus=True)
        assert not r.allowed and "σ_eff > 0.95, got 0.900" in r.reason
        r = self.enf.check(R1, act, 0.97)
        assert not r.allowed and r.requires_consensus
        assert self.enf.check(R1, act, 0.97, has_consensus=True).allowed

    def test_ring2_sigma(self):
        r = self.enf.check(R2, _act(), 0.5)
        assert not r.allowed and "Ring 2 requires" in r.reason
        assert self.enf.check(R2, _act(), 0.7).allowed

    def test_insufficient_ring(self):
        r = self.enf.check(R3, _act(), 0.99)
        assert not r.allowed and r.reason == "Agent ring 3 insufficient for required ring 2"

    def test_sandbox_reads_always_allowed(self):
        r = self.enf.check(R3, _act(is_read_only=True), 0.0)
        assert r.allowed and r.reason == "Access granted" and r.required_ring == R3

    def test_compute_ring_and_demotion(self):
        assert self.enf.compute_ring(0.97, has_consensus=True) == R1
        assert self.enf.should_demote(R2, 0.3)
        assert not self.enf.should_demote(R2, 0.8)
        assert not self.enf.should_demote(R3, 0.1)


# ------------------------------------------------------------ classifier


class TestClassifier:
    def test_classify_and_cache(self):
        c = ActionClassifier()
        a = _act("x", rev=ReversibilityLevel.PARTIAL)
        r = c.classify(a)
        assert r.ring == R2 and r.risk_weight == pytest.approx(0.65) and r.confidence == 1.0
        # cached by id: a changed descriptor with the same id returns the cached result
        assert c.classify(_act("x", rev=ReversibilityLevel.NONE)) is r
        c.clear_cache()
        assert c.classify(_act("x", rev=ReversibilityLevel.NONE)).ring == R1

    def test_override_wins(self):
        c = ActionClassifier()
        c.classify(_act("y"))
        c.set_override("y", ring=R1)
        r = c.classify(_act("y"))
        assert r.ring == R1 and r.risk_weight == pytest.approx(0.2) and r.confidence == 0.9

    def test_override_of_unknown_action(self):
        c = ActionClassifier()
        c.set_override("z", risk_weight=0.7)
        r = c.classify(_act("z"))
        assert r.ring == R3 and r.risk_weight == 0.7 and r.reversibility == ReversibilityLevel.NONE


# ------------------------------------------------------------- elevation


class TestElevation:
    def test_grant_and_effective_ring(self):
        clk = FakeClock()
        m = RingElevationManager()
        e = m.request_elevation("a", "s", R3, R2, ttl_seconds=60, reason="deploy")
        assert e.elevation_id.startswith("elev:") and e.remaining_seconds == 60
        assert m.get_effective_ring("a", "s", R3) == R2
        assert m.get_effective_ring("a", "other", R3) == R3
        clk.advance(seconds=61)
        assert e.is_expired and m.get_effective_ring("a", "s", R3) == R3
        assert [x.elevation_id for x in m.tick()] == [e.elevation_id] and not e.is_active

    def test_rejections(self):
        FakeClock()
        m = RingElevationManager()
        with pytest.raises(RingElevationError, match="not more privileged"):
            m.request_elevation("a", "s", R2, R2)
        with pytest.raises(RingElevationError, match="Ring 0"):
            m.request_elevation("a", "s", R2, R0)
        m.request_elevation("a", "s", R3, R2)
        with pytest.raises(RingElevationError, match="already has active elevation"):
            m.request_elevation("a", "s", R3, R1)

    def test_ttl_default_and_cap(self):
        FakeClock()
        m = RingElevationManager()
        assert m.request_elevation("a", "s", R3, R2).remaining_seconds == 300
        assert m.request_elevation("b", "s", R3, R2, ttl_seconds=10**6).remaining_seconds == 3600

    def test_revoke(self):
        FakeClock()
        m = RingElevationManager()
        e = m.request_elevation("a", "s", R3, R2)
        m.revoke_elevation(e.elevation_id)
        assert m.active_elevations == [] and m.elevation_count == 1
        m.request_elevation("a", "s", R3, R2)  # allowed again
        with pytest.raises(RingElevationError):
            m.revoke_elevation("elev:missing")

    def test_child_inheritance(self):
        m = RingElevationManager()
        assert m.register_child("p", "c1", R1) == R2
        assert m.register_child("p", "c2", R3) == R3
        assert m.get_parent("c1") == "p" and m.get_children("p") == ["c1", "c2"]
        assert m.get_max_child_ring(R0) == R1 and m.get_parent("zz") is None


# ------------------------------------------------------------ breach


class TestBreach:
    @pytest.mark.parametrize("rate,sev", [(0.0, "none"), (0.29, "none"), (0.3, "low"), (0.5, "medium"),
                                          (0.7, "high"), (0.9, "critical"), (1.0, "critical")])
    def test_classify_rate(self, rate, sev):
        assert classify_rate(rate).value == sev

    def test_needs_min_calls(self):
        FakeClock()
        d = RingBreachDetector()
        for _ in range(4):
            assert d.record_call("a", "s", R3, R0) is None
        ev = d.record_call("a", "s", R3, R0)
        assert ev is not None and ev.severity == BreachSeverity.CRITICAL and ev.call_count_window == 5
        assert d.breach_count == 1 and "5/5" in ev.details

    def test_breaker_trips_and_cools_down(self):
        clk = FakeClock()
        d = RingBreachDetector()
        for _ in range(5):
            d.record_call("a", "s", R3, R1)
        assert d.is_breaker_tripped("a", "s")
        assert d.record_call("a", "s", R3, R1) is None  # cooling: analysis suppressed
        clk.advance(seconds=31)
        assert not d.is_breaker_tripped("a", "s")
        d.reset_breaker("a", "s")
        assert not d.is_breaker_tripped("zz", "s")

    def test_window_prunes_old_calls(self):
        clk = FakeClock()
        d = RingBreachDetector(window_seconds=10)
        for _ in range(5):
            d.record_call("a", "s", R2, R3)
        clk.advance(seconds=11)
        d.record_call("a", "s", R2, R3)
        st = d.get_agent_stats("a", "s")
        assert st["window_calls"] == 1 and st["total_calls"] == 6 and st["ring_distribution"] == {3: 6}

    def test_mixed_rate_medium(self):
        FakeClock()
        d = RingBreachDetector()
        evs = [d.record_call("a", "s", R2, R1 if k % 2 else R3) for k in range(10)]
        assert evs[-1].severity == BreachSeverity.MEDIUM and evs[-1].anomaly_score == 0.5

    def test_unknown_agent_stats(self):
        assert RingBreachDetector().get_agent_stats("x", "y") == {
            "total_calls": 0, "window_calls": 0, "breaker_tripped": False}


# -------------------------------------------------------- reversibility


class TestReversibilityRegistry:
    def test_register_and_query(self):
        r = ReversibilityRegistry("s")
        r.register(_act("a", rev=ReversibilityLevel.FULL, undo="/ua"))
        r.register(_act("b", rev=ReversibilityLevel.NONE, undo=None))
        assert r.get_undo_api("a") == "/ua" and r.get_undo_api("zz") is None
        assert r.is_reversible("a") and not r.is_reversible("b") and not r.is_reversible("zz")
        assert r.get_risk_weight("a") == pytest.approx(0.2)
        assert r.get_risk_weight("unknown") == pytest.approx(0.95)
        assert r.has_non_reversible_actions() and r.non_reversible_actions == ["b"]

    def test_overwrite_updates_mode_negotiation(self):
        r = ReversibilityRegistry("s")
        assert not r.has_non_reversible_actions()
        r.register(_act("a", rev=ReversibilityLevel.NONE))
        r.register(_act("a", rev=ReversibilityLevel.FULL))
        assert not r.has_non_reversible_actions() and len(r.entries) == 1

    def test_manifest_and_health(self):
        r = ReversibilityRegistry("s")
        assert r.register_from_manifest([_act("a"), _act("b")]) == 2
        r.mark_undo_unhealthy("a")
        r.mark_undo_unhealthy("zz")
        assert not r.get("a").undo_api_healthy and r.get("b").undo_api_healthy


# ------------------------------------------------------------ history


def _hist(n, start=T0, step=1, bad=None):
    out = []
    for k in range(n):
        h = f"{k:032x}" if bad != k else "short"
        out.append(TransactionRecord(session_id=f"s{k}", summary_hash=h, timestamp=start + timedelta(hours=step * k)))
    return out


class TestHistoryVerifier:
    def test_no_history_probationary(self):
        r = TransactionHistoryVerifier().verify("a")
        assert r.status == VerificationStatus.PROBATIONARY and r.is_trustworthy

    def test_short_history(self):
        r = TransactionHistoryVerifier().verify("a", _hist(3))
        assert r.status == VerificationStatus.PROBATIONARY and "Only 3" in r.inconsistencies[0]

    def test_verified(self):
        r = TransactionHistoryVerifier().verify("a", _hist(6))
        assert r.status == VerificationStatus.VERIFIED and r.transactions_checked == 6

    def test_suspicious_cases(self):
        v = TransactionHistoryVerifier()
        assert v.verify("a", _hist(6, bad=2)).status == VerificationStatus.SUSPICIOUS
        assert v.verify("b", _hist(6, step=-1)).status == VerificationStatus.SUSPICIOUS
        dup = _hist(6)
        dup[4].summary_hash = dup[1].summary_hash
        r = v.verify("c", dup)
        assert r.status == VerificationStatus.SUSPICIOUS and not r.is_trustworthy
        assert any("Duplicate" in i for i in r.inconsistencies)

    def test_cache(self):
        v = TransactionHistoryVerifier()
        r1 = v.verify("a", _hist(6))
        r2 = v.verify("a")
        assert r2 is r1 and r2.cached
        v.clear_cache("a")
        assert v.verify("a").status == VerificationStatus.PROBATIONARY
        v.clear_cache()
