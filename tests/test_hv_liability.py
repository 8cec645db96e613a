"""Joint liability: vouching/bonding, slashing cascades, the liability matrix,
causal fault attribution, quarantine and the liability ledger (reference
liability/*.py; SURVEY §2 C16–C23)."""

from __future__ import annotations

from datetime import datetime, timedelta, timezone

import pytest

from hypervisor import _clock, config
from hypervisor.liability import LiabilityMatrix
from hypervisor.liability.attribution import CausalAttributor
from hypervisor.liability.ledger import LedgerEntryType, LiabilityLedger
from hypervisor.liability.quarantine import QuarantineManager, QuarantineReason
from hypervisor.liability.slashing import SlashingEngine, clip_sigma
from hypervisor.liability.vouching import VouchingEngine, VouchingError

T0 = datetime(2026, 4, 1, tzinfo=timezone.utc)


@pytest.fixture()
def clock():
    class C:
        t = T0

        def advance(self, **kw):
            self.t += timedelta(**kw)

    c = C()
    _clock.set_clock(lambda: c.t)
    return c


# ----------------------------------------------------------------- vouching


class TestVouching:
    def test_bond_amount_and_defaults(self):
        ve = VouchingEngine()
        r = ve.vouch("hi", "lo", "s", 0.9)
        assert r.vouch_id.startswith("vouch:") and r.bonded_sigma_pct == 0.2
        assert r.bonded_amount == pytest.approx(0.18) and r.is_active and r.is_live
        assert r.session_id == "s" and r.expiry is None and r.released_at is None

    def test_pct_clamped(self):
        ve = VouchingEngine(max_exposure=1.0)
        assert ve.vouch("a", "b", "s", 0.8, bond_pct=-1).bonded_amount == 0.0
        assert ve.vouch("a", "c", "s", 0.8, bond_pct=5).bonded_amount == pytest.approx(0.8)

    def test_rejections(self):
        ve = VouchingEngine()
        with pytest.raises(VouchingError, match="yourself"):
            ve.vouch("a", "a", "s", 0.9)
        with pytest.raises(VouchingError, match="below minimum"):
            ve.vouch("a", "b", "s", 0.49)
        ve.vouch("a", "b", "s", 0.9)
        with pytest.raises(VouchingError, match="Circular"):
            ve.vouch("b", "a", "s", 0.9)
        ve.vouch("b", "a", "other-session", 0.9)  # cycles are session-scoped

    def test_transitive_cycle(self):
        ve = VouchingEngine()
        ve.vouch("a", "b", "s", 0.9, bond_pct=0.1)
        ve.vouch("b", "c", "s", 0.9, bond_pct=0.1)
        with pytest.raises(VouchingError, match="Circular"):
            ve.vouch("c", "a", "s", 0.9, bond_pct=0.1)

    def test_diamond_is_not_a_cycle_but_parity_mode_reproduces_reference(self):
        def build():
            ve = VouchingEngine()
            ve.vouch("b", "c", "s", 0.9, bond_pct=0.1)
            ve.vouch("b", "d", "s", 0.9, bond_pct=0.1)
            ve.vouch("c", "e", "s", 0.9, bond_pct=0.1)
            ve.vouch("d", "e", "s", 0.9, bond_pct=0.1)
            return ve

        build().vouch("a", "b", "s", 0.9, bond_pct=0.1)  # fixed behaviour: admitted
        config.set_parity_mode(True)
        with pytest.raises(VouchingError, match="Circular"):
            build().vouch("a", "b", "s", 0.9, bond_pct=0.1)  # reference BFS false positive (Q05)

    def test_exposure_limit(self):
        ve = VouchingEngine()
        for k in range(4):
            ve.vouch("a", f"v{k}", "s", 1.0)  # 4 × 0.2 = 0.8 = limit
        with pytest.raises(VouchingError, match="max exposure"):
            ve.vouch("a", "v9", "s", 1.0)
        assert ve.get_total_exposure("a", "s") == pytest.approx(0.8)
        assert ve.get_total_exposure("a", "other") == 0.0

    def test_sigma_eff(self):
        ve = VouchingEngine()
        ve.vouch("a", "z", "s", 0.9, bond_pct=0.5)
        ve.vouch("b", "z", "s", 0.8, bond_pct=0.5)
        assert ve.compute_sigma_eff("z", "s", 0.3, 0.5) == pytest.approx(0.3 + 0.5 * (0.45 + 0.4))
        assert ve.compute_sigma_eff("z", "s", 0.9, 1.0) == 1.0  # capped
        assert ve.compute_sigma_eff("z", "other", 0.3, 0.5) == 0.3

    def test_expiry_excludes_bond(self, clock):
        ve = VouchingEngine()
        r = ve.vouch("a", "z", "s", 0.9, expiry=T0 + timedelta(seconds=10))
        assert ve.get_vouchers_for("z", "s") == [r]
        clock.advance(seconds=11)
        assert r.is_expired and ve.get_vouchers_for("z", "s") == []
        assert ve.compute_sigma_eff("z", "s", 0.3, 1.0) == 0.3

    def test_release(self):
        ve = VouchingEngine()
        r = ve.vouch("a", "z", "s", 0.9)
        ve.vouch("b", "z", "s", 0.9)
        ve.release_bond(r.vouch_id)
        assert not r.is_active and r.released_at is not None
        with pytest.raises(VouchingError, match="not found"):
            ve.release_bond("vouch:nope")
        assert ve.release_session_bonds("s") == 1 and ve.release_session_bonds("s") == 0
        assert len(ve.records("s")) == 2 and len(ve.records()) == 2


# ------------------------------------------------------------------ slashing


class TestSlashing:
    def test_clip_formula(self):
        assert clip_sigma(0.8, 0.5) == pytest.approx(0.4)
        assert clip_sigma(0.1, 0.95) == 0.05

    def test_slash_clips_vouchers_and_releases(self):
        ve = VouchingEngine()
        se = SlashingEngine(ve)
        ve.vouch("v1", "bad", "s", 0.9)
        ve.vouch("v2", "bad", "s", 0.8)
        scores = {"bad": 0.7, "v1": 0.9, "v2": 0.8}
        res = se.slash("bad", "s", 0.7, 0.5, "drift", scores)
        assert scores["bad"] == 0.0
        assert scores["v1"] == pytest.approx(0.45) and scores["v2"] == pytest.approx(0.4)
        assert [c.voucher_did for c in res.voucher_clips] == ["v1", "v2"]
        assert res.vouchee_sigma_after == 0.0 and res.cascade_depth == 0 and res.slash_id.startswith("slash:")
        assert ve.get_vouchers_for("bad", "s") == []

    def test_unknown_voucher_starts_from_zero(self):
        ve = VouchingEngine()
        ve.vouch("ghost", "bad", "s", 0.9)
        scores = {}
        SlashingEngine(ve).slash("bad", "s", 0.5, 0.5, "r", scores)
        assert scores["ghost"] == 0.05

    def test_cascade_to_depth_two(self):
        ve = VouchingEngine()
        se = SlashingEngine(ve)
        ve.vouch("c", "b", "s", 0.9)
        ve.vouch("b", "a", "s", 0.9)
        ve.vouch("d", "c", "s", 0.9)
        ve.vouch("e", "d", "s", 0.9)
        scores = {k: 0.9 for k in "abcde"}
        se.slash("a", "s", 0.9, 0.99, "root", scores)
        hist = se.history
        assert [h.vouchee_did for h in hist] == ["a", "b", "c"]
        assert [h.cascade_depth for h in hist] == [0, 1, 2]
        assert hist[1].reason.startswith("Cascade from a:")
        assert scores["d"] == 0.05 and scores["e"] == 0.9  # depth limit stops before e

    def test_no_cascade_when_voucher_stays_above_floor(self):
        ve = VouchingEngine()
        se = SlashingEngine(ve)
        ve.vouch("b", "a", "s", 0.9)
        ve.vouch("c", "b", "s", 0.9)
        scores = {"a": 0.5, "b": 0.9, "c": 0.9}
        se.slash("a", "s", 0.5, 0.3, "minor", scores)
        assert len(se.history) == 1 and scores["c"] == 0.9


# ------------------------------------------------------------------ matrix


class TestLiabilityMatrix:
    def test_edges_and_exposure(self):
        m = LiabilityMatrix("s")
        m.add_edge("a", "b", 0.2, "v1")
        m.add_edge("a", "c", 0.3, "v2")
        assert m.total_exposure("a") == pytest.approx(0.5)
        assert [e.vouch_id for e in m.who_is_vouched_by("a")] == ["v1", "v2"]
        assert [e.voucher_did for e in m.who_vouches_for("c")] == ["a"]
        m.remove_edge("v1")
        assert len(m.edges) == 1
        m.clear()
        assert m.edges == []

    def test_cycle_detection(self):
        m = LiabilityMatrix("s")
        m.add_edge("a", "b", 0.1, "1")
        m.add_edge("b", "c", 0.1, "2")
        assert not m.has_cycle()
        m.add_edge("c", "a", 0.1, "3")
        assert m.has_cycle()

    def test_cascade_paths(self):
        m = LiabilityMatrix("s")
        m.add_edge("a", "b", 0.1, "1")
        m.add_edge("b", "c", 0.1, "2")
        m.add_edge("c", "d", 0.1, "3")
        paths = m.cascade_path("a", max_depth=2)
        assert ["a", "b"] in paths and ["a", "b", "c"] in paths
        assert all(len(p) <= 4 for p in paths)
        assert m.cascade_path("d") == []


# -------------------------------------------------------------- attribution


class TestAttribution:
    def test_direct_cause_dominates(self):
        ca = CausalAttributor()
        res = ca.attribute(
            "saga", "s",
            {"a": [{"action_id": "x", "step_id": "1", "success": True}],
             "b": [{"action_id": "y", "step_id": "2", "success": False}]},
            failure_step_id="2", failure_agent_did="b",
        )
        assert res.attributions[0].agent_did == "b" and res.attributions[0].is_direct_cause
        assert res.root_cause_agent == "b" and res.causal_chain_length == 2
        assert sum(a.liability_score for a in res.attributions) == pytest.approx(1.0, abs=1e-3)
        assert res.get_liability("nobody") == 0.0 and set(res.agents_involved) == {"a", "b"}
        assert res.attribution_id.startswith("attr:") and ca.attribution_history == [res]

    def test_raw_scores_formula(self):
        ca = CausalAttributor()
        nodes = ca.build_causal_dag(
            {"a": [{"action_id": "w", "step_id": "1", "success": False},
                   {"action_id": "w", "step_id": "2", "success": False}],
             "b": [{"action_id": "q", "step_id": "3", "success": False}]},
            failure_step_id="3", failure_agent_did="b")
        raw = ca.raw_scores(nodes, ["a", "b"], {"w": 0.9})
        # a: two enabling failures (0.3/2 each) + proximity 0.2*0.9/2 per node
        assert raw["a"] == pytest.approx(0.3 + 0.2 * 0.9)
        assert raw["b"] == pytest.approx(0.5 + 0.2 * 0.5)

    def test_risk_weight_default(self):
        ca = CausalAttributor()
        res = ca.attribute("g", "s", {"a": [{"action_id": "x", "step_id": "1"}]}, "1", "a")
        assert res.attributions[0].liability_score == 1.0


# ---------------------------------------------------------------- quarantine


class TestQuarantine:
    def test_enter_escalate_release(self, clock):
        qm = QuarantineManager()
        r = qm.quarantine("a", "s", QuarantineReason.RING_BREACH, "first", forensic_data={"k": 1})
        assert qm.is_quarantined("a", "s") and r.quarantine_id.startswith("quar:")
        r2 = qm.quarantine("a", "s", QuarantineReason.MANUAL, "second", forensic_data={"j": 2})
        assert r2 is r and r.details == "first; escalated: second" and r.forensic_data == {"k": 1, "j": 2}
        clock.advance(seconds=5)
        rel = qm.release("a", "s")
        assert rel is r and not r.is_active and r.duration_seconds == 5
        assert qm.release("a", "s") is None

    def test_default_duration_and_tick(self, clock):
        qm = QuarantineManager()
        r = qm.quarantine("a", "s", QuarantineReason.MANUAL, duration_seconds=None)
        assert r.expires_at == T0 + timedelta(seconds=300)
        clock.advance(seconds=301)
        assert not qm.is_quarantined("a", "s") and qm.quarantine_count == 0
        assert qm.tick() == [r] and r.released_at is not None

    def test_history_filters(self):
        qm = QuarantineManager()
        qm.quarantine("a", "s1", QuarantineReason.MANUAL)
        qm.quarantine("b", "s1", QuarantineReason.MANUAL)
        qm.quarantine("a", "s2", QuarantineReason.MANUAL)
        assert len(qm.get_history()) == 3 and len(qm.get_history(agent_did="a")) == 2
        assert len(qm.get_history(session_id="s1")) == 2 and len(qm.active_quarantines) == 3


# -------------------------------------------------------------------- ledger


class TestLedger:
    def test_empty_profile(self):
        p = LiabilityLedger().compute_risk_profile("x")
        assert p.risk_score == 0.0 and p.recommendation == "admit"

    def test_risk_accumulates_and_clamps(self):
        led = LiabilityLedger()
        for _ in range(3):
            led.record("a", LedgerEntryType.SLASH_RECEIVED, severity=0.2)  # 0.15 * max(0.2, 0.5)
        p = led.compute_risk_profile("a")
        assert p.risk_score == pytest.approx(0.225) and p.recommendation == "admit" and p.slash_count == 3
        led.record("a", LedgerEntryType.QUARANTINE_ENTERED, severity=1.0)
        assert led.compute_risk_profile("a").recommendation == "probation"
        for _ in range(5):
            led.record("a", LedgerEntryType.SLASH_CASCADED, severity=1.0)
        p = led.compute_risk_profile("a")
        assert p.risk_score == 1.0 and p.recommendation == "deny"
        ok, why = led.should_admit("a")
        assert not ok and "exceeds threshold" in why

    def test_clean_sessions_reduce_risk(self):
        led = LiabilityLedger()
        led.record("a", LedgerEntryType.FAULT_ATTRIBUTED, severity=0.8)
        led.record("a", LedgerEntryType.CLEAN_SESSION)
        led.record("a", LedgerEntryType.CLEAN_SESSION)
        p = led.compute_risk_profile("a")
        assert p.risk_score == 0.0 and p.fault_score_avg == 0.8 and p.clean_session_count == 2
        assert led.should_admit("a") == (True, "admit")

    def test_queries(self):
        led = LiabilityLedger()
        led.record("a", LedgerEntryType.VOUCH_GIVEN, session_id="s", related_agent="b")
        led.record("b", LedgerEntryType.VOUCH_RECEIVED, session_id="s", related_agent="a")
        assert led.total_entries == 2 and sorted(led.tracked_agents) == ["a", "b"]
        assert led.get_agent_history("a")[0].related_agent == "b"
