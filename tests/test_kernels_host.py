"""Host twins of the batched kernels (K01–K22) against the Python engines of the
``hypervisor`` package, which are themselves pinned to the reference behaviour.

The host twins run the exact ``__host__ __device__`` element bodies compiled
into the gfx950 kernels; ``tests/test_gpu_kernels.py`` checks device == host.
"""

from __future__ import annotations

import hashlib
import random
from datetime import datetime, timedelta, timezone

import pytest
import torch

from agent_hypervisor_amd.ops import audit as A
from agent_hypervisor_amd.ops import ledger as L
from agent_hypervisor_amd.ops import liability as LI
from agent_hypervisor_amd.ops import rings as R
from agent_hypervisor_amd.ops import saga as SG
from agent_hypervisor_amd.ops import security as SEC
from agent_hypervisor_amd.ops import session as SE
from hypervisor import _clock
from hypervisor.models import ActionDescriptor, ExecutionRing, ReversibilityLevel

f64, u8, i32, i64 = torch.float64, torch.uint8, torch.int32, torch.int64
T0 = datetime(2026, 1, 1, tzinfo=timezone.utc)


# ----------------------------------------------------------------- rings K01/K02


def test_ring_gate_matches_from_sigma_eff():
    rng = random.Random(1)
    sig = [rng.random() for _ in range(500)] + [0.0, 0.6, 0.95, 0.96, 1.0, 0.5999999, 0.9500001]
    cons = [rng.random() < 0.5 for _ in sig]
    out = R.ring_gate(torch.tensor(sig, dtype=f64), torch.tensor(cons, dtype=u8)).tolist()
    assert out == [ExecutionRing.from_sigma_eff(s, c).value for s, c in zip(sig, cons)]
    out0 = R.ring_gate(torch.tensor(sig, dtype=f64)).tolist()
    assert out0 == [ExecutionRing.from_sigma_eff(s, False).value for s in sig]


def test_ring_check_matches_enforcer():
    from hypervisor.rings.enforcer import RingEnforcer

    enf = RingEnforcer()
    rng = random.Random(2)
    rows = []
    for _ in range(2000):
        rev = rng.choice(list(ReversibilityLevel))
        act = ActionDescriptor(
            action_id="a", name="a", execute_api="/x", undo_api=None,
            reversibility=rev, is_read_only=rng.random() < 0.3, is_admin=rng.random() < 0.2,
        )
        rows.append((rng.randint(0, 3), act, rng.choice([rng.random(), 0.6, 0.95, 0.97]),
                     rng.random() < 0.5, rng.random() < 0.5))
    flags = [R.action_flags(a.is_admin, a.is_read_only, a.reversibility == ReversibilityLevel.NONE) for _, a,
             *_ in rows]
    req, reason = R.ring_check(
        torch.tensor([r[0] for r in rows], dtype=u8), torch.tensor(flags, dtype=u8),
        torch.tensor([r[2] for r in rows], dtype=f64), torch.tensor([r[3] for r in rows], dtype=u8),
        torch.tensor([r[4] for r in rows], dtype=u8),
    )
    for k, (ring, act, s, c, w) in enumerate(rows):
        res = enf.check(ExecutionRing(ring), act, s, c, w)
        assert req[k].item() == act.required_ring.value
        assert (reason[k].item() == 0) == res.allowed
        assert reason[k].item() == enf.check_code(ring, act.required_ring.value, s, c, w)


# ------------------------------------------------------------ liability K03–K07


def _random_vouch_world(n_sessions=40, seed=3, expiry=True):
    from hypervisor.liability.vouching import VouchingEngine, VouchingError

    rng = random.Random(seed)
    _clock.set_clock(lambda: T0)
    ve = VouchingEngine()
    sids, parts, sigmas = [], [], []
    for s in range(n_sessions):
        sid = f"s{s}"
        n = rng.randint(2, 16)
        p = [f"did:{s}:{k}" for k in range(n)]
        sg = {d: rng.uniform(0.3, 1.0) for d in p}
        for _ in range(rng.randint(0, 30)):
            a, b = rng.sample(p, 2)
            exp = None
            if expiry and rng.random() < 0.2:
                exp = T0 + timedelta(seconds=rng.choice([-5, 5]))
            try:
                ve.vouch(a, b, sid, sg[a], bond_pct=rng.choice([None, 0.1, 0.3, 0.5]), expiry=exp)
            except VouchingError:
                pass
        sids.append(sid)
        parts.append(p)
        sigmas.append(sg)
    return ve, sids, parts, sigmas


def test_sigma_eff_exact_and_mfma_tiles_match_vouching_engine():
    ve, sids, parts, sigmas = _random_vouch_world()
    now_us = _clock.to_us(T0)
    vb = LI.from_engine(ve, sids, parts)
    S = len(sids)
    sigma = torch.zeros((S, 16), dtype=f64)
    for s, p in enumerate(parts):
        for k, d in enumerate(p):
            sigma[s, k] = sigmas[s][d]
    omega = torch.tensor([0.1 + 0.05 * (s % 10) for s in range(S)], dtype=f64)
    exact = LI.sigma_eff_exact(vb, sigma, omega, now_us)
    tiles = LI.build_tiles(vb, now_us)
    se, expo, bonded_in = LI.bond_tiles(tiles, sigma, omega)
    for s, (sid, p) in enumerate(zip(sids, parts)):
        for k, d in enumerate(p):
            want = ve.compute_sigma_eff(d, sid, sigmas[s][d], omega[s].item())
            assert exact[s, k].item() == want  # bit parity (creation order)
            assert se[s, k].item() == pytest.approx(want, abs=1e-12)
            assert expo[s, k].item() == pytest.approx(ve.get_total_exposure(d, sid), abs=1e-12)


def test_vouch_admit_matches_engine_sequence():
    from hypervisor.liability.vouching import VouchingEngine, VouchingError

    rng = random.Random(4)
    _clock.set_clock(lambda: T0)
    now_us = _clock.to_us(T0)
    S = 30
    ve = VouchingEngine()
    parts = [[f"d{s}:{k}" for k in range(rng.randint(3, 16))] for s in range(S)]
    sig = [{d: rng.uniform(0.3, 1.0) for d in p} for p in parts]
    # requests per session, admitted sequentially by the Python engine
    reqs = []
    for s in range(S):
        reqs.append([(*rng.sample(range(len(parts[s])), 2), rng.choice([0.1, 0.25, 0.4])) for _ in range(25)])
        if rng.random() < 0.3:
            reqs[-1].append((0, 0, 0.2))  # self-vouch
    want_code, want_bonded = [], []
    for s in range(S):
        for v, e, pct in reqs[s]:
            vd, ed = parts[s][v], parts[s][e]
            try:
                rec = ve.vouch(vd, ed, f"s{s}", sig[s][vd], bond_pct=pct)
                want_code.append(LI.ADMIT_OK)
                want_bonded.append(rec.bonded_amount)
            except VouchingError as exc:
                msg = str(exc)
                code = (LI.ADMIT_SELF if "yourself" in msg else LI.ADMIT_LOW_SIGMA if "below minimum" in msg
                        else LI.ADMIT_CYCLE if "Circular" in msg else LI.ADMIT_EXPOSURE)
                want_code.append(code)
                want_bonded.append(0.0)
    empty = LI.VouchBatch(torch.zeros(S + 1, dtype=i32), *(torch.zeros(0, dtype=d) for d in (u8, u8, f64, u8, i64,
                                                                                             i64)))
    r_off = [0]
    for s in range(S):
        r_off.append(r_off[-1] + len(reqs[s]))
    flat = [(s, *q) for s in range(S) for q in reqs[s]]
    code, bonded = LI.vouch_admit(
        empty, torch.tensor(r_off, dtype=i32), torch.tensor([q[1] for q in flat], dtype=u8),
        torch.tensor([q[2] for q in flat], dtype=u8),
        torch.tensor([sig[q[0]][parts[q[0]][q[1]]] for q in flat], dtype=f64),
        torch.tensor([q[3] for q in flat], dtype=f64), now_us,
    )
    assert code.tolist() == want_code
    assert bonded.tolist() == want_bonded


@pytest.mark.parametrize("clip_cap", [64, 1])
def test_slash_cascade_matches_slashing_engine(clip_cap):
    """clip_cap=1: records are truncated, but scores, releases and the cascade
    (which re-reads every clip) still equal SlashingEngine."""
    from hypervisor.liability.slashing import SlashingEngine

    ve, sids, parts, sigmas = _random_vouch_world(n_sessions=60, seed=5, expiry=False)
    now_us = _clock.to_us(T0)
    vb = LI.from_engine(ve, sids, parts)
    S = len(sids)
    rng = random.Random(6)
    targets = [rng.randrange(len(p)) for p in parts]
    omega = torch.tensor([rng.choice([0.5, 0.9, 0.99]) for _ in range(S)], dtype=f64)
    scores = torch.full((S, 16), float("nan"), dtype=f64)
    py_scores = []
    for s, p in enumerate(parts):
        d = {}
        for k, did in enumerate(p):
            if rng.random() < 0.9:
                d[did] = sigmas[s][did]
                scores[s, k] = sigmas[s][did]
        py_scores.append(d)
    out = LI.slash(vb, torch.tensor(targets, dtype=u8), omega, scores, now_us, clip_cap=clip_cap)
    se = SlashingEngine(ve)
    for s, (sid, p) in enumerate(zip(sids, parts)):
        before = len(se.history)
        se.slash(p[targets[s]], sid, 0.5, omega[s].item(), "t", py_scores[s])
        # flatten clip records in history order of the clips themselves
        res = se.history[before:]
        n = out.clip_count[s].item()
        assert n == sum(len(r.voucher_clips) for r in res)
        for k, did in enumerate(p):
            if did in py_scores[s]:
                assert out.scores[s, k].item() == py_scores[s][did]
            else:
                assert torch.isnan(out.scores[s, k])
        if n > clip_cap:
            assert out.truncated[s]
            continue
        got = {(p[out.clip_voucher[s, c].item()], out.clip_before[s, c].item(), out.clip_after[s, c].item())
               for c in range(n)}
        want = {(c.voucher_did, c.sigma_before, c.sigma_after) for r in res for c in r.voucher_clips}
        assert got == want
    # released edges mirror the engine's bonds
    vb2 = LI.from_engine(ve, sids, parts)
    assert vb.active.tolist() == vb2.active.tolist()


def test_fused_slash_sigma_eff_matches_engines():
    """K06+K03 fused: σ_eff over the post-slash bonds equals, bit for bit, the
    separate sigma_eff pass and VouchingEngine.compute_sigma_eff after
    SlashingEngine.slash; storm subsets (target 255) get σ_eff too."""
    from hypervisor.liability.slashing import SlashingEngine

    ve, sids, parts, sigmas = _random_vouch_world(n_sessions=50, seed=15, expiry=False)
    now_us = _clock.to_us(T0)
    vb = LI.from_engine(ve, sids, parts)
    vb_sep = LI.from_engine(ve, sids, parts)
    S = len(sids)
    rng = random.Random(16)
    targets = [rng.randrange(len(p)) if s % 3 else 255 for s, p in enumerate(parts)]
    omega = torch.tensor([rng.choice([0.3, 0.9]) for _ in range(S)], dtype=f64)
    scores = torch.full((S, 16), float("nan"), dtype=f64)
    py_scores = []
    for s, p in enumerate(parts):
        d = {}
        for k, did in enumerate(p):
            d[did] = sigmas[s][did]
            scores[s, k] = sigmas[s][did]
        py_scores.append(d)
    tgt = torch.tensor(targets, dtype=u8)
    fused = LI.slash(vb, tgt, omega, scores.clone(), now_us, with_sigma_eff=True)
    sep = LI.slash(vb_sep, tgt, omega, scores.clone(), now_us)
    assert torch.equal(fused.sigma_eff, LI.sigma_eff_exact(vb_sep, sep.scores, omega, now_us))
    se = SlashingEngine(ve)
    for s, (sid, p) in enumerate(zip(sids, parts)):
        if targets[s] != 255:
            se.slash(p[targets[s]], sid, 0.5, omega[s].item(), "t", py_scores[s])
        for k, did in enumerate(p):
            want = ve.compute_sigma_eff(did, sid, py_scores[s][did], omega[s].item())
            assert fused.sigma_eff[s, k].item() == want


def test_release_bonds_matches_release_session_bonds():
    ve, sids, parts, _ = _random_vouch_world(n_sessions=20, seed=7)
    now_us = _clock.to_us(T0)
    vb = LI.from_engine(ve, sids, parts)
    got = LI.release_bonds(vb, now_us).tolist()
    want = [ve.release_session_bonds(s) for s in sids]
    assert got == want
    assert int(vb.active.sum()) == 0


# ------------------------------------------------------------------- audit K09–K12


def test_hash_many_matches_hashlib():
    rng = random.Random(8)
    msgs = [bytes(rng.randrange(256) for _ in range(n)) for n in
            [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4096] + [rng.randrange(300) for _ in range(50)]]
    data, offs = A.pack_bytes(msgs)
    assert A.digests_to_hex(A.sha256_many(data, offs)) == [hashlib.sha256(m).hexdigest() for m in msgs]
    contents = ["hello", "", "ünïcødé ✓", "x" * 300]
    assert A.content_hashes(contents) == [hashlib.sha256(c.encode()).hexdigest() for c in contents]
    from hypervisor.saga.checkpoint import SemanticCheckpoint

    assert A.goal_hashes(["g1", "goal two"], ["s1", "step-2"]) == [
        SemanticCheckpoint.compute_goal_hash("g1", "s1"), SemanticCheckpoint.compute_goal_hash("goal two", "step-2")]


def _delta_engines(n=12, seed=9):
    from hypervisor.audit.delta import DeltaEngine, VFSChange

    rng = random.Random(seed)
    engines = []
    for s in range(n):
        de = DeltaEngine(f"session:{s}")
        for t in range(rng.randint(0, 9)):
            de.capture(f"did:a{t % 3}", [VFSChange(f"/f{t}", "add", f"h{t}")])
        engines.append(de)
    return engines


def test_chain_hashes_rederive_delta_engine_chains():
    engines = _delta_engines(seed=21)
    packed = A.pack_chains([de.deltas for de in engines])
    got = A.digests_to_hex(A.chain_hashes(packed))
    want = [d.delta_hash for de in engines for d in de.deltas]
    assert got == want
    # continuing a chain from a seed parent: hash the tail of each chain alone
    tails = [de.deltas[2:] for de in engines if len(de.deltas) > 2]
    seeds = [de.deltas[1].delta_hash for de in engines if len(de.deltas) > 2]
    p2 = A.pack_chains(tails)
    got2 = A.chain_hashes(p2, A.hex_to_digests(seeds), torch.ones(len(seeds), dtype=u8))
    assert A.digests_to_hex(got2) == [d.delta_hash for t in tails for d in t]


def test_chain_hashes_midstate_split_every_prefix_length():
    """K08 midstate split: prefixes of 2-6 whole blocks at every arena alignment give
    the same digests as the single-phase pass and the scalar DeltaEngine."""
    from hypervisor.audit.delta import DeltaEngine, VFSChange

    rng = random.Random(5)
    chains = []
    for s in range(40):
        de = DeltaEngine(f"session:{s}")
        for t in range(rng.randint(1, 5)):
            did = "did:" + "x" * rng.randint(1, 200)  # prefixes of 2-6 whole blocks, odd offsets
            de.capture(did, [VFSChange(f"/p{t}", "add", "h" * rng.randint(0, 90))])
        chains.append(de.deltas)
    packed = A.pack_chains(chains)
    want = [d.delta_hash for c in chains for d in c]
    assert {int(x) % 4 for x in packed["pre_off"]} == {0, 1, 2, 3}
    assert len({int(x) // 64 for x in packed["pre_len"]}) >= 4
    split = A.chain_hashes(packed)
    assert torch.equal(split, A.chain_hashes(packed, midstate=False))
    assert A.digests_to_hex(split) == want


def test_merkle_roots_match_delta_engine():
    engines = _delta_engines()
    leaves, offs = [], [0]
    for de in engines:
        leaves += [d.delta_hash for d in de.deltas]
        offs.append(len(leaves))
    roots = A.merkle_roots(torch.tensor(offs, dtype=i32), A.hex_to_digests(leaves))
    for de, h in zip(engines, A.digests_to_hex(roots)):
        want = de.compute_merkle_root()
        assert h == (want if want is not None else "0" * 64)


def test_verify_chains_detects_tampering_without_mutating():
    engines = _delta_engines(seed=10)
    packed = A.pack_delta_engines(engines)
    dok, cok = A.verify_chains(*packed)
    assert all(dok.tolist()) and all(cok.tolist())
    # tamper one delta's stored hash and another chain's parent link
    victims = [k for k, de in enumerate(engines) if len(de.deltas) >= 2][:2]
    engines[victims[0]].deltas[1].delta_hash = "f" * 64
    engines[victims[1]].deltas[1].parent_hash = "0" * 64
    data, offs, stored, parent, has_parent, chain_offs = A.pack_delta_engines(engines)
    stored_before = stored.clone()
    dok, cok = A.verify_chains(data, offs, stored, parent, has_parent, chain_offs)
    assert torch.equal(stored, stored_before)
    for k, de in enumerate(engines):
        assert bool(cok[k]) == (k not in victims)


# ------------------------------------------------------------------- saga K13–K15


@pytest.mark.parametrize("saga", [False, True])
def test_fsm_matches_state_machine(saga):
    from hypervisor.saga.state_machine import Saga, SagaState, SagaStateError, SagaStep, StepState

    enum = SagaState if saga else StepState
    states = list(enum)
    pairs = [(a, b) for a in states for b in states]
    st = torch.tensor([SG.SAGA[a.value] if saga else SG.STEP[a.value] for a, _ in pairs], dtype=u8)
    tg = torch.tensor([SG.SAGA[b.value] if saga else SG.STEP[b.value] for _, b in pairs], dtype=u8)
    started = torch.zeros(len(pairs), dtype=i64)
    completed = torch.zeros(len(pairs), dtype=i64)
    ok = SG.transition(st, tg, 77, saga=saga, started_us=None if saga else started, completed_us=completed)
    for k, (a, b) in enumerate(pairs):
        obj = Saga(saga_id="x", session_id="s") if saga else SagaStep(step_id="x", action_id="a", agent_did="d",
                                                                     execute_api="/e")
        obj.state = a
        try:
            obj.transition(b)
            allowed = True
        except SagaStateError:
            allowed = False
        assert bool(ok[k]) == allowed, (a, b)
        if allowed:
            assert (completed[k].item() == 77) == (obj.completed_at is not None)
            if not saga:
                assert (started[k].item() == 77) == (obj.started_at is not None)


def test_fanout_policy_matches_orchestrator_rule():
    from hypervisor.saga.fan_out import FanOutPolicy, policy_satisfied

    rng = random.Random(11)
    groups = [(rng.choice(list(FanOutPolicy)), [rng.random() < 0.5 for _ in range(rng.randint(0, 9))])
              for _ in range(300)]
    offs = [0]
    for _, b in groups:
        offs.append(offs[-1] + len(b))
    sat, cnt, comp = SG.fanout_policy(
        torch.tensor(offs, dtype=i32), torch.tensor([SG.POLICY[p.value] for p, _ in groups], dtype=u8),
        torch.tensor([x for _, b in groups for x in b], dtype=u8),
    )
    for g, (p, b) in enumerate(groups):
        want = policy_satisfied(p, sum(b), len(b))
        assert bool(sat[g]) == want and cnt[g].item() == sum(b)
        assert comp[offs[g]:offs[g + 1]].tolist() == [int(x and not want) for x in b]


def test_compensation_plan_reverse_committed_order():
    st = torch.tensor([[2, 2, 6, 0], [2, 2, 2, 2]], dtype=u8)
    undo = torch.tensor([[1, 0, 1, 1], [1, 1, 1, 1]], dtype=torch.bool)
    order = SG.compensation_plan(st, undo, 5)
    assert order.tolist() == [[1, 0, -1, -1], [3, 2, 1, 0]]
    assert st.tolist() == [[3, 5, 6, 0], [3, 3, 3, 3]]


# --------------------------------------------------------------- security K16–K18


def test_breach_window_matches_detector():
    from hypervisor.rings.breach_detector import RingBreachDetector

    rng = random.Random(12)
    n, steps = 12, 120
    det = RingBreachDetector()
    prof = SEC.BreachProfiles.allocate(n, cap=1000)
    t = T0
    for step in range(steps):
        t = t + timedelta(seconds=rng.choice([0.5, 1, 3, 20]))
        _clock.set_clock(lambda: t)
        agent_ring = [rng.choice([1, 2, 3]) for _ in range(n)]
        called = [rng.choice([0, 1, 2, 3]) for _ in range(n)]
        sev, rate, hits, ev, _ = SEC.breach_record(
            prof, torch.full((n,), _clock.to_us(t), dtype=i64), torch.tensor(agent_ring, dtype=u8),
            torch.tensor(called, dtype=u8),
        )
        for p in range(n):
            e = det.record_call(f"a{p}", "s", ExecutionRing(agent_ring[p]), ExecutionRing(called[p]))
            assert bool(ev[p]) == (e is not None), (step, p)
            if e is not None:
                assert rate[p].item() == e.anomaly_score
                assert L.SEVERITY[sev[p].item()] == e.severity.value
    for p in range(n):
        st = det.get_agent_stats(f"a{p}", "s")
        assert prof.count[p].item() == st["window_calls"] and prof.total[p].item() == st["total_calls"]


def test_token_bucket_matches_rate_limiter_bucket():
    from hypervisor.security.rate_limiter import TokenBucket

    rng = random.Random(13)
    n = 16
    t = T0
    _clock.set_clock(lambda: t)
    caps = [rng.choice([10.0, 40.0, 200.0]) for _ in range(n)]
    rates = [rng.choice([5.0, 20.0, 100.0]) for _ in range(n)]
    buckets = [TokenBucket(capacity=c, tokens=c, refill_rate=r) for c, r in zip(caps, rates)]
    tokens = torch.tensor(caps, dtype=f64)
    last = torch.full((n,), _clock.to_us(t), dtype=i64)
    for _ in range(200):
        t = t + timedelta(microseconds=rng.choice([0, 1000, 50_000, 700_000]))
        _clock.set_clock(lambda: t)
        cost = [rng.choice([1.0, 2.0, 5.0]) for _ in range(n)]
        ok = SEC.token_bucket(tokens, last, torch.tensor(caps, dtype=f64), torch.tensor(rates, dtype=f64),
                              torch.tensor(cost, dtype=f64), _clock.to_us(t))
        for i in range(n):
            assert bool(ok[i]) == buckets[i].consume(cost[i])
            assert tokens[i].item() == pytest.approx(buckets[i].tokens, rel=1e-12, abs=1e-9)


def test_expiry_tick_strictly_before_now():
    active = torch.tensor([1, 1, 1, 0, 1], dtype=u8)
    exp = torch.tensor([10, 11, -1, 5, 9], dtype=i64)
    rel = torch.zeros(5, dtype=i64)
    out = SEC.expiry_tick(active, exp, 10, rel)
    assert out.tolist() == [0, 0, 0, 0, 1]
    assert active.tolist() == [1, 1, 1, 0, 0] and rel.tolist() == [0, 0, 0, 0, 10]


# ------------------------------------------------------------- ledger K21 / K22


def test_ledger_risk_matches_liability_ledger():
    from hypervisor.liability.ledger import LedgerEntryType, LiabilityLedger

    rng = random.Random(14)
    led = LiabilityLedger()
    agents = [f"a{k}" for k in range(50)]
    types = list(LedgerEntryType)
    offs, ty, sv = [0], [], []
    for a in agents:
        for _ in range(rng.randint(0, 12)):
            t = rng.choice(types)
            s = rng.choice([0.0, 0.2, 0.5, 0.9, rng.random()])
            led.record(a, t, severity=s)
            ty.append(L.LEDGER_CODE[t.value])
            sv.append(s)
        offs.append(len(ty))
    out = L.risk_profiles(torch.tensor(offs, dtype=i32), torch.tensor(ty, dtype=u8), torch.tensor(sv, dtype=f64))
    for g, a in enumerate(agents):
        p = led.compute_risk_profile(a)
        assert round(out["risk"][g].item(), 4) == p.risk_score
        assert L.RECOMMENDATION[out["recommendation"][g].item()] == p.recommendation
        assert out["slash_count"][g].item() == p.slash_count
        assert out["quarantine_count"][g].item() == p.quarantine_count
        assert out["clean_count"][g].item() == p.clean_session_count
        assert round(out["fault_avg"][g].item(), 4) == p.fault_score_avg


def test_drift_severity_matches_cmvk():
    from hypervisor.integrations.cmvk_adapter import DriftThresholds, classify_drift

    rng = random.Random(15)
    xs = [0.0, 0.1, 0.15, 0.2, 0.3, 0.49, 0.5, 0.74, 0.75, 1.0] + [rng.random() for _ in range(50)]
    out = L.drift_severity(torch.tensor(xs, dtype=f64)).tolist()
    assert [L.SEVERITY[k] for k in out] == [classify_drift(x, DriftThresholds()).value for x in xs]


def test_attribution_raw_matches_causal_attributor():
    from hypervisor.liability.attribution import CausalAttributor

    rng = random.Random(16)
    ca = CausalAttributor()
    node_offs, agent_offs, aon, succ, root, rw = [0], [0], [], [], [], []
    want = []
    for _ in range(40):
        agents = [f"a{k}" for k in range(rng.randint(1, 6))]
        actions = {a: [{"action_id": f"x{rng.randint(0, 3)}", "step_id": f"st{rng.randint(0, 4)}",
                        "success": rng.random() < 0.6} for _ in range(rng.randint(1, 4))] for a in agents}
        fa, fs = rng.choice(agents), f"st{rng.randint(0, 4)}"
        weights = {"x0": 0.9, "x1": 0.1}
        nodes = ca.build_causal_dag(actions, fs, fa)
        raw = ca.raw_scores(nodes, agents, weights)
        want += [raw[a] for a in agents]
        idx = {a: k for k, a in enumerate(agents)}
        for nd in nodes:
            aon.append(idx[nd.agent_did])
            succ.append(int(nd.success))
            root.append(int(nd.is_root_cause))
            rw.append(weights.get(nd.action_id, 0.5))
        node_offs.append(len(aon))
        agent_offs.append(agent_offs[-1] + len(agents))
    got = L.attribution_raw(torch.tensor(node_offs, dtype=i32), torch.tensor(agent_offs, dtype=i32),
                            torch.tensor(aon, dtype=i32), torch.tensor(succ, dtype=u8),
                            torch.tensor(root, dtype=u8), torch.tensor(rw, dtype=f64))
    assert got.tolist() == want


# ------------------------------------------------------------ sessions K19 / K20


def test_vector_clocks_match_manager():
    from hypervisor.session.vector_clock import CausalViolationError, VectorClockManager

    rng = random.Random(17)
    G, P, Ag = 8, 5, 6
    mgrs = [VectorClockManager() for _ in range(G)]
    offs, ops, paths, agents, cols, want = [0], [], [], [], [], []
    for g in range(G):
        for _ in range(60):
            op, p, a = rng.random() < 0.5, rng.randrange(P), rng.randrange(Ag)
            if op:
                try:
                    mgrs[g].write(f"/p{p}", f"a{a}")
                    want.append(1)
                except CausalViolationError:
                    want.append(0)
            else:
                mgrs[g].read(f"/p{p}", f"a{a}")
                want.append(1)
            ops.append(int(op))
            paths.append(g * P + p)
            agents.append(g * Ag + a)
            cols.append(a)
        offs.append(len(ops))
    pc = torch.zeros((G * P, Ag), dtype=i32)
    ac = torch.zeros((G * Ag, Ag), dtype=i32)
    ok = SE.vector_clock_ops(torch.tensor(offs, dtype=i32), torch.tensor(ops, dtype=u8),
                             torch.tensor(paths, dtype=i32), torch.tensor(agents, dtype=i32),
                             torch.tensor(cols, dtype=i32), pc, ac)
    assert ok.tolist() == want
    for g in range(G):
        for p in range(P):
            c = mgrs[g].get_path_clock(f"/p{p}").clocks
            assert pc[g * P + p].tolist() == [c.get(f"a{a}", 0) for a in range(Ag)]


def test_lock_conflicts_match_intent_lock_manager():
    from hypervisor.session.intent_locks import IntentLockManager, LockContentionError, LockIntent

    rng = random.Random(18)
    mgr = IntentLockManager()
    R_, intents = 6, list(LockIntent)
    for _ in range(30):
        try:
            mgr.acquire(f"a{rng.randrange(5)}", "s", f"/r{rng.randrange(R_)}", rng.choice(intents))
        except LockContentionError:
            pass
    res_offs, la, li = [0], [], []
    for r in range(R_):
        for l in mgr.get_resource_locks(f"/r{r}"):
            la.append(int(l.agent_did[1:]))
            li.append(SE.LOCK_INTENT[l.intent.value])
        res_offs.append(len(la))
    reqs = [(rng.randrange(R_), rng.randrange(6), rng.choice(intents)) for _ in range(200)]
    got = SE.lock_conflicts(torch.tensor(res_offs, dtype=i32), torch.tensor(la, dtype=i32),
                            torch.tensor(li, dtype=u8), torch.tensor([q[0] for q in reqs], dtype=i32),
                            torch.tensor([q[1] for q in reqs], dtype=i32),
                            torch.tensor([SE.LOCK_INTENT[q[2].value] for q in reqs], dtype=u8))
    for k, (r, a, it) in enumerate(reqs):
        assert got[k].item() == len(mgr._check_contention(f"/r{r}", f"a{a}", it))


def test_bond_fused_host_twin_matches_creation_order():
    """Host twin of the fused K03/K04 kernel: σ_eff bit-identical to the
    creation-order CSR path, exposure equal to the dense-tile pair."""
    import random as _r

    from agent_hypervisor_amd.ops import liability as LI

    rng = _r.Random(3)
    S = 300
    offs, vr, ve, bd, ac, ex = [0], [], [], [], [], []
    for _ in range(S):
        for _ in range(rng.randint(0, 30)):
            a, b = rng.sample(range(16), 2)
            vr.append(a), ve.append(b), bd.append(rng.uniform(0, 0.4))
            ac.append(int(rng.random() < 0.9)), ex.append(rng.choice([-1, 50, 150]))
        offs.append(len(vr))
    vb = LI.VouchBatch(torch.tensor(offs, dtype=torch.int32), torch.tensor(vr, dtype=torch.uint8),
                       torch.tensor(ve, dtype=torch.uint8), torch.tensor(bd, dtype=torch.float64),
                       torch.tensor(ac, dtype=torch.uint8), torch.tensor(ex, dtype=torch.int64),
                       torch.zeros(len(vr), dtype=torch.int64))
    sigma = torch.rand((S, 16), dtype=torch.float64)
    omega = torch.rand(S, dtype=torch.float64)
    se, expo, bi = LI.bond_fused(vb, sigma, omega, 100, bonded_in=True)
    assert torch.equal(se, LI.sigma_eff_exact(vb, sigma, omega, 100))
    t_se, t_ex, t_bi = LI.bond_tiles(LI.build_tiles(vb, 100), sigma, omega)
    torch.testing.assert_close(expo, t_ex, rtol=0, atol=1e-12)
    torch.testing.assert_close(bi, t_bi, rtol=0, atol=1e-12)


def test_render_rows_stamps_and_hex():
    tmpl = torch.frombuffer(bytearray(b'{"id": "#######", "us": "......", "h": "' + b"?" * 8 + b'"}'), dtype=u8)
    L = tmpl.numel()
    out = torch.zeros(5 * L, dtype=u8)
    src = torch.arange(5 * 4, dtype=torch.int32).reshape(5, 4)  # 16 bytes per row
    ids = torch.tensor([4, 0, 2], dtype=torch.int64)
    tb = bytes(tmpl.tolist())
    p_id, p_us, p_h = tb.index(b"#"), tb.index(b"."), tb.index(b"?")
    A.render_rows(out, tmpl, ids, stamps=[(p_id, 7, 0, 0), (p_us, 6, 3, 998)], hex_field=(p_h, src, 4))
    rows = out.view(5, L)
    for i in ids.tolist():
        want = bytearray(tmpl.tolist())
        want[p_id:p_id + 7] = f"{i:07d}".encode()
        want[p_us:p_us + 6] = f"{i % 3 + 998:06d}".encode()
        want[p_h:p_h + 8] = src[i].contiguous().view(u8)[:4].numpy().tobytes().hex().encode()
        assert bytes(rows[i].tolist()) == bytes(want)
    assert int(rows[1].sum()) == 0 and int(rows[3].sum()) == 0  # rows not listed stay untouched
    with pytest.raises(ValueError):
        A.render_rows(out, tmpl, torch.tensor([5]), stamps=[(p_id, 7, 0, 0)])


def test_agent_gather_is_session_order_sum_of_voucher_rows():
    """X01 input without atomics: AgentIndex lists each agent's voucher slots in
    session order, and the segmented reduction adds their exposure rows in that
    order (members that vouch for nobody carry 0 and are skipped)."""
    import random

    rng = random.Random(4)
    S, A = 200, 60
    offs, vr, ve = [0], [], []
    for _ in range(S):
        for _ in range(rng.randint(0, 12)):
            a, b = rng.sample(range(16), 2)
            vr.append(a)
            ve.append(b)
        offs.append(len(vr))
    E = len(vr)
    vb = LI.VouchBatch(torch.tensor(offs, dtype=torch.int32), torch.tensor(vr, dtype=torch.uint8),
                       torch.tensor(ve, dtype=torch.uint8), torch.rand(E, dtype=torch.float64),
                       torch.ones(E, dtype=torch.uint8), torch.full((E,), -1, dtype=torch.int64),
                       torch.zeros(E, dtype=torch.int64))
    members = torch.randint(0, A, (S, 16), generator=torch.Generator().manual_seed(2))
    sigma = torch.rand((S, 16), dtype=torch.float64)
    omega = torch.rand(S, dtype=torch.float64)
    idx = LI.agent_index(vb, members, A)
    out = torch.empty(A, dtype=torch.float64)
    _, ex, _ = LI.bond_fused(vb, sigma, omega, 0, agent_exposure=out, agent_idx=idx)
    want = [0.0] * A
    for s in range(S):
        vouchers = sorted({vr[k] for k in range(offs[s], offs[s + 1])})
        for j in vouchers:
            want[int(members[s, j])] += float(ex[s, j])
    assert out.tolist() == want
    legacy = torch.zeros(A, dtype=torch.float64)  # the atomic form adds every member's row
    LI.bond_fused(vb, sigma, omega, 0, members=members, agent_exposure=legacy)
    torch.testing.assert_close(legacy, out, rtol=1e-12, atol=1e-15)


def test_slash_touched_list_is_sessions_with_clips():
    import random

    rng = random.Random(21)
    S = 300
    offs, vr, ve = [0], [], []
    for _ in range(S):
        for _ in range(rng.randint(0, 20)):
            a, b = rng.sample(range(16), 2)
            vr.append(a)
            ve.append(b)
        offs.append(len(vr))
    E = len(vr)
    vb = LI.VouchBatch(torch.tensor(offs, dtype=torch.int32), torch.tensor(vr, dtype=torch.uint8),
                       torch.tensor(ve, dtype=torch.uint8), torch.rand(E, dtype=torch.float64),
                       torch.ones(E, dtype=torch.uint8), torch.full((E,), -1, dtype=torch.int64),
                       torch.zeros(E, dtype=torch.int64))
    tgt = torch.randint(0, 16, (S,), dtype=torch.uint8)
    tgt[torch.rand(S) < 0.7] = 255
    out = LI.slash(vb, tgt, torch.full((S,), 0.9, dtype=torch.float64), torch.rand((S, 16), dtype=torch.float64),
                   5, with_touched=True)
    assert torch.equal(out.touched, torch.nonzero(out.clip_count > 0).flatten())
