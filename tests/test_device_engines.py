"""Device-resident governance engines vs the host Python engines.

Every test replays one random call stream (pinned clock) through the host
engine of the reference semantics and through ``Engine(device=...)`` — the
variant whose state lives in device columns and whose batched method is one
kernel launch (K16 breach, K17 buckets, K18 expiry, K22 ledger, K19 clocks,
K20 lock contention) — and compares every return value, event, error message
and stat.  ``cpu`` runs the kernels' host twins here; ``cuda`` the gfx950
kernels (``-m gpu``)."""

from __future__ import annotations

import random
from datetime import datetime, timedelta, timezone

import pytest

from hypervisor import _clock
from hypervisor.liability.ledger import LedgerEntryType, LiabilityLedger
from hypervisor.liability.quarantine import QuarantineManager, QuarantineReason
from hypervisor.models import ExecutionRing
from hypervisor.rings.breach_detector import RingBreachDetector
from hypervisor.rings.elevation import RingElevationManager
from hypervisor.security.rate_limiter import AgentRateLimiter, RateLimitExceeded
from hypervisor.session.intent_locks import IntentLockManager, LockIntent
from hypervisor.session.vector_clock import VectorClockManager

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
T0 = datetime(2026, 3, 1, tzinfo=timezone.utc)
R = list(ExecutionRing)


class Clock:
    def __init__(self) -> None:
        self.t = T0
        _clock.set_clock(lambda: self.t)

    def advance(self, seconds: float) -> None:
        self.t = self.t + timedelta(seconds=seconds)


def _dev(device):
    if device == "cuda":
        import torch

        if not torch.cuda.is_available():
            pytest.fail("GPU test selected but no HIP device is visible")
    return device


def _ev(e):
    if e is None:
        return None
    return (e.agent_did, e.session_id, e.severity, e.anomaly_score, e.call_count_window, e.actual_rate, e.details,
            e.timestamp)


@pytest.mark.parametrize("device", DEVICES)
def test_breach_detector_matches_host(device):
    rng = random.Random(1)
    clk = Clock()
    host, dev = RingBreachDetector(), RingBreachDetector(device=_dev(device), capacity=4, window_cap=1000)
    assert type(dev).__name__ == "DeviceRingBreachDetector"
    keys = [(f"did:a{i}", f"s{i % 3}") for i in range(24)]
    for step in range(60):
        clk.advance(rng.choice([0.2, 1, 3, 25]))
        calls = []
        for _ in range(rng.randint(1, 40)):  # repeated profiles inside one batch
            a, s = rng.choice(keys)
            calls.append((a, s, rng.choice(R[1:]), rng.choice(R)))
        he = host.record_calls_batch(calls)
        de = dev.record_calls_batch(calls)
        assert [_ev(e) for e in he] == [_ev(e) for e in de], step
        if step % 7 == 3:
            a, s = rng.choice(keys)
            host.reset_breaker(a, s)
            dev.reset_breaker(a, s)
        for a, s in keys[:8]:
            assert host.is_breaker_tripped(a, s) == dev.is_breaker_tripped(a, s)
            assert host.get_agent_stats(a, s) == dev.get_agent_stats(a, s)
    a, s = keys[0]
    assert _ev(host.record_call(a, s, R[3], R[0])) == _ev(dev.record_call(a, s, R[3], R[0]))
    assert host.breach_count == dev.breach_count > 0
    assert [_ev(e) for e in host.breach_history] == [_ev(e) for e in dev.breach_history]
    assert dev.get_agent_stats("nobody", "x") == host.get_agent_stats("nobody", "x")


@pytest.mark.parametrize("device", DEVICES)
def test_rate_limiter_matches_host(device):
    rng = random.Random(2)
    clk = Clock()
    host, dev = AgentRateLimiter(), AgentRateLimiter(device=_dev(device), capacity=2)
    keys = [(f"did:a{i}", f"s{i % 2}") for i in range(12)]
    ring_of = {k: rng.choice(R) for k in keys}
    for step in range(80):
        clk.advance(rng.choice([0.01, 0.1, 0.5, 2.0]))
        reqs = []
        for _ in range(rng.randint(1, 60)):
            k = rng.choice(keys)
            reqs.append((k[0], k[1], ring_of[k], rng.choice([1.0, 1.0, 2.5])))
        assert host.check_batch(reqs) == dev.check_batch(reqs), step
        if step % 9 == 4:
            k = rng.choice(keys)
            ring_of[k] = rng.choice(R)
            host.update_ring(k[0], k[1], ring_of[k])
            dev.update_ring(k[0], k[1], ring_of[k])
        for k in keys[:5]:
            hs, ds = host.get_stats(*k), dev.get_stats(*k)
            assert (hs is None) == (ds is None)
            if hs is not None:
                assert (hs.agent_did, hs.ring, hs.total_requests, hs.rejected_requests, hs.capacity) == \
                       (ds.agent_did, ds.ring, ds.total_requests, ds.rejected_requests, ds.capacity)
                assert hs.tokens_available == pytest.approx(ds.tokens_available, rel=0, abs=1e-9)
    # scalar check raises with the same message once the bucket is dry
    k = keys[0]
    msgs = []
    for eng in (host, dev):
        try:
            for _ in range(500):
                eng.check(k[0], k[1], ring_of[k])
        except RateLimitExceeded as e:
            msgs.append(str(e))
    assert len(msgs) == 2 and msgs[0] == msgs[1]
    assert host.tracked_agents == dev.tracked_agents


@pytest.mark.parametrize("device", DEVICES)
def test_quarantine_and_elevation_ticks_match_host(device):
    rng = random.Random(3)
    clk = Clock()
    hq, dq = QuarantineManager(), QuarantineManager(device=_dev(device), capacity=2)
    he, de = RingElevationManager(), RingElevationManager(device=device, capacity=2)
    agents = [f"did:q{i}" for i in range(10)]
    reasons = list(QuarantineReason)
    for step in range(50):
        clk.advance(rng.choice([1, 30, 120, 400]))
        qs = [(rng.choice(agents), "s", rng.choice(reasons), f"d{step}", rng.choice([None, 60, 600]))
              for _ in range(rng.randint(0, 4))]
        h_rec, d_rec = hq.quarantine_batch(qs), dq.quarantine_batch(qs)
        assert [(r.agent_did, r.details, r.expires_at) for r in h_rec] == \
               [(r.agent_did, r.details, r.expires_at) for r in d_rec]
        if step % 5 == 2:
            a = rng.choice(agents)
            assert (hq.release(a, "s") is None) == (dq.release(a, "s") is None)
        assert [(r.agent_did, r.released_at) for r in hq.tick()] == [(r.agent_did, r.released_at) for r in dq.tick()]
        assert [hq.is_quarantined(a, "s") for a in agents] == [dq.is_quarantined(a, "s") for a in agents]
        es = [(rng.choice(agents), "s", R[3], rng.choice(R[:3]), rng.choice([0, 30, 200, 5000]))
              for _ in range(rng.randint(0, 3))]
        hr, dr = he.request_elevation_batch(es), de.request_elevation_batch(es)
        assert [str(x) if isinstance(x, Exception) else (x.agent_did, x.expires_at) for x in hr] == \
               [str(x) if isinstance(x, Exception) else (x.agent_did, x.expires_at) for x in dr]
        if step % 6 == 1 and he.active_elevations:
            i = rng.randrange(len(he.active_elevations))
            he.revoke_elevation(he.active_elevations[i].elevation_id)
            de.revoke_elevation(de.active_elevations[i].elevation_id)
        assert [e.agent_did for e in he.tick()] == [e.agent_did for e in de.tick()]
        assert [e.agent_did for e in he.active_elevations] == [e.agent_did for e in de.active_elevations]
    assert hq.quarantine_count == dq.quarantine_count


@pytest.mark.parametrize("device", DEVICES)
def test_ledger_profiles_match_host(device):
    rng = random.Random(4)
    Clock()
    host, dev = LiabilityLedger(), LiabilityLedger(device=_dev(device), capacity=8)
    agents = [f"did:l{i}" for i in range(30)]
    types = list(LedgerEntryType)
    for _ in range(600):
        a, t, sev = rng.choice(agents), rng.choice(types), rng.choice([0.0, 0.2, 0.5, 0.9, 1.0, rng.random()])
        host.record(a, t, "s", sev)
        dev.record(a, t, "s", sev)
    ask = agents + ["did:unknown"]
    assert host.compute_risk_profiles(ask) == dev.compute_risk_profiles(ask)
    assert host.compute_risk_profile(agents[3]) == dev.compute_risk_profile(agents[3])
    assert host.should_admit(agents[5]) == dev.should_admit(agents[5])


@pytest.mark.parametrize("device", DEVICES)
def test_vector_clocks_match_host(device):
    rng = random.Random(5)
    host, dev = VectorClockManager(), VectorClockManager(device=_dev(device), capacity=2)
    agents = [f"did:v{i}" for i in range(9)]
    paths = [f"/p{i}" for i in range(7)]
    for step in range(40):
        ops = [(rng.choice(["read", "write", "write"]), rng.choice(paths), rng.choice(agents))
               for _ in range(rng.randint(1, 30))]
        assert host.apply_batch(ops) == dev.apply_batch(ops), step
        assert host.conflict_count == dev.conflict_count
    for p in paths:
        assert host.get_path_clock(p) == dev.get_path_clock(p)
    for a in agents:
        assert host.get_agent_clock(a) == dev.get_agent_clock(a)
    assert host.tracked_paths == dev.tracked_paths
    assert host.read(paths[0], agents[0]) == dev.read(paths[0], agents[0])
    assert host.write(paths[0], agents[0]) == dev.write(paths[0], agents[0])


@pytest.mark.parametrize("device", DEVICES)
def test_intent_locks_match_host(device):
    rng = random.Random(6)
    host = IntentLockManager(record_waits=True)
    dev = IntentLockManager(record_waits=True, device=_dev(device))
    agents = [f"did:k{i}" for i in range(6)]
    paths = [f"/r{i}" for i in range(5)]
    intents = list(LockIntent)

    def norm(x):
        return (type(x).__name__, str(x)) if isinstance(x, Exception) else (x.agent_did, x.resource_path, x.intent)

    for step in range(40):
        reqs = [(rng.choice(agents), "s", rng.choice(paths), rng.choice(intents)) for _ in range(rng.randint(1, 8))]
        hr, dr = host.acquire_batch(reqs), dev.acquire_batch(reqs)
        assert [norm(x) for x in hr] == [norm(x) for x in dr], step
        if step % 3 == 2:
            a = rng.choice(agents)
            assert host.release_agent_locks(a, "s") == dev.release_agent_locks(a, "s")
        assert host.active_lock_count == dev.active_lock_count
        assert sorted(host.contention_points) == sorted(dev.contention_points)


@pytest.mark.parametrize("device", DEVICES)
def test_ring_check_batch_matches_check(device):
    from hypervisor.models import ActionDescriptor, ReversibilityLevel
    from hypervisor.rings.enforcer import RingEnforcer

    rng = random.Random(7)
    enf = RingEnforcer()
    acts = [ActionDescriptor(action_id=f"a{i}", name="x", execute_api="/x", is_admin=rng.random() < 0.2,
                             is_read_only=rng.random() < 0.3, reversibility=rng.choice(list(ReversibilityLevel)))
            for i in range(300)]
    rings = [rng.choice(R) for _ in acts]
    sig = [rng.choice([0.0, 0.59, 0.6, 0.61, 0.94, 0.95, 0.96, rng.random()]) for _ in acts]
    cons = [rng.random() < 0.5 for _ in acts]
    wit = [rng.random() < 0.5 for _ in acts]
    got = enf.check_batch(rings, acts, sig, cons, wit, device=_dev(device))
    want = [enf.check(r, a, s, c, w) for r, a, s, c, w in zip(rings, acts, sig, cons, wit)]
    assert got == want


@pytest.mark.parametrize("device", DEVICES)
def test_attribution_batch_matches_attribute(device):
    from hypervisor.liability.attribution import CausalAttributor

    rng = random.Random(8)
    cases = []
    for c in range(40):
        agents = [f"did:x{j}" for j in range(rng.randint(1, 6))]
        acts = {a: [{"action_id": f"act{rng.randint(0, 5)}", "step_id": f"st{rng.randint(0, 4)}",
                     "success": rng.random() < 0.6} for _ in range(rng.randint(0, 5))] for a in agents}
        cases.append(dict(saga_id=f"saga{c}", session_id="s", agent_actions=acts,
                          failure_step_id=f"st{rng.randint(0, 4)}", failure_agent_did=rng.choice(agents),
                          risk_weights={f"act{k}": rng.random() for k in range(3)}))
    host, dev = CausalAttributor(), CausalAttributor()
    want = [host.attribute(**c) for c in cases]
    got = dev.attribute_batch(cases, device=_dev(device))

    def norm(r):
        return (r.saga_id, r.causal_chain_length, r.root_cause_agent,
                sorted((a.agent_did, a.liability_score, a.causal_contribution, a.is_direct_cause)
                       for a in r.attributions))

    assert [norm(r) for r in got] == [norm(r) for r in want]
    # unsorted too: the same ranking, ties included
    assert [[(a.agent_did, a.liability_score) for a in r.attributions] for r in got] == \
        [[(a.agent_did, a.liability_score) for a in r.attributions] for r in want]


@pytest.mark.parametrize("device", DEVICES)
def test_drift_batch_matches_classify(device):
    from hypervisor.integrations.cmvk_adapter import CMVKAdapter, classify_drift

    rng = random.Random(9)
    seen = []
    ad = CMVKAdapter(on_drift_detected=seen.append)
    scores = [rng.choice([0.0, 0.15, 0.3, 0.5, 0.75, 1.0, rng.random()]) for _ in range(500)]
    res = ad.record_drift_batch([f"did:d{i % 7}" for i in range(500)], ["s"] * 500, scores, device=_dev(device))
    assert [r.severity for r in res] == [classify_drift(s, ad.thresholds) for s in scores]
    assert ad.total_checks == 500 and ad.total_violations == len(seen) == sum(not r.passed for r in res)


@pytest.mark.parametrize("device", DEVICES)
def test_tensor_paths_match_host(device):
    """record_rows / check_rows (calls already on the device) vs the host engines."""
    import torch

    rng = random.Random(10)
    clk = Clock()
    hb, db = RingBreachDetector(), RingBreachDetector(device=_dev(device), capacity=8)
    hl, dl = AgentRateLimiter(), AgentRateLimiter(device=device, capacity=8)
    keys = [(f"did:t{i}", "s") for i in range(50)]
    ring_of = {k: rng.choice(R[1:]) for k in keys}
    brows = db.rows_for(keys)
    lrows = dl.rows_for([(a, s, ring_of[(a, s)]) for a, s in keys])
    hl_keys = keys  # the host creates buckets lazily on first check
    for step in range(30):
        clk.advance(rng.choice([0.05, 0.5, 3, 20]))
        pick = [rng.randrange(len(keys)) for _ in range(rng.randint(1, 200))]
        called = [rng.choice(R) for _ in pick]
        want = [hb.record_call(keys[i][0], keys[i][1], ring_of[keys[i]], c) for i, c in zip(pick, called)]
        idx = torch.tensor(pick, device=brows.device)
        got = db.record_rows(brows[idx], torch.tensor([ring_of[keys[i]].value for i in pick], dtype=torch.uint8,
                                                      device=brows.device),
                             torch.tensor([c.value for c in called], dtype=torch.uint8, device=brows.device))
        assert got["event"].cpu().tolist() == [int(e is not None) for e in want]
        costs = [rng.choice([1.0, 3.0]) for _ in pick]
        hw = [hl.try_check(hl_keys[i][0], hl_keys[i][1], ring_of[keys[i]], c) for i, c in zip(pick, costs)]
        ok = dl.check_rows(lrows[idx.to(lrows.device)], torch.tensor(costs, dtype=torch.float64,
                                                                      device=lrows.device))
        assert [bool(x) for x in ok.cpu().tolist()] == hw
    assert [_ev(e) for e in hb.breach_history] == [_ev(e) for e in db.breach_history]


@pytest.mark.parametrize("device", DEVICES)
def test_intent_lock_rows_match_sequential_acquire(device):
    """Tensor-native K20 (acquire_rows / release_rows over the device summaries)
    grants exactly the requests a sequential host manager grants, across
    interleaved batches, record-path acquires and releases of both kinds."""
    import torch

    from hypervisor.session.intent_locks import LockIntent

    rng = random.Random(13)
    dev = IntentLockManager(device=_dev(device))
    host = IntentLockManager()
    agents = [f"did:t{i}" for i in range(5)]
    paths = [f"/q{i}" for i in range(6)]
    kinds = list(LockIntent)
    held = []  # (path, intent, host lock) of row-path grants
    for step in range(25):
        batch = [(rng.choice(agents), rng.choice(paths), rng.choice(kinds)) for _ in range(rng.randint(1, 30))]
        want = []
        for a, p, k in batch:
            try:
                want.append(host.acquire(a, "s", p, k))
            except Exception:  # noqa: BLE001 - contention / deadlock: refused
                want.append(None)
        rows = torch.tensor([dev.resource_row(p) for _, p, _ in batch], dtype=torch.int32, device=_dev(device))
        ags = torch.tensor([dev.agent_row(a) for a, _, _ in batch], dtype=torch.int32, device=_dev(device))
        its = torch.tensor([{"read": 0, "write": 1, "exclusive": 2}[k.value] for _, _, k in batch],
                           dtype=torch.uint8, device=_dev(device))
        got = dev.acquire_rows(ags, rows, its).cpu().tolist()
        assert got == [int(w is not None) for w in want], step
        held += [(p, k, w) for (a, p, k), w in zip(batch, want) if w is not None]
        rng.shuffle(held)
        drop, held = held[: len(held) // 3], held[len(held) // 3:]
        for _, _, w in drop:
            host.release(w.lock_id)
        if drop:
            rel = dev.release_rows(
                torch.tensor([dev.agent_row(w.agent_did) for _, _, w in drop], dtype=torch.int32, device=_dev(device)),
                torch.tensor([dev.resource_row(p) for p, _, _ in drop], dtype=torch.int32, device=_dev(device)),
                torch.tensor([0 if k is LockIntent.READ else 1 for _, k, _ in drop], dtype=torch.uint8,
                             device=_dev(device)))
            assert rel.cpu().tolist() == [1] * len(drop)


@pytest.mark.parametrize("device", DEVICES)
def test_intent_locks_more_readers_than_holder_slots(device):
    from hypervisor.session.intent_locks import LockIntent

    host, dev = IntentLockManager(), IntentLockManager(device=_dev(device))

    def norm(x):
        return (type(x).__name__, str(x)) if isinstance(x, Exception) else (x.agent_did, x.resource_path, x.intent)

    reads = [(f"did:r{i}", "s", "/hot", LockIntent.READ) for i in range(24)]
    assert [norm(x) for x in host.acquire_batch(reads)] == [norm(x) for x in dev.acquire_batch(reads)]
    w = [("did:r0", "s", "/hot", LockIntent.WRITE)]
    assert [norm(x) for x in host.acquire_batch(w)] == [norm(x) for x in dev.acquire_batch(w)]
    for i in range(1, 24):
        assert host.release_agent_locks(f"did:r{i}", "s") == dev.release_agent_locks(f"did:r{i}", "s")
    got = dev.acquire_batch(w)
    assert [norm(x) for x in host.acquire_batch(w)] == [norm(x) for x in got]
    assert not isinstance(got[0], Exception)
