"""VouchingEngine.vouch_batch (K05 over every session's requests in one launch)
must equal calling vouch() in list order: same admitted records (bond amounts
bit-for-bit), same rejections with the same messages, same engine state."""

from __future__ import annotations

import random
from datetime import timedelta

import pytest

from hypervisor._clock import now as _now
from hypervisor.liability.vouching import VouchingEngine, VouchingError


def _requests(seed: int, sessions: int = 12, n: int = 400, agents: int = 9):
    rnd = random.Random(seed)
    out = []
    for _ in range(n):
        s = f"session:{rnd.randrange(sessions)}"
        a, b = f"did:{rnd.randrange(agents)}", f"did:{rnd.randrange(agents)}"
        sigma = rnd.choice([0.3, 0.49, 0.5, 0.55, 0.7, 0.9, 1.0])
        pct = rnd.choice([None, 0.05, 0.1, 0.2, 0.35, 0.8, 1.5, -0.2])
        exp = rnd.choice([None, None, _now() + timedelta(hours=1)])
        out.append((a, b, s, sigma, pct, exp))
    return out


def _outcome(x):
    if isinstance(x, VouchingError):
        return ("err", str(x))
    return ("ok", x.voucher_did, x.vouchee_did, x.session_id, x.bonded_sigma_pct, x.bonded_amount, x.expiry)


def _state(eng: VouchingEngine):
    return sorted((v.session_id, v.voucher_did, v.vouchee_did, v.bonded_amount, v.is_active) for v in eng.records())


def _check(seed: int, device: str, prefill: int = 60):
    reqs = _requests(seed)
    seq, bat = VouchingEngine(), VouchingEngine()
    for e in (seq, bat):  # identical pre-existing live edges (some released)
        for r in reqs[:prefill]:
            try:
                e.vouch(*r)
            except VouchingError:
                pass
        for rec in list(e.records())[::5]:
            e.release_bond(rec.vouch_id)
    expect = []
    for r in reqs[prefill:]:
        try:
            expect.append(seq.vouch(*r))
        except VouchingError as err:
            expect.append(err)
    got = bat.vouch_batch(reqs[prefill:], device=device)
    assert [_outcome(x) for x in got] == [_outcome(x) for x in expect]
    assert _state(bat) == _state(seq)
    kinds = {str(x).split(" ")[0] for x in expect if isinstance(x, VouchingError)}
    return sum(isinstance(x, VouchingError) for x in expect), kinds


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_vouch_batch_equals_sequential_cpu(seed):
    errors, kinds = _check(seed, "cpu")
    assert errors > 20 and {"Cannot", "Voucher", "Circular"} <= kinds


def test_wide_sessions_and_parity_mode_take_scalar_path(monkeypatch):
    reqs = [(f"did:{k}", f"did:{k + 1}", "session:wide", 0.9, 0.1) for k in range(20)]  # 21 agents > 16
    a, b = VouchingEngine(), VouchingEngine()
    want = [a.vouch(*r) for r in reqs]
    got = b.vouch_batch(reqs)
    assert [_outcome(x) for x in got] == [_outcome(x) for x in want]
    monkeypatch.setenv("AHV_PARITY_MODE", "1")
    diamond = [("did:a", "did:b", "s", 0.9), ("did:a", "did:c", "s", 0.9), ("did:b", "did:d", "s", 0.9),
               ("did:c", "did:d", "s", 0.9), ("did:d", "did:a", "s", 0.9), ("did:a", "did:d", "s", 0.9)]
    a, b = VouchingEngine(), VouchingEngine()
    want = []
    for r in diamond:
        try:
            want.append(a.vouch(*r))
        except VouchingError as e:
            want.append(e)
    assert [_outcome(x) for x in b.vouch_batch(diamond)] == [_outcome(x) for x in want]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_vouch_batch_equals_sequential_gpu(seed):
    errors, _ = _check(seed, "cuda")
    assert errors > 20
