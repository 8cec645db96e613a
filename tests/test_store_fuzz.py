"""Differential fuzzing of the device-authoritative store against the host engines.

Random programs of public API calls — session lifecycle, joins at boundary σ,
audit captures with awkward strings, vouches, σ_eff / exposure queries, slashes
with cascades, sagas that commit / fail / compensate, Merkle roots, chain
verification, terminations — run on ``Hypervisor(device="host")`` and on the
store (``device="cpu"``: the CPU twin of the gfx950 command processor; ``"cuda"``
under ``-m gpu``).  Every call's observable outcome (return value, exact floats,
state, or exception type and message with ids normalised) must match.  Digests
cannot match across the two runs (session ids are random uuid4s), so each run's
audit results are also checked against host SHA-256 of its own records.
"""

from __future__ import annotations

import asyncio
import random
import re
from datetime import datetime, timezone

import pytest

from agent_hypervisor_amd._native import C
from hypervisor import Hypervisor, SessionConfig
from hypervisor import _clock
from hypervisor.audit.delta import VFSChange, delta_digest
from hypervisor.models import ConsistencyMode

_ID = re.compile(r"(session|saga|step|vouch|delta|ckpt|snap):[0-9a-f-]{8,36}")
AGENTS = [f"did:mesh:{n}" for n in ("alice", "bob", "carol", "dave", "erin", "frank", "grace")]
SIGMAS = [0.0, 0.3, 0.49, 0.5, 0.59999999, 0.6, 0.60000001, 0.7, 0.85, 0.95, 0.950001, 1.0]
STRINGS = ["plain", "quote\"d", "back\\slash", "tab\tnew\nline", "ünïcødé", "emoji 🚀", "\x01ctl", ""]


def _norm(x):
    if isinstance(x, BaseException):
        return ("raise", type(x).__name__, _ID.sub(r"\1:<id>", str(x)))
    if isinstance(x, str):
        return _ID.sub(r"\1:<id>", x)
    if isinstance(x, (list, tuple)):
        return tuple(_norm(v) for v in x)
    return x


def program(seed: int, n: int = 240) -> list:
    rnd = random.Random(seed)
    ops = [("create", 6, 0.5, False), ("create", 3, 0.6, True), ("create", 10, 0.3, False)]
    for s in range(3):
        ops += [("join", s, AGENTS[s], 0.8), ("join", s, AGENTS[s + 1], 0.96), ("activate", s)]
    for _ in range(n):
        k = rnd.random()
        s = -1 - rnd.randrange(4)  # recent sessions: they are the live ones
        a, b = rnd.choice(AGENTS), rnd.choice(AGENTS)
        if k < 0.08:
            ops.append(("create", rnd.randint(1, 6), rnd.choice([0.3, 0.5, 0.6, 0.7]), rnd.random() < 0.3))
        elif k < 0.26:
            ops.append(("join", s, a, rnd.choice(SIGMAS)))
        elif k < 0.32:
            ops.append(("activate", s))
        elif k < 0.46:
            nch = rnd.randint(1, 3)
            ops.append(("capture", s, a, [(f"/{rnd.choice(STRINGS)}/{i}", rnd.choice(["add", "modify", "delete"]),
                                           rnd.choice([None, rnd.choice(STRINGS)])) for i in range(nch)]))
        elif k < 0.56:
            ops.append(("vouch", s, a, b, rnd.choice(SIGMAS), rnd.choice([None, 0.1, 0.2, 0.45, 0.9, 1.3])))
        elif k < 0.62:
            ops.append(("sigma", s, a, rnd.choice(SIGMAS), rnd.choice([0.0, 0.5, 0.65, 1.0])))
        elif k < 0.66:
            ops.append(("slash", s, a, rnd.choice([0.4, 0.8]), rnd.choice([0.5, 0.95]),
                        {d: rnd.choice(SIGMAS) for d in rnd.sample(AGENTS, 4)}))
        elif k < 0.74:
            ops.append(("saga", s, rnd.randint(1, 3), rnd.random() < 0.3, rnd.random() < 0.5, a))
        elif k < 0.80:
            ops.append(("root", s))
        elif k < 0.86:
            ops.append(("verify", s))
        elif k < 0.90:
            ops.append(("terminate", s) if rnd.random() < 0.5 else ("activate", s))
        elif k < 0.95:
            ops.append(("state", s))
        else:
            ops.append(("exposure", s, a))
    return ops


async def run(device: str, ops: list) -> list:
    hv = Hypervisor(device=device)
    sessions: list = []
    out: list = []

    def sess(i):
        if not sessions:
            raise LookupError("no sessions")
        return sessions[i % len(sessions)]

    for op in ops:
        kind = op[0]
        try:
            if kind == "create":
                cfg = SessionConfig(max_participants=op[1], min_sigma_eff=op[2],
                                    consistency_mode=ConsistencyMode.STRONG if op[3] else ConsistencyMode.EVENTUAL)
                m = await hv.create_session(cfg, creator_did="did:mesh:admin")
                sessions.append(m)
                res = (m.sso.state.value, m.sso.consistency_mode.value)
            elif kind == "join":
                m = sess(op[1])
                ring = await hv.join_session(m.sso.session_id, op[2], sigma_raw=op[3])
                res = (ring.name, m.sso.participant_count)
            elif kind == "activate":
                m = sess(op[1])
                await hv.activate_session(m.sso.session_id)
                res = m.sso.state.value
            elif kind == "capture":
                m = sess(op[1])
                d = m.delta_engine.capture(op[2], [VFSChange(path=p, operation=o, content_hash=h) for p, o, h in op[3]])
                res = (d.turn_id, d.delta_id, d.parent_hash is None, delta_digest(d) == d.delta_hash)
            elif kind == "vouch":
                m = sess(op[1])
                r = hv.vouching.vouch(op[2], op[3], m.sso.session_id, op[4], bond_pct=op[5])
                res = (r.bonded_amount, r.bonded_sigma_pct, r.is_active)
            elif kind == "sigma":
                m = sess(op[1])
                res = hv.vouching.compute_sigma_eff(op[2], m.sso.session_id, op[3], op[4])
            elif kind == "exposure":
                m = sess(op[1])
                res = hv.vouching.get_total_exposure(op[2], m.sso.session_id)
            elif kind == "slash":
                m = sess(op[1])
                scores = dict(op[5])
                r = hv.slashing.slash(op[2], m.sso.session_id, op[3], op[4], "fuzz", scores)
                res = (r.vouchee_did, r.vouchee_sigma_before, r.vouchee_sigma_after, r.cascade_depth,
                       [(c.voucher_did, c.sigma_before, c.sigma_after) for c in r.voucher_clips],
                       sorted(scores.items()))
            elif kind == "saga":
                m = sess(op[1])
                saga = m.saga.create_saga(m.sso.session_id)
                steps = [m.saga.add_step(saga.saga_id, f"a{j}", op[5], f"/x/{j}",
                                         undo_api=f"/u/{j}" if j % 2 == 0 else None)
                         for j in range(op[2])]
                fail = op[3]
                trail = []
                for j, st in enumerate(steps):
                    async def ex(j=j):
                        if fail and j == len(steps) - 1:
                            raise RuntimeError(f"step {j} refused")
                        return j
                    try:
                        trail.append(await m.saga.execute_step(saga.saga_id, st.step_id, executor=ex))
                    except Exception as e:  # noqa: BLE001
                        trail.append(_norm(e))
                        if op[4]:
                            failed = await m.saga.compensate(saga.saga_id, lambda step: asyncio.sleep(0))
                            trail.append(len(failed))
                        break
                res = (trail, saga.state.value, [s.state.value for s in saga.steps])
            elif kind == "root":
                m = sess(op[1])
                root = m.delta_engine.compute_merkle_root()
                ds = m.delta_engine.deltas
                res = (root is None, len(ds), root == (C.merkle_root([d.delta_hash for d in ds]) if ds else None))
            elif kind == "verify":
                res = sess(op[1]).delta_engine.verify_chain()
            elif kind == "terminate":
                m = sess(op[1])
                ds = m.delta_engine.deltas
                want = C.merkle_root([d.delta_hash for d in ds]) if ds else None
                root = await hv.terminate_session(m.sso.session_id)
                res = (root == want if m.sso.config.enable_audit else root is None, m.sso.state.value)
            elif kind == "state":
                m = sess(op[1])
                res = (m.sso.state.value, m.sso.participant_count,
                       sorted((p.agent_did, p.ring.name, p.sigma_eff) for p in m.sso.participants))
            else:
                raise AssertionError(kind)
        except Exception as e:  # noqa: BLE001 - the exception is the outcome
            res = e
        out.append((kind, _norm(res)))
    return out


def _differential(device: str, seed: int) -> None:
    fixed = datetime(2026, 5, 1, 12, 0, 0, 250000, tzinfo=timezone.utc)
    prev = _clock._override
    _clock.set_clock(lambda: fixed)
    try:
        ops = program(seed)
        host = asyncio.run(run("host", ops))
        dev = asyncio.run(run(device, ops))
    finally:
        _clock.set_clock(prev)
    for i, (h, d) in enumerate(zip(host, dev)):
        assert h == d, f"seed {seed} op {i} {ops[i]}:\n host   {h}\n device {d}"
    kinds = {k for k, r in host if not (isinstance(r, tuple) and r and r[0] == "raise")}
    assert len(kinds) >= 8, kinds  # the program exercised most of the API successfully


@pytest.mark.parametrize("seed", range(6))
def test_store_twin_matches_host_engines(seed):
    _differential("cpu", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6, 10))
def test_device_store_matches_host_engines(seed):
    _differential("cuda", seed)
