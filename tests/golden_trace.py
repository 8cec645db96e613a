"""Reference-pinned golden trace of the public API.

The reference package (``/root/reference/src/hypervisor``) is not present on the GPU
box, so its 326 tests can only be run here against the CPU twin store.  This module
closes that gap: seeded scripts of 1,300–2,500 public-API operations (session lifecycle,
joins with boundary σ values and action manifests, VFS writes / snapshots / permissions,
participant ring updates, audit captures and
Merkle roots, sagas with failing/retrying executors and compensation, vouch / σ_eff /
exposure / slash with cascades and bond expiry, ring checks, GC) is executed once by
the REFERENCE implementation on the CPU and every observable result is recorded in
``tests/fixtures/reference_trace*.json`` (``scripts/gen_reference_trace.py``).  The
replay (:func:`replay`) runs the same operations through THIS package with any store
(``host`` engines, the ``cpu`` twin, or ``cuda`` — the gfx950 store worker) and the
results must match the reference's record exactly: states, rings, error types and
messages, float values bit for bit, delta hashes and Merkle roots.

Determinism: both sides run under the same pinned clock (the reference's
``datetime.now`` is replaced in its modules while the trace is generated; this package
pins :mod:`hypervisor._clock`), session ids are the reference's (passed explicitly to
``create_session``), and generated ids (saga/step/vouch/slash uuids) are replaced by
their ordinals before comparison.

This file imports no ``hypervisor`` module at import time: the generator loads it
under the reference's package, the tests under this repository's.
"""

from __future__ import annotations

import asyncio
import json
import random
import re
from datetime import datetime, timedelta, timezone
from enum import Enum
from typing import Any, Callable, Optional

BASE_US = 1_767_225_600_000_000  # 2026-01-01T00:00:00Z
OP_US = 1_000  # the clock advances 1 ms per operation
DIDS = [f"did:mesh:g{i}" for i in range(8)]
SIGMAS = [0.0, 0.3, 0.49, 0.5, 0.59999999, 0.6, 0.60000001, 0.7, 0.85, 0.95, 0.950001, 1.0]
RISK = [0.0, 0.1, 0.25, 0.5, 0.9, 1.0]
REVERSIBILITY = ["full", "partial", "none"]
_UUID = re.compile(r"\b(saga|step|vouch|slash|snap|ckpt|branch|fanout):[0-9a-f-]{8,36}\b")


def at(us: int) -> datetime:
    return datetime(1970, 1, 1, tzinfo=timezone.utc) + timedelta(microseconds=us)


# ---------------------------------------------------------------------------
# the operation script (pure data; stored in the fixture)
# ---------------------------------------------------------------------------
def _action(rng: random.Random, i: int) -> list:
    return [f"act{i}", rng.choice(REVERSIBILITY), rng.random() < 0.2, rng.random() < 0.08, rng.random() < 0.6]


def make_ops(seed: int = 2026, n_sessions: int = 32, n_ops: int = 1200) -> list:
    rng = random.Random(seed)
    ops: list = []
    for k in range(n_sessions):
        cfg = {"max_participants": rng.choice([2, 3, 10]), "min_sigma_eff": rng.choice([0.3, 0.6, 0.9]),
               "enable_audit": rng.random() < 0.8, "consistency_mode": rng.choice(["eventual", "strong"])}
        ops.append(["create", k, cfg, rng.choice(DIDS)])
    n_sagas = 0
    steps: dict[int, int] = {}
    files: list[str] = [f"/doc{i}.txt" for i in range(5)]
    for _ in range(n_ops):
        r = rng.random()
        k = rng.randrange(n_sessions)
        did = rng.choice(DIDS)
        if r < 0.16:
            acts = [_action(rng, i) for i in range(rng.randrange(3))] if rng.random() < 0.4 else None
            ops.append(["join", k, did, rng.choice(SIGMAS), acts])
        elif r < 0.21:
            ops.append(["activate", k])
        elif r < 0.34:
            changes = [[rng.choice(files), rng.choice(["add", "modify", "delete", "permission"]),
                        rng.choice([None, f"h{rng.randrange(1000)}"]), rng.choice([None, f"p{rng.randrange(99)}"])]
                       for _ in range(rng.randrange(4))]
            ops.append(["capture", k, did, changes])
        elif r < 0.37:
            ops.append(["leave", k, did])
        elif r < 0.38:
            ops.append(["terminate", k])
        elif r < 0.43:
            ops.append(["vfs_write", k, rng.choice(files), f"content-{rng.randrange(50)}", did])
        elif r < 0.45:
            ops.append(["vfs_read", k, rng.choice(files)])
        elif r < 0.46:
            ops.append(["vfs_delete", k, rng.choice(files), did])
        elif r < 0.49:
            ops.append(["saga", k])
            n_sagas += 1
        elif r < 0.55 and n_sagas:
            g = rng.randrange(n_sagas)
            ops.append(["add_step", g, f"a{rng.randrange(20)}", did,
                        rng.choice([None, "/api/undo"]), rng.choice([0, 0, 1])])
            steps[g] = steps.get(g, 0) + 1
        elif r < 0.63 and steps:
            g = rng.choice(sorted(steps))
            ops.append(["exec", g, rng.randrange(steps[g]), rng.choice(["ok", "ok", "fail", "fail1"])])
        elif r < 0.66 and n_sagas:
            ops.append(["compensate", rng.randrange(n_sagas), rng.choice(["ok", "ok", "fail"])])
        elif r < 0.76:
            voucher, vouchee = rng.sample(DIDS[:6], 2)
            expiry = rng.choice([None, None, None, -OP_US, 3 * OP_US, 40 * OP_US])
            ops.append(["vouch", voucher, vouchee, k, rng.choice(SIGMAS), rng.choice([None, 0.1, 0.2, 0.35, 0.5, 1.5,
                                                                                      -0.1]),
                        expiry])
        elif r < 0.80:
            ops.append(["sigma_eff", did, k, rng.choice(SIGMAS), rng.choice(RISK)])
        elif r < 0.83:
            ops.append(["exposure", did, k])
        elif r < 0.85:
            ops.append(["vouchers", did, k])
        elif r < 0.89:
            scores = {d: rng.choice(SIGMAS) for d in rng.sample(DIDS[:6], rng.randrange(1, 6))}
            ops.append(["slash", rng.choice(DIDS[:6]), k, rng.choice(SIGMAS), rng.choice(RISK),
                        f"violation-{rng.randrange(9)}", scores])
        elif r < 0.93:
            ops.append(["ring_check", rng.randrange(4), _action(rng, 0), rng.choice(SIGMAS),
                        rng.random() < 0.3, rng.random() < 0.3])
        elif r < 0.95:
            ops.append(["verify_chain", k])
        elif r < 0.96:
            ops.append(["root", k])
        elif r < 0.97:
            ops.append(["state", k])
        else:  # participant / VFS-snapshot / permission / hypervisor-view operations
            q = rng.random()
            if q < 0.2:
                ops.append(["update_ring", k, did, rng.randrange(4)])
            elif q < 0.35:
                ops.append(["get_participant", k, did])
            elif q < 0.5:
                ops.append(["snapshot", k])
            elif q < 0.65:
                ops.append(["restore", k, rng.randrange(4), did])
            elif q < 0.8:
                ops.append(["perm", k, rng.choice(files), sorted(rng.sample(DIDS, rng.randrange(1, 3))), did])
            elif q < 0.9:
                ops.append(["views"])
            else:
                ops.append(["edits", k, did])
    for k in range(n_sessions):
        ops.append(["terminate", k])
        ops.append(["state", k])
    ops.append(["gc_history"])
    return ops


# ---------------------------------------------------------------------------
# the runner (works against either implementation of the public API)
# ---------------------------------------------------------------------------
def _v(x: Any) -> Any:
    return x.value if isinstance(x, Enum) else x


def _err(e: BaseException) -> dict:
    return {"error": type(e).__name__, "msg": str(e)}


class _Ids:
    """Generated ids → ordinals (uuids differ between the two runs)."""

    def __init__(self) -> None:
        self.seen: dict[str, str] = {}

    def scrub(self, x: Any) -> Any:
        if isinstance(x, str):
            return _UUID.sub(lambda m: self.seen.setdefault(m.group(0), f"<{m.group(1)}#{len(self.seen)}>"), x)
        if isinstance(x, list):
            return [self.scrub(y) for y in x]
        if isinstance(x, dict):
            return {k: self.scrub(v) for k, v in x.items()}
        return x


async def run_ops(ops: list, set_now: Callable[[int], None], hv_kwargs: Optional[dict] = None,
                  session_ids: Optional[list] = None) -> dict:
    """Execute ``ops`` through the importable ``hypervisor`` package.

    ``set_now(us)`` pins the implementation's clock; ``session_ids`` (replay) are the
    reference's session ids, passed to ``create_session``.  Returns ``{"sids": [...],
    "results": [...]}`` with one JSON-able result per operation.
    """
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor.audit.delta import VFSChange
    from hypervisor.models import ActionDescriptor, ConsistencyMode, ExecutionRing, ReversibilityLevel

    hv = Hypervisor(**(hv_kwargs or {}))
    ids = _Ids()
    sids: list[str] = []
    sessions: list = []
    sagas: list = []  # (managed session, saga, [steps])
    res: list = []
    calls: dict[tuple, int] = {}
    snaps: dict[int, list] = {}

    def action(spec: list) -> Any:
        aid, rev, ro, admin, undo = spec
        return ActionDescriptor(action_id=aid, name=aid, execute_api=f"/api/{aid}",
                                undo_api=f"/api/{aid}/undo" if undo else None,
                                reversibility=ReversibilityLevel(rev), is_read_only=ro, is_admin=admin)

    def participants(m) -> list:
        return [[p.agent_did, _v(p.ring), p.sigma_raw, p.sigma_eff, p.is_active] for p in m.sso.participants]

    for i, op in enumerate(ops):
        now = BASE_US + i * OP_US
        set_now(now)
        kind = op[0]
        try:
            if kind == "create":
                _, k, cfg, creator = op
                c = SessionConfig(consistency_mode=ConsistencyMode(cfg["consistency_mode"]),
                                  max_participants=cfg["max_participants"], min_sigma_eff=cfg["min_sigma_eff"],
                                  enable_audit=cfg["enable_audit"])
                if session_ids is None:
                    m = await hv.create_session(c, creator)
                else:
                    m = await hv.create_session(c, creator, session_id=session_ids[k])
                sessions.append(m)
                sids.append(m.sso.session_id)
                out = {"state": _v(m.sso.state), "mode": _v(m.sso.consistency_mode)}
            elif kind == "join":
                _, k, did, sigma, acts = op
                ring = await hv.join_session(sids[k], did, actions=[action(a) for a in acts] if acts else None,
                                             sigma_raw=sigma)
                m = sessions[k]
                out = {"ring": _v(ring), "mode": _v(m.sso.consistency_mode), "participants": participants(m)}
            elif kind == "activate":
                await hv.activate_session(sids[op[1]])
                out = {"state": _v(sessions[op[1]].sso.state)}
            elif kind == "capture":
                _, k, did, changes = op
                d = sessions[k].delta_engine.capture(
                    did, [VFSChange(path=p, operation=o, content_hash=h, previous_hash=ph) for p, o, h, ph in changes])
                out = {"turn": d.turn_id, "hash": d.delta_hash, "parent": d.parent_hash}
            elif kind == "leave":
                sessions[op[1]].sso.leave(op[2])
                out = {"participants": participants(sessions[op[1]])}
            elif kind == "terminate":
                root = await hv.terminate_session(sids[op[1]])
                out = {"root": root, "state": _v(sessions[op[1]].sso.state)}
            elif kind == "vfs_write":
                _, k, path, content, did = op
                e = sessions[k].sso.vfs.write(path, content, did)
                out = {"op": _v(getattr(e, "operation", None)), "path": getattr(e, "path", None)}
            elif kind == "vfs_read":
                out = {"content": sessions[op[1]].sso.vfs.read(op[2]),
                       "files": sorted(sessions[op[1]].sso.vfs.list_files())}
            elif kind == "vfs_delete":
                sessions[op[1]].sso.vfs.delete(op[2], op[3])
                out = {"files": sorted(sessions[op[1]].sso.vfs.list_files())}
            elif kind == "saga":
                m = sessions[op[1]]
                m.saga.DEFAULT_RETRY_DELAY_SECONDS = 0.0
                g = m.saga.create_saga(sids[op[1]])
                sagas.append((m, g, []))
                out = {"state": _v(g.state), "session": g.session_id == sids[op[1]]}
            elif kind == "add_step":
                _, gi, aid, did, undo, retries = op
                m, g, sts = sagas[gi]
                st = m.saga.add_step(g.saga_id, aid, did, f"/api/{aid}", undo_api=undo, max_retries=retries)
                sts.append(st)
                out = {"state": _v(st.state), "n": len(sts)}
            elif kind == "exec":
                _, gi, ti, outcome = op
                m, g, sts = sagas[gi]
                st = sts[ti]
                key = (gi, ti)

                async def executor(key=key, outcome=outcome, i=i):
                    n = calls[key] = calls.get(key, 0) + 1
                    if outcome == "fail" or (outcome == "fail1" and n == 1):
                        raise RuntimeError(f"boom-{i}")
                    return f"r{i}"

                try:
                    ret = await m.saga.execute_step(g.saga_id, st.step_id, executor=executor)
                    r = {"ret": ret}
                except Exception as e:  # noqa: BLE001 - the error is part of the record
                    r = _err(e)
                r.update(state=_v(st.state), step_error=st.error, retry=st.retry_count, saga=_v(g.state),
                         result=st.execute_result)
                out = r
            elif kind == "compensate":
                _, gi, outcome = op
                m, g, sts = sagas[gi]

                async def compensator(step, outcome=outcome, i=i):
                    if outcome == "fail":
                        raise RuntimeError(f"undo-{i}")
                    return f"u{i}"

                try:
                    failed = await m.saga.compensate(g.saga_id, compensator)
                    r = {"failed": [sts.index(s) if s in sts else -1 for s in failed]}
                except Exception as e:  # noqa: BLE001
                    r = _err(e)
                r.update(saga=_v(g.state), saga_error=g.error,
                         steps=[[_v(s.state), s.error, s.compensation_result] for s in sts])
                out = r
            elif kind == "vouch":
                _, voucher, vouchee, k, sigma, pct, exp = op
                rec = hv.vouching.vouch(voucher, vouchee, sids[k], sigma, bond_pct=pct,
                                        expiry=None if exp is None else at(now + exp))
                out = {"amount": rec.bonded_amount, "pct": rec.bonded_sigma_pct, "active": rec.is_active}
            elif kind == "sigma_eff":
                _, did, k, sigma, w = op
                out = {"sigma_eff": hv.vouching.compute_sigma_eff(did, sids[k], sigma, w)}
            elif kind == "exposure":
                out = {"exposure": hv.vouching.get_total_exposure(op[1], sids[op[2]])}
            elif kind == "vouchers":
                out = {"vouchers": [[v.voucher_did, v.bonded_amount, v.bonded_sigma_pct]
                                    for v in hv.vouching.get_vouchers_for(op[1], sids[op[2]])]}
            elif kind == "slash":
                _, vouchee, k, sigma, w, reason, scores = op
                before = len(hv.slashing.history)
                sc = dict(scores)
                r = hv.slashing.slash(vouchee, sids[k], sigma, w, reason, sc)
                hist = hv.slashing.history[before:]
                out = {"before": r.vouchee_sigma_before, "after": r.vouchee_sigma_after,
                       "clips": [[c.voucher_did, c.sigma_before, c.sigma_after,
                                  c.risk_weight] for c in r.voucher_clips],
                       "cascade": [[h.vouchee_did, h.cascade_depth, h.reason, len(h.voucher_clips)] for h in hist],
                       "scores": sorted(sc.items())}
            elif kind == "ring_check":
                _, ring, spec, sigma, cons, wit = op
                c = hv.ring_enforcer.check(ExecutionRing(ring), action(spec), sigma, has_consensus=cons,
                                           has_sre_witness=wit)
                out = {"allowed": c.allowed, "required": _v(c.required_ring), "agent": _v(c.agent_ring),
                       "sigma": c.sigma_eff, "reason": c.reason, "consensus": c.requires_consensus,
                       "witness": c.requires_sre_witness, "ring_for_sigma": _v(hv.ring_enforcer.compute_ring(sigma)),
                       "demote": hv.ring_enforcer.should_demote(ExecutionRing(ring), sigma)}
            elif kind == "verify_chain":
                de = sessions[op[1]].delta_engine
                out = {"ok": de.verify_chain(), "turns": de.turn_count, "n": len(de.deltas)}
            elif kind == "root":
                out = {"root": sessions[op[1]].delta_engine.compute_merkle_root()}
            elif kind == "state":
                m = sessions[op[1]]
                out = {"state": _v(m.sso.state), "mode": _v(m.sso.consistency_mode), "count": m.sso.participant_count,
                       "participants": participants(m),
                       "commit": (lambda c: None if c is None else [c.merkle_root, c.participant_dids, c.delta_count])(
                           hv.commitment.get_commitment(sids[op[1]]))}
            elif kind == "update_ring":
                _, k, did, ring = op
                sessions[k].sso.update_ring(did, ExecutionRing(ring))
                out = {"participants": participants(sessions[k])}
            elif kind == "get_participant":
                p_ = sessions[op[1]].sso.get_participant(op[2])
                out = {"p": [p_.agent_did, _v(p_.ring), p_.sigma_raw, p_.sigma_eff, p_.is_active]}
            elif kind == "snapshot":
                snap = sessions[op[1]].sso.create_vfs_snapshot()
                snaps.setdefault(op[1], []).append(snap)
                out = {"snap": snap, "n": sessions[op[1]].sso.vfs.snapshot_count}
            elif kind == "restore":
                _, k, j, did = op
                lst = snaps.get(k, [])
                sessions[k].sso.restore_vfs_snapshot(lst[j % len(lst)] if lst else "snap:missing", did)
                vfs = sessions[k].sso.vfs
                out = {"files": sorted(vfs.list_files()), "contents": [vfs.read(f) for f in sorted(vfs.list_files())]}
            elif kind == "perm":
                _, k, path, allowed, did = op
                e = sessions[k].sso.vfs.set_permissions(path, set(allowed), did)
                out = {"op": _v(getattr(e, "operation", None)),
                       "perms": sorted(sessions[k].sso.vfs.get_permissions(path) or [])}
            elif kind == "views":
                out = {"active": sorted(sids.index(m.sso.session_id) for m in hv.active_sessions),
                       "known": [hv.get_session(x) is not None for x in sids]}
            elif kind == "edits":
                vfs = sessions[op[1]].sso.vfs
                log = vfs.edit_log
                mine = vfs.edits_by_agent(op[2])
                out = {"n": len(log), "last": [log[-1].operation, log[-1].agent_did] if log else None,
                       "mine": len(mine), "count": vfs.file_count}
            elif kind == "gc_history":
                out = {"gc": [[sids.index(h.session_id) if h.session_id in sids else -1, h.retained_deltas,
                               h.purged_vfs_files, h.purged_caches] for h in hv.gc.history]}
            else:
                raise ValueError(f"unknown op {kind}")
        except Exception as e:  # noqa: BLE001 - errors are part of the observable behaviour
            out = _err(e)
        res.append(ids.scrub(out))
    return {"sids": sids, "results": res}


def replay(fixture: dict, device: str, parity: bool = True) -> list:
    """Run the fixture's operations through this package on ``device``; return the
    list of ``(index, op, expected, got)`` mismatches (empty = parity).

    ``parity``: run with ``hypervisor.config`` parity mode on — the one documented
    behavioural divergence of this package is that terminate-time GC really empties
    the session VFS (the reference's GC calls ``vfs.delete(path)`` without the agent
    argument and swallows the TypeError, so its files survive); parity mode
    reproduces the reference's outcome."""
    from hypervisor._clock import set_clock
    from hypervisor.config import parity_mode, set_parity_mode

    cur = [BASE_US]
    set_clock(lambda: at(cur[0]))
    was = parity_mode()
    set_parity_mode(parity)

    def set_now(us: int) -> None:
        cur[0] = us

    try:
        got = asyncio.run(run_ops(fixture["ops"], set_now, {"device": device}, session_ids=fixture["sids"]))
    finally:
        set_clock(None)
        set_parity_mode(was)
    bad = []
    res = json.loads(json.dumps(got["results"]))  # tuples → lists, as in the fixture
    for i, (op, exp, g) in enumerate(zip(fixture["ops"], fixture["results"], res)):
        if exp != g:
            bad.append((i, op, exp, g))
    return bad
