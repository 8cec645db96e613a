"""Vouching & bonding: a high-σ agent locks part of its reputation behind a
low-σ agent inside one session.

Parity target: reference ``liability/vouching.py:19-234``.

* ``vouch`` rejects, in order: self-vouch; voucher σ < 0.50; a cycle through
  active vouches of the same session; exposure ``current + σ·pct > σ·max``
  (strict fp64 ``>``).  ``pct`` is clamped to [0, 1]; ``max_exposure`` 0 or None
  selects 0.80.
* ``compute_sigma_eff = min(σ + ω · Σ bonded(active, unexpired vouches of the
  vouchee in the session), 1)`` summed in vouch-creation order (bit parity).
* Everything is session-scoped.

Differences from the reference:

* records are indexed per session (insertion-ordered), so queries cost
  O(vouches in the session) instead of O(all vouches ever) — the reference's
  ``vouching_sigma_eff`` benchmark degrades to 1.45 ms because of that scan;
* the cycle check reports only real cycles.  The reference BFS re-enqueues nodes
  reached by two paths and rejects diamond-shaped graphs as "circular"
  (SURVEY Appendix A, Q05); ``hypervisor.config`` parity mode restores that.

The batched twins are kernels K03 (σ_eff on MFMA), K04 (exposure), K05 (admit)
and K07 (release) in ``csrc/hip/liability_kernels.hip``.
"""

from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from datetime import datetime
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor import config as _cfg
from hypervisor._clock import now as _now


@dataclass
class VouchRecord:
    vouch_id: str
    voucher_did: str
    vouchee_did: str
    session_id: str
    bonded_sigma_pct: float
    bonded_amount: float
    created_at: datetime = field(default_factory=_now)
    expiry: Optional[datetime] = None
    is_active: bool = True
    released_at: Optional[datetime] = None

    @property
    def is_expired(self) -> bool:
        return self.expiry is not None and _now() > self.expiry

    @property
    def is_live(self) -> bool:
        return self.is_active and (self.expiry is None or _now() <= self.expiry)


class VouchingError(Exception):
    """Vouching protocol violation."""


class VouchingEngine:
    SCORE_SCALE = 1000.0
    MIN_VOUCHER_SCORE = 0.50
    DEFAULT_BOND_PCT = 0.20
    DEFAULT_MAX_EXPOSURE = 0.80

    def __init__(self, max_exposure: Optional[float] = None) -> None:
        self._vouches: dict[str, VouchRecord] = {}
        self._by_session: dict[str, list[VouchRecord]] = {}
        self.max_exposure = max_exposure or self.DEFAULT_MAX_EXPOSURE

    # -- internal views ----------------------------------------------------
    def _session_records(self, session_id: str) -> list[VouchRecord]:
        return self._by_session.get(session_id, [])

    def _live(self, session_id: str):
        t = _now()
        for v in self._session_records(session_id):
            if v.is_active and (v.expiry is None or t <= v.expiry) and v.session_id == session_id:
                yield v

    def _active_vouches_for(self, agent_did: str, session_id: str) -> list[VouchRecord]:
        return [v for v in self._live(session_id) if v.vouchee_did == agent_did]

    # -- protocol ------------------------------------------------------------
    def vouch(
        self,
        voucher_did: str,
        vouchee_did: str,
        session_id: str,
        voucher_sigma: float,
        bond_pct: Optional[float] = None,
        expiry: Optional[datetime] = None,
    ) -> VouchRecord:
        if voucher_did == vouchee_did:
            raise VouchingError("Cannot vouch for yourself")
        if voucher_sigma < self.MIN_VOUCHER_SCORE:
            raise VouchingError(
                f"Voucher σ ({voucher_sigma:.2f}) below minimum ({self.MIN_VOUCHER_SCORE:.2f})"
            )
        if self._creates_cycle(voucher_did, vouchee_did, session_id):
            raise VouchingError(
                f"Circular vouching detected: {vouchee_did} already vouches for "
                f"{voucher_did} in session {session_id}"
            )
        pct = self.DEFAULT_BOND_PCT if bond_pct is None else bond_pct
        pct = max(0.0, min(1.0, pct))
        bonded = voucher_sigma * pct
        current = self.get_total_exposure(voucher_did, session_id)
        limit = voucher_sigma * self.max_exposure
        if current + bonded > limit:
            raise VouchingError(
                f"Voucher {voucher_did} would exceed max exposure "
                f"({self.max_exposure:.0%} of σ). Current: {current:.3f}, "
                f"requested: {bonded:.3f}, limit: {limit:.3f}"
            )
        rec = VouchRecord(
            vouch_id=_C.uuid4("vouch:"),
            voucher_did=voucher_did,
            vouchee_did=vouchee_did,
            session_id=session_id,
            bonded_sigma_pct=pct,
            bonded_amount=bonded,
            expiry=expiry,
        )
        self._vouches[rec.vouch_id] = rec
        self._by_session.setdefault(session_id, []).append(rec)
        return rec

    def vouch_batch(self, requests: list, device: Optional[str] = None) -> list:
        """Admit many vouch requests at once; returns, per request, the new
        :class:`VouchRecord` or the :class:`VouchingError` that ``vouch`` would
        have raised — exactly as if ``vouch(*req)`` were called in list order.

        ``requests``: tuples ``(voucher_did, vouchee_did, session_id,
        voucher_sigma[, bond_pct[, expiry]])``.  Sessions are independent, so
        every session's requests are admitted in one K05 launch (adjacency
        bit-matrix cycle closure + running per-voucher exposure, fp64 in the
        reference's addition order) over the session's live edges.  Sessions with
        more than 16 distinct agents, and parity mode (the reference's diamond
        "cycles"), take the scalar path."""
        import torch

        from agent_hypervisor_amd.ops import liability as LI
        from hypervisor._clock import to_us

        reqs = [tuple(r) + (None,) * (6 - len(r)) for r in requests]
        out: list = [None] * len(reqs)
        now = _now()
        by_sess: dict[str, list[int]] = {}
        for i, r in enumerate(reqs):
            by_sess.setdefault(r[2], []).append(i)
        batched: list[tuple[str, list[int], list, dict]] = []
        for sid, idx in by_sess.items():
            live = list(self._live(sid))
            local: dict[str, int] = {}
            for v in live:
                local.setdefault(v.voucher_did, len(local))
                local.setdefault(v.vouchee_did, len(local))
            for i in idx:
                local.setdefault(reqs[i][0], len(local))
                local.setdefault(reqs[i][1], len(local))
            stale = any(reqs[i][5] is not None and reqs[i][5] < now for i in idx)  # born expired: not live later
            if _cfg.parity_mode() or len(local) > 16 or stale:
                for i in idx:  # scalar path, in order
                    try:
                        out[i] = self.vouch(*reqs[i])
                    except VouchingError as e:
                        out[i] = e
                continue
            batched.append((sid, idx, live, local))
        if not batched:
            return out
        dev = torch.device(device) if device else torch.device("cpu")
        e_off, e_vr, e_ve, e_bd, r_off, r_vr, r_ve, r_sg, r_pc = [0], [], [], [], [0], [], [], [], []
        for sid, idx, live, local in batched:
            for v in live:  # every edge passed is live now: active, expiry -1
                e_vr.append(local[v.voucher_did])
                e_ve.append(local[v.vouchee_did])
                e_bd.append(v.bonded_amount)
            e_off.append(len(e_vr))
            for i in idx:
                r = reqs[i]
                r_vr.append(local[r[0]])
                r_ve.append(local[r[1]])
                r_sg.append(float(r[3]))
                r_pc.append(self.DEFAULT_BOND_PCT if r[4] is None else float(r[4]))
            r_off.append(len(r_vr))
        t = lambda x, dt: torch.tensor(x, dtype=dt).to(dev)  # noqa: E731
        u8, i32, i64, f64 = torch.uint8, torch.int32, torch.int64, torch.float64
        E = len(e_vr)
        vb = LI.VouchBatch(t(e_off, i32), t(e_vr, u8), t(e_ve, u8), t(e_bd, f64), torch.ones(E, dtype=u8, device=dev),
                           torch.full((E,), -1, dtype=i64, device=dev), torch.full((E,), -1, dtype=i64, device=dev))
        code, bonded = LI.vouch_admit(vb, t(r_off, i32), t(r_vr, u8), t(r_ve, u8), t(r_sg, f64), t(r_pc, f64),
                                      to_us(now), self.max_exposure)
        code, bonded = code.cpu().tolist(), bonded.cpu().tolist()
        q = 0
        for sid, idx, _live, _local in batched:
            for i in idx:
                vr, ve, _s, sig, pct, expiry = reqs[i]
                c = code[q]
                q += 1
                if c == 0:
                    p = self.DEFAULT_BOND_PCT if pct is None else pct
                    rec = VouchRecord(vouch_id=_C.uuid4("vouch:"), voucher_did=vr, vouchee_did=ve, session_id=sid,
                                      bonded_sigma_pct=max(0.0, min(1.0, p)), bonded_amount=bonded[q - 1],
                                      expiry=expiry)
                    self._vouches[rec.vouch_id] = rec
                    self._by_session.setdefault(sid, []).append(rec)
                    out[i] = rec
                else:
                    out[i] = self._admit_error(c, vr, ve, sid, sig, pct)
        return out

    def _admit_error(self, code: int, voucher_did, vouchee_did, session_id, sigma, pct) -> VouchingError:
        """The error ``vouch`` raises for a K05 rejection code (message rebuilt on the host)."""
        if code == 1:
            return VouchingError("Cannot vouch for yourself")
        if code == 2:
            return VouchingError(f"Voucher σ ({sigma:.2f}) below minimum ({self.MIN_VOUCHER_SCORE:.2f})")
        if code == 3:
            return VouchingError(f"Circular vouching detected: {vouchee_did} already vouches for "
                                 f"{voucher_did} in session {session_id}")
        p = max(0.0, min(1.0, self.DEFAULT_BOND_PCT if pct is None else pct))
        return VouchingError(
            f"Voucher {voucher_did} would exceed max exposure ({self.max_exposure:.0%} of σ). "
            f"Current: {self.get_total_exposure(voucher_did, session_id):.3f}, requested: {sigma * p:.3f}, "
            f"limit: {sigma * self.max_exposure:.3f}"
        )

    def compute_sigma_eff(
        self,
        vouchee_did: str,
        session_id: str,
        vouchee_sigma: float,
        risk_weight: float,
    ) -> float:
        contrib = 0.0
        for v in self._live(session_id):
            if v.vouchee_did == vouchee_did:
                contrib += v.bonded_amount
        return min(vouchee_sigma + risk_weight * contrib, 1.0)

    def records(self, session_id: Optional[str] = None) -> list[VouchRecord]:
        """All vouch records (active or not), optionally of one session."""
        if session_id is not None:
            return list(self._session_records(session_id))
        return list(self._vouches.values())

    def get_vouchers_for(self, agent_did: str, session_id: str) -> list[VouchRecord]:
        return self._active_vouches_for(agent_did, session_id)

    def get_total_exposure(self, voucher_did: str, session_id: str) -> float:
        return sum(v.bonded_amount for v in self._live(session_id) if v.voucher_did == voucher_did)

    def release_bond(self, vouch_id: str) -> None:
        rec = self._vouches.get(vouch_id)
        if rec is None:
            raise VouchingError(f"Vouch {vouch_id} not found")
        rec.is_active = False
        rec.released_at = _now()

    def release_session_bonds(self, session_id: str) -> int:
        n = 0
        t = None
        for v in self._session_records(session_id):
            if v.is_active and v.session_id == session_id:
                if t is None:
                    t = _now()
                v.is_active = False
                v.released_at = t
                n += 1
        return n

    # -- cycle detection --------------------------------------------------------
    def _creates_cycle(self, voucher_did: str, vouchee_did: str, session_id: str) -> bool:
        """Would voucher→vouchee close a cycle among live vouches of the session?"""
        out: dict[str, list[str]] = {}
        for v in self._live(session_id):
            out.setdefault(v.voucher_did, []).append(v.vouchee_did)
        if voucher_did in out.get(vouchee_did, ()):
            return True
        if _cfg.parity_mode():
            return self._creates_cycle_reference_bfs(voucher_did, vouchee_did, out)
        seen = {vouchee_did}
        q = deque([vouchee_did])
        while q:
            cur = q.popleft()
            for nxt in out.get(cur, ()):
                if nxt == voucher_did:
                    return True
                if nxt not in seen:
                    seen.add(nxt)
                    q.append(nxt)
        return False

    @staticmethod
    def _creates_cycle_reference_bfs(voucher_did: str, vouchee_did: str, out: dict[str, list[str]]) -> bool:
        # Reference algorithm (vouching.py:214-229): a node enqueued twice before
        # being visited is reported as a cycle (diamond false positive).
        visited = {voucher_did}
        q = deque([vouchee_did])
        while q:
            cur = q.popleft()
            if cur in visited:
                return True
            visited.add(cur)
            for nxt in out.get(cur, ()):
                if nxt not in visited:
                    q.append(nxt)
        return False
