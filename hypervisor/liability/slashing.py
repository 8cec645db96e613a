"""Collateral slashing: blacklist the violator, clip everyone who vouched for it.

Parity target: reference ``liability/slashing.py:17-147``.

For a slash of ``vouchee`` in ``session`` with risk weight ω:

1. ``agent_scores[vouchee] = 0`` (the caller-owned dict is mutated in place);
2. for each live voucher of the vouchee, in vouch-creation order:
   ``σ ← max(σ·(1−ω), 0.05)`` (an unknown voucher starts from 0.0), record a
   :class:`VoucherClip`, release that bond;
3. append the result to history;
4. below ``MAX_CASCADE_DEPTH`` (2), every clipped voucher left at
   ``σ < SIGMA_FLOOR + 0.01`` that itself has live vouchers is slashed in turn
   (depth + 1, same ω, reason prefixed "Cascade from …").

Batched twin: kernel K06 (``slash_cascade``) in ``csrc/hip/liability_kernels.hip``
runs the same frontier expansion for thousands of sessions at once; duplicate
vouches compound as (1−ω)^k exactly as the sequential loop does.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now


@dataclass
class VoucherClip:
    voucher_did: str
    sigma_before: float
    sigma_after: float
    risk_weight: float
    vouch_id: str


@dataclass
class SlashResult:
    slash_id: str
    vouchee_did: str
    vouchee_sigma_before: float
    vouchee_sigma_after: float
    voucher_clips: list[VoucherClip]
    reason: str
    session_id: str
    timestamp: datetime = field(default_factory=_now)
    cascade_depth: int = 0


def clip_sigma(sigma: float, risk_weight: float, floor: float = 0.05) -> float:
    """σ after one collateral clip (shared formula with the K06 kernel)."""
    return max(sigma * (1.0 - risk_weight), floor)


class SlashingEngine:
    MAX_CASCADE_DEPTH = 2
    SIGMA_FLOOR = 0.05

    def __init__(self, vouching_engine: object) -> None:
        self._vouching = vouching_engine
        self._slash_history: list[SlashResult] = []

    def slash(
        self,
        vouchee_did: str,
        session_id: str,
        vouchee_sigma: float,
        risk_weight: float,
        reason: str,
        agent_scores: dict[str, float],
        cascade_depth: int = 0,
    ) -> SlashResult:
        agent_scores[vouchee_did] = 0.0
        clips: list[VoucherClip] = []
        for vr in self._vouching.get_vouchers_for(vouchee_did, session_id):
            before = agent_scores.get(vr.voucher_did, 0.0)
            after = clip_sigma(before, risk_weight, self.SIGMA_FLOOR)
            agent_scores[vr.voucher_did] = after
            clips.append(VoucherClip(vr.voucher_did, before, after, risk_weight, vr.vouch_id))
            self._vouching.release_bond(vr.vouch_id)

        result = SlashResult(
            slash_id=_C.uuid4("slash:"),
            vouchee_did=vouchee_did,
            vouchee_sigma_before=vouchee_sigma,
            vouchee_sigma_after=0.0,
            voucher_clips=clips,
            reason=reason,
            session_id=session_id,
            cascade_depth=cascade_depth,
        )
        self._slash_history.append(result)

        if cascade_depth < self.MAX_CASCADE_DEPTH:
            wiped = self.SIGMA_FLOOR + 0.01
            for c in clips:
                if c.sigma_after < wiped and self._vouching.get_vouchers_for(c.voucher_did, session_id):
                    self.slash(
                        vouchee_did=c.voucher_did,
                        session_id=session_id,
                        vouchee_sigma=c.sigma_after,
                        risk_weight=risk_weight,
                        reason=f"Cascade from {vouchee_did}: {reason}",
                        agent_scores=agent_scores,
                        cascade_depth=cascade_depth + 1,
                    )
        return result

    @property
    def history(self) -> list[SlashResult]:
        return list(self._slash_history)
