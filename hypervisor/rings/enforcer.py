"""Ring gate: may an agent in ring R perform an action at σ_eff?

Parity target: reference ``rings/enforcer.py:15-137``.  Rules, first match wins:

1. required ring 0 without an SRE witness → deny (``requires_sre_witness``)
2. required ring 1 with σ_eff < 0.95 → deny; without consensus → deny
   (``requires_consensus``)
3. required ring 2 with σ_eff < 0.60 → deny
4. agent ring numerically above the required ring → deny ("insufficient")
5. allow ("Access granted")

Note the thresholds here are *non-strict* ``<`` whereas ring derivation
(:meth:`ExecutionRing.from_sigma_eff`) is strict ``>`` — both preserved
(SURVEY Appendix A, Q12).  The batched form of this predicate is kernel K02
(``ring_check`` in ``csrc/include/ahv/semantics.h``), which returns a reason code
that :func:`reason_text` turns back into the exact strings below.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from hypervisor.models import ActionDescriptor, ExecutionRing

# Reason codes shared with the device kernel (semantics.h: RingReason).
REASON_GRANTED = 0
REASON_NEEDS_WITNESS = 1
REASON_RING1_SIGMA = 2
REASON_NEEDS_CONSENSUS = 3
REASON_RING2_SIGMA = 4
REASON_INSUFFICIENT = 5


@dataclass
class RingCheckResult:
    allowed: bool
    required_ring: ExecutionRing
    agent_ring: ExecutionRing
    sigma_eff: float
    reason: str
    requires_consensus: bool = False
    requires_sre_witness: bool = False


class RingEnforcer:
    RING_1_THRESHOLD = 0.95
    RING_2_THRESHOLD = 0.60

    def __init__(self) -> None:
        self._sre_witness_callback: Optional[object] = None

    def reason_text(self, code: int, agent_ring: int, required: int, sigma_eff: float) -> str:
        if code == REASON_GRANTED:
            return "Access granted"
        if code == REASON_NEEDS_WITNESS:
            return "Ring 0 actions require SRE Witness co-sign"
        if code == REASON_RING1_SIGMA:
            return f"Ring 1 requires σ_eff > {self.RING_1_THRESHOLD}, got {sigma_eff:.3f}"
        if code == REASON_NEEDS_CONSENSUS:
            return "Ring 1 non-reversible actions require consensus"
        if code == REASON_RING2_SIGMA:
            return f"Ring 2 requires σ_eff > {self.RING_2_THRESHOLD}, got {sigma_eff:.3f}"
        return f"Agent ring {agent_ring} insufficient for required ring {required}"

    def check_code(
        self,
        agent_ring: int,
        required: int,
        sigma_eff: float,
        has_consensus: bool = False,
        has_sre_witness: bool = False,
    ) -> int:
        """Scalar twin of the device predicate; returns a reason code."""
        if required == 0 and not has_sre_witness:
            return REASON_NEEDS_WITNESS
        if required == 1:
            if sigma_eff < self.RING_1_THRESHOLD:
                return REASON_RING1_SIGMA
            if not has_consensus:
                return REASON_NEEDS_CONSENSUS
        if required == 2 and sigma_eff < self.RING_2_THRESHOLD:
            return REASON_RING2_SIGMA
        if agent_ring > required:
            return REASON_INSUFFICIENT
        return REASON_GRANTED

    def check(
        self,
        agent_ring: ExecutionRing,
        action: ActionDescriptor,
        sigma_eff: float,
        has_consensus: bool = False,
        has_sre_witness: bool = False,
    ) -> RingCheckResult:
        required = action.required_ring
        code = self.check_code(
            int(agent_ring.value), int(required.value), sigma_eff, has_consensus, has_sre_witness
        )
        return RingCheckResult(
            allowed=code == REASON_GRANTED,
            required_ring=required,
            agent_ring=agent_ring,
            sigma_eff=sigma_eff,
            reason=self.reason_text(code, agent_ring.value, required.value, sigma_eff),
            requires_consensus=code == REASON_NEEDS_CONSENSUS,
            requires_sre_witness=code == REASON_NEEDS_WITNESS,
        )

    def check_batch(
        self,
        agent_rings,
        actions,
        sigma_effs,
        has_consensus=None,
        has_sre_witness=None,
        device="cpu",
    ) -> list[RingCheckResult]:
        """:meth:`check` for many (agent ring, action, σ_eff) triples with one
        K02 launch on ``device`` (``cpu`` runs the kernel's host twin)."""
        import torch

        from agent_hypervisor_amd.ops import rings as RG

        n = len(actions)
        flags = [RG.action_flags(a.is_admin, a.is_read_only, a.required_ring is ExecutionRing.RING_1_PRIVILEGED)
                 for a in actions]
        u8 = torch.uint8
        cons = [bool(x) for x in (has_consensus or [False] * n)]
        wit = [bool(x) for x in (has_sre_witness or [False] * n)]
        packed = torch.tensor([[int(ExecutionRing(r).value) for r in agent_rings], flags, cons, wit], dtype=u8)
        packed = packed.to(device)
        sig = torch.tensor([float(s) for s in sigma_effs], dtype=torch.float64).to(device)
        req, reason = RG.ring_check(packed[0], packed[1], sig, packed[2], packed[3])
        host = torch.stack([req, reason]).cpu().tolist()
        out = []
        for i in range(n):
            ar, required, code = ExecutionRing(agent_rings[i]), ExecutionRing(host[0][i]), host[1][i]
            out.append(RingCheckResult(
                allowed=code == REASON_GRANTED,
                required_ring=required,
                agent_ring=ar,
                sigma_eff=float(sigma_effs[i]),
                reason=self.reason_text(code, ar.value, required.value, float(sigma_effs[i])),
                requires_consensus=code == REASON_NEEDS_CONSENSUS,
                requires_sre_witness=code == REASON_NEEDS_WITNESS,
            ))
        return out

    def compute_ring(self, sigma_eff: float, has_consensus: bool = False) -> ExecutionRing:
        return ExecutionRing.from_sigma_eff(sigma_eff, has_consensus)

    def should_demote(self, current_ring: ExecutionRing, sigma_eff: float) -> bool:
        return self.compute_ring(sigma_eff).value > current_ring.value
